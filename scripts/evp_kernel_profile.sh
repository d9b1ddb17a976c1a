#!/bin/bash
# Kernel durations behind the EVP per-call path and the queue
# (rocprofv3 kernel trace of oracle/_ref/cpubench over libtlsgpu.so).
# usage: scripts/evp_kernel_profile.sh TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/$1
mkdir -p $O
B=$R/oracle/_ref/cpubench
LIB=$R/talos_amd/libtlsgpu.so
for len in 1400 16384; do
  timeout -k 10 90 rocprofv3 --kernel-trace --stats -d $O/percall_$len -o run -- $B $LIB aes-128-gcm seal $len 64 1 1 || exit 1
  TLSGPU_EVP_BATCH_US=50 TLSGPU_EVP_POOL=256 timeout -k 10 90 rocprofv3 --kernel-trace --stats -d $O/queue16_$len -o run -- $B $LIB aes-128-gcm seal $len 128 16 1 || exit 1
done
find $O -name "*kernel_stats.csv" | sort | while read f; do echo "== $f"; cat "$f"; done
