#!/bin/bash
# EVP drop-in throughput with real pthreads (no GIL): oracle/_ref/cpubench
# dlopen()s a library exporting the EVP_AEAD ABI and calls EVP_AEAD_CTX_seal /
# _open from T threads over 64 contexts.  Run against libtlsgpu.so per call and
# with the coalescing queue (TLSGPU_EVP_BATCH_US), and against the reference
# (oracle/_ref/libref.so) on the same thread counts.
# usage: scripts/evp_queue_bench.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
B=$R/oracle/_ref/cpubench
export TLSGPU_EVP_DOORBELL=${TLSGPU_EVP_DOORBELL:-0}  # round-3 semantics: the launched per-call path
LIB=$R/talos_amd/libtlsgpu.so
REF=$R/oracle/_ref/libref.so
out=$O/evp_queue.jsonl
: > $out
: > $O/evp_queue_stats.log
for len in 1400 16384; do
  for t in 1 4 16 64; do
    n=$((t * 8))
    timeout -k 10 60 $B $REF aes-128-gcm seal $len $n $t 2 | sed "s/^{/{\"lib\": \"reference\", /" >> $out || exit 1
    timeout -k 10 60 $B $LIB aes-128-gcm seal $len $n $t 2 | sed "s/^{/{\"lib\": \"libtlsgpu per-call\", /" >> $out || exit 1
    for w in 50 200; do
      TLSGPU_EVP_STATS=1 TLSGPU_EVP_BATCH_US=$w TLSGPU_EVP_POOL=256 timeout -k 10 60 $B $LIB aes-128-gcm seal $len $n $t 2 \
        2>> $O/evp_queue_stats.log | sed "s/^{/{\"lib\": \"libtlsgpu queue ${w}us\", /" >> $out || exit 1
    done
  done
done
cat $out
