#!/bin/bash
# round 5 call E: connection churn with the host-built session image vs the
# device install kernel (TLSGPU_EVP_DEVICE_INSTALL=1), launched path and
# doorbell; then the whole GPU suite with the doorbell on for every test
# (the default-on candidate) and the crash reporter armed.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05e
mkdir -p $O
cd $R
OUT=$O/churn.jsonl; : > $OUT
for t in 1 16 64; do
  timeout -k 10 60 oracle/_ref/cpubench oracle/_ref/libref.so aes-128-gcm init 1400 $t $t 2 \
    | sed "s/^{/{\"lib\": \"reference\", /" >> $OUT || exit 1
  for inst in host device; do
    for db in 0 64; do
      di=0; [ $inst = device ] && di=1
      TLSGPU_EVP_DEVICE_INSTALL=$di TLSGPU_EVP_DOORBELL=$db timeout -k 10 60 oracle/_ref/cpubench \
        talos_amd/libtlsgpu.so aes-128-gcm init 1400 $t $t 2 \
        | sed "s/^{/{\"lib\": \"libtlsgpu install=$inst doorbell=$db\", /" >> $OUT || exit 1
    done
  done
done
TLSGPU_EVP_DOORBELL=64 TLSGPU_CRASH_TRACE=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -v \
  --timeout 200 --timeout-method thread > $O/suite_doorbell64.log 2>&1 || exit $?
