#!/bin/bash
# round 6 call B: GPU suite on the staging / scrub-ring / claim changes, then
# per-call and connection-churn rates with the phases of one connection
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06b
mkdir -p $O
cd $R
bash scripts/gpu_suite.sh r06b/suite; rc=$?
tail -3 $O/suite_tests.log; grep -E 'FAILED|ERROR' $O/suite_tests.log | head -20
[ $rc -ne 0 ] && exit $rc
OUT=$O/evp.jsonl; : > $OUT
for t in 1 16 64; do
  timeout -k 10 60 oracle/_ref/cpubench talos_amd/libtlsgpu.so aes-128-gcm seal 1400 $((t * 8)) $t 2 \
    | sed "s/^{/{\"lib\": \"libtlsgpu (default)\", /" >> $OUT || exit 1
  timeout -k 10 60 oracle/_ref/cpubench talos_amd/libtlsgpu.so aes-128-gcm init 1400 $t $t 2 \
    | sed "s/^{/{\"lib\": \"libtlsgpu (default)\", /" >> $OUT || exit 1
  timeout -k 10 60 oracle/_ref/cpubench oracle/_ref/libref.so aes-128-gcm init 1400 $t $t 2 \
    | sed "s/^{/{\"lib\": \"reference\", /" >> $OUT || exit 1
done
for t in 1 16; do
  TLSGPU_EVP_ASYNC_SCRUB=0 timeout -k 10 60 oracle/_ref/cpubench talos_amd/libtlsgpu.so aes-128-gcm init 1400 $t $t 2 \
    | sed "s/^{/{\"lib\": \"libtlsgpu (synchronous cleanup scrub)\", /" >> $OUT || exit 1
done
TLSGPU_EVP_DOORBELL_TRACE=1 timeout -k 10 60 oracle/_ref/cpubench talos_amd/libtlsgpu.so aes-128-gcm init 1400 1 1 2 \
  > $O/init1_trace.json 2> $O/init1_trace.err || exit 1
cat $OUT | cut -c1-330
cat $O/init1_trace.json; tail -20 $O/init1_trace.err
