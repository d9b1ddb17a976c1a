#!/bin/bash
# round 6 call D: compact doorbell install (Shoup tables expanded on device)
# slots counted as callers; churn phases; the record-layer consumer's bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06d
mkdir -p $O
cd $R
bash scripts/gpu_suite.sh r06d/suite; rc=$?
tail -3 $O/suite_tests.log; grep -E 'FAILED|ERROR' $O/suite_tests.log | head -20
[ $rc -ne 0 ] && exit $rc
OUT=$O/evp.jsonl; : > $OUT
for t in 1 16 64; do
  timeout -k 10 60 oracle/_ref/cpubench talos_amd/libtlsgpu.so aes-128-gcm init 1400 $t $t 2 \
    | sed "s/^{/{\"lib\": \"libtlsgpu (default)\", /" >> $OUT || exit 1
done
for t in 1 16; do
  TLSGPU_EVP_ASYNC_SCRUB=0 timeout -k 10 60 oracle/_ref/cpubench talos_amd/libtlsgpu.so aes-128-gcm init 1400 $t $t 2 \
    | sed "s/^{/{\"lib\": \"libtlsgpu (synchronous cleanup scrub)\", /" >> $OUT || exit 1
  timeout -k 10 60 oracle/_ref/cpubench talos_amd/libtlsgpu.so aes-128-gcm seal 1400 $((t * 8)) $t 2 \
    | sed "s/^{/{\"lib\": \"libtlsgpu (default)\", /" >> $OUT || exit 1
done
TLSGPU_EVP_DOORBELL_TRACE=1 timeout -k 10 60 oracle/_ref/cpubench talos_amd/libtlsgpu.so aes-128-gcm init 1400 1 1 2 \
  > $O/init1_trace.json 2> $O/init1_trace.err || exit 1
cat $OUT | cut -c1-330
cat $O/init1_trace.json; tail -20 $O/init1_trace.err
for n in 1024; do
  timeout -k 10 300 tests/ssl_batch/_build/batch_server -p tests/golden/server.pem -c ECDHE-RSA-AES128-GCM-SHA256 \
    -n $n -b -r 8 -l 16384 > $O/ssl_batch_n$n.json 2> $O/ssl_batch_n$n.err || exit 1
  cat $O/ssl_batch_n$n.json
done
