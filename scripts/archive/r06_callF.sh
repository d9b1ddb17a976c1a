#!/bin/bash
# round 6 call F: install without scratch, early input staging; harness buffers pre-faulted
# churn and the consumer bench with its phases
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06f
mkdir -p $O
cd $R
bash scripts/gpu_suite.sh r06f/suite; rc=$?
tail -3 $O/suite_tests.log; grep -E 'FAILED|ERROR' $O/suite_tests.log | head -20
[ $rc -ne 0 ] && exit $rc
OUT=$O/evp.jsonl; : > $OUT
for t in 1 16; do
  timeout -k 10 60 oracle/_ref/cpubench talos_amd/libtlsgpu.so aes-128-gcm init 1400 $t $t 2 \
    | sed "s/^{/{\"lib\": \"libtlsgpu (default)\", /" >> $OUT || exit 1
done
TLSGPU_EVP_DOORBELL_TRACE=1 timeout -k 10 60 oracle/_ref/cpubench talos_amd/libtlsgpu.so aes-128-gcm init 1400 1 1 2 \
  > $O/init1_trace.json 2> $O/init1_trace.err || exit 1
cat $OUT | cut -c1-330
cat $O/init1_trace.json; tail -20 $O/init1_trace.err
timeout -k 10 300 tests/ssl_batch/_build/batch_server -p tests/golden/server.pem -c ECDHE-RSA-AES128-GCM-SHA256 \
  -n 1024 -b -r 8 -l 16384 > $O/ssl_batch_n1024.json 2> $O/ssl_batch_n1024.err || exit 1
cat $O/ssl_batch_n1024.json
