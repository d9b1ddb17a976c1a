#!/bin/bash
# round 6 call G: batched scrub sweeps (try_lock); suite; churn with the
# asynchronous vs synchronous cleanup scrub at 1 / 4 / 16 / 64 threads, twice
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06g
mkdir -p $O
cd $R
bash scripts/gpu_suite.sh r06g/suite; rc=$?
tail -3 $O/suite_tests.log; grep -E 'FAILED|ERROR' $O/suite_tests.log | head -20
[ $rc -ne 0 ] && exit $rc
OUT=$O/evp.jsonl; : > $OUT
for rep in 1 2; do
  for t in 1 4 16 64; do
    for a in 1 0; do
      TLSGPU_EVP_ASYNC_SCRUB=$a timeout -k 10 60 oracle/_ref/cpubench talos_amd/libtlsgpu.so aes-128-gcm init 1400 $t $t 2 \
        | sed "s/^{/{\"lib\": \"libtlsgpu async_scrub=$a\", \"rep\": $rep, /" >> $OUT || exit 1
    done
  done
done
cut -c1-300 $OUT
