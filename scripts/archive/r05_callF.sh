#!/bin/bash
# round 5 call F: deferred EVP install + doorbell scrub (doorbell on by
# default): the new tests, the whole GPU suite with the default environment,
# connection churn and per-call rates.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05f
mkdir -p $O
cd $R
export TLSGPU_CRASH_TRACE=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_evp_deferred_install.py tests/test_evp_churn.py tests/test_evp_doorbell.py \
  tests/test_evp_shutdown.py > $O/tests_new.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  > $O/suite.log 2>&1 || exit $?
OUT=$O/churn.jsonl; : > $OUT
for t in 1 16 64; do
  for db in 64 0; do
    TLSGPU_EVP_DOORBELL=$db timeout -k 10 60 oracle/_ref/cpubench talos_amd/libtlsgpu.so \
      aes-128-gcm init 1400 $t $t 2 | sed "s/^{/{\"lib\": \"libtlsgpu doorbell=$db\", /" >> $OUT || exit 1
  done
done
for t in 1 16 64; do
  for db in 64 0; do
    TLSGPU_EVP_DOORBELL=$db timeout -k 10 60 oracle/_ref/cpubench talos_amd/libtlsgpu.so \
      aes-128-gcm seal 1400 $((t * 8)) $t 2 | sed "s/^{/{\"lib\": \"libtlsgpu doorbell=$db\", /" >> $O/percall.jsonl || exit 1
  done
done
