#!/bin/bash
# Round-4 call G: doorbell parity, job-phase trace (both waves), per-call
# bench.  usage: scripts/r04_callG.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04m}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_evp_doorbell.py tests/test_evp_churn.py tests/test_gpu_parity.py -x -v \
  --timeout 120 --timeout-method thread -m gpu -k "doorbell or churn or split_jobs or chacha_wave or aeadtests" \
  > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
B="$R/oracle/_ref/cpubench $R/talos_amd/libtlsgpu.so"
for spec in "aes-128-gcm seal 1400 1 1" "aes-128-gcm seal 1400 8 1" "aes-128-gcm open 1400 1 1" \
            "aes-256-gcm seal 1400 1 1" "chacha20-poly1305 seal 1400 1 1"; do
  set -- $spec
  TLSGPU_EVP_DOORBELL=16 TLSGPU_EVP_DOORBELL_TRACE=1 timeout -k 10 60 $B $1 $2 $3 $4 $5 2 \
    >> $O/trace.jsonl 2>> $O/trace.err || exit $?
  echo "trace $spec: $(tail -2 $O/trace.err | tr '\n' ' ')"
done
timeout -k 10 420 scripts/evp_doorbell_bench.sh "$O/doorbell_bench.jsonl" > $O/doorbell_bench.log 2>&1 || exit $?
echo "doorbell bench done"
exit 0
