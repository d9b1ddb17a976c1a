#!/bin/bash
# Round-4 call P: raw-job / doorbell parity after the E_K(J0) change, the
# per-call trace at 1,400 B and 16 KiB, and bench B (split path unchanged).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04u}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_evp_doorbell.py tests/test_gpu_parity.py tests/test_evp_queue.py -x -v \
  --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { echo "tests rc=$?"; grep -E "FAILED|Error" $O/tests.log | head; tail -5 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
B="$R/oracle/_ref/cpubench $R/talos_amd/libtlsgpu.so"
for spec in "aes-128-gcm seal 1400 1 1" "aes-128-gcm seal 16384 1 1" "aes-256-gcm seal 16384 1 1"; do
  set -- $spec
  TLSGPU_EVP_DOORBELL_TRACE=1 timeout -k 10 60 $B $1 $2 $3 $4 $5 2 >> $O/trace.jsonl 2>> $O/trace.err || exit $?
  echo "trace $spec: $(tail -2 $O/trace.err | tr '\n' ' ' | cut -c1-700)"
done
for spec in "aes-128-gcm seal 16384 8 1" "aes-128-gcm seal 16384 128 16"; do
  set -- $spec
  TLSGPU_EVP_DOORBELL=0 timeout -k 10 60 $B $1 $2 $3 $4 $5 2 | sed 's/^/launched: /'
done
exit 0
