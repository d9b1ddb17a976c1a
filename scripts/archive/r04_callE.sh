#!/bin/bash
# Round-4 call E: doorbell GCM job phases (TLSGPU_EVP_DOORBELL_TRACE, gcm_raw.h
# marks) and the config C time split (tools/cc_diag.py, TLSGPU_CC_DIAG bits).
# usage: scripts/r04_callE.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04k}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
B="$R/oracle/_ref/cpubench $R/talos_amd/libtlsgpu.so"
timeout -k 10 300 python -u -m pytest tests/test_evp_doorbell.py tests/test_gpu_parity.py -x -v \
  --timeout 120 --timeout-method thread -m gpu -k "doorbell or split_jobs or chacha_wave or aeadtests" \
  > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
for spec in "aes-128-gcm seal 1400 1 1" "aes-128-gcm seal 1400 8 1" "aes-128-gcm open 1400 1 1" \
            "aes-128-gcm seal 16384 1 1"; do
  set -- $spec
  TLSGPU_EVP_DOORBELL=16 TLSGPU_EVP_DOORBELL_TRACE=1 timeout -k 10 60 $B $1 $2 $3 $4 $5 2 \
    >> $O/trace.jsonl 2>> $O/trace.err || exit $?
  echo "trace $spec: $(tail -2 $O/trace.err | tr '\n' ' ')"
done
if [ -f tools/var/libtlsgpu_as1.so ]; then  # A/B: session reads through global pointers
  for spec in "aes-128-gcm seal 1400 1 1" "aes-128-gcm seal 1400 8 1"; do
    set -- $spec
    TLSGPU_EVP_DOORBELL=16 TLSGPU_EVP_DOORBELL_TRACE=1 timeout -k 10 60 $R/oracle/_ref/cpubench \
      $R/tools/var/libtlsgpu_as1.so $1 $2 $3 $4 $5 2 >> $O/trace_as1.jsonl 2>> $O/trace_as1.err || exit $?
    echo "trace as1 $spec: $(tail -2 $O/trace_as1.err | tr '\n' ' ')"
  done
fi
for d in 0 1 2 3 4 7; do
  TLSGPU_CC_DIAG=$d timeout -k 10 240 python tools/cc_diag.py >> $O/cc_diag.jsonl 2> $O/cc_diag_$d.err || exit $?
  tail -1 $O/cc_diag.jsonl
done
exit 0
