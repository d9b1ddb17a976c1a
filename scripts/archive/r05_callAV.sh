#!/bin/bash
# round 5 call AV: ChaCha keys from s_load for one-session waves (UKEY) —
# parity, then same-box A/B against TLSGPU_CC_UKEY=0 on C
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05av
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_batch_digests.py tests/test_gpu_parity.py tests/test_wire_reference.py tests/test_seal_wire.py tests/test_wire.py -m gpu \
  > $O/tests.log 2>&1 || exit $?
bash scripts/env_ab.sh r05av/abC 4 "TLSGPU_CC_UKEY=0|-" --config C > $O/abC.txt 2>&1 || exit $?
