#!/bin/bash
# round 5 call S: an odd full 64-block step through the pipelined one-step
# loop (TG_XN_ODD_STEP) — parity of that build, then same-box A/B on D and B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05s
mkdir -p $O
cd $R
TLSGPU_LIBRARY=$R/_variants/lib_odd.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 \
  --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_batch_digests.py > $O/tests_odd.log 2>&1 || exit $?
bash scripts/ab_bench.sh r05s/abD 4 "_variants/lib_base.so _variants/lib_odd.so" --config D > $O/abD.txt 2>&1 || exit $?
bash scripts/ab_bench.sh r05s/abB 2 "_variants/lib_base.so _variants/lib_odd.so" --config B > $O/abB.txt 2>&1 || exit $?
