#!/bin/bash
# round 5 call D: the new GPU tests (fused prologue, host session image,
# hinted digests, shutdown), then kernel-trace stats of B and D with the
# HEAD-base and the new library (where the fused path's time goes).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05d
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_session_image.py tests/test_evp_churn.py tests/test_evp_shutdown.py \
  "tests/test_gpu_parity.py::test_batch_fused_prologue" "tests/test_gpu_parity.py::test_batch_bounds" \
  "tests/test_gpu_batch_digests.py" > $O/tests.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
for v in base new; do
  for c in B D; do
    TLSGPU_LIBRARY=$R/_variants/lib_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k_${v}_$c -o run -- \
      python3 $R/bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > $O/k_${v}_$c.log 2>&1 || exit 1
  done
done
