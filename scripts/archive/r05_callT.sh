#!/bin/bash
# round 5 call T: the pack's layout and segmented-XOR scans on DPP instead of
# __shfl_up — parity (in-tree build), then same-box A/B on D.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05t
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_batch_digests.py > $O/tests.log 2>&1 || exit $?
bash scripts/ab_bench.sh r05t/abD 4 "_variants/lib_shfl.so _variants/lib_dpp.so" --config D > $O/abD.txt 2>&1 || exit $?
