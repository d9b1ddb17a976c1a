#!/bin/bash
# round 5 call AU: the pack path's Shoup multiply pipelined two reads ahead
# (TG_PACK_SHOUP_PF2) — pack parity with it, then same-box A/B on D
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05au
mkdir -p $O
cd $R
TLSGPU_LIBRARY=$R/_variants/lib_pf2.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_batch_digests.py tests/test_gpu_parity.py -m gpu -k "pack or D or random or fused" > $O/tests.log 2>&1 || exit $?
bash scripts/ab_bench.sh r05au/abD 3 "_variants/lib_base.so _variants/lib_pf2.so" --config D > $O/abD.txt 2>&1 || exit $?
