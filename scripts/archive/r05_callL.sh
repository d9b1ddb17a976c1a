#!/bin/bash
# round 5 call L: fused ChaCha batches (bounds in the staged kernel) — parity,
# then a same-box A/B of config C with TLSGPU_FUSED=0 vs the default.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05l
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_batch_digests.py tests/test_wire.py tests/test_wire_reference.py tests/test_host_pipeline.py \
  > $O/tests.log 2>&1 || exit $?
bash scripts/env_ab.sh r05l/abC 3 "TLSGPU_FUSED=0|-" --config C > $O/abC.txt 2>&1 || exit $?
