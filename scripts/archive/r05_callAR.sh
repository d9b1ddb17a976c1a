#!/bin/bash
# round 5 call AR: NARROW by buffer-relative 32-bit offsets (every fused batch
# with buffers <= 4 GiB, both directions) — parity, A/B on C, warm PMC of C
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ar
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_batch_digests.py tests/test_gpu_parity.py tests/test_wire_reference.py tests/test_seal_wire.py tests/test_wire.py -m gpu \
  > $O/tests.log 2>&1 || exit $?
bash scripts/env_ab.sh r05ar/abC 3 "TLSGPU_CC_NARROW=0|-" --config C > $O/abC.txt 2>&1 || exit $?
bash scripts/pmc.sh r05ar/pmcC --config C > $O/pmcC.txt 2>&1 || exit $?
