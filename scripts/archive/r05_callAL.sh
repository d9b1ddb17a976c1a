#!/bin/bash
# round 5 call AL: ChaCha tags through dword accesses — parity, then same-box
# A/B on C and wire C (warm-start bench)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05al
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_batch_digests.py tests/test_gpu_parity.py tests/test_wire_reference.py tests/test_seal_wire.py -m gpu \
  > $O/tests.log 2>&1 || exit $?
bash scripts/ab_bench.sh r05al/abC 3 "_variants/lib_base.so _variants/lib_tag16.so" --config C > $O/abC.txt 2>&1 || exit $?
bash scripts/ab_bench.sh r05al/abW 2 "_variants/lib_base.so _variants/lib_tag16.so" --config C --mode wire > $O/abW.txt 2>&1 || exit $?
