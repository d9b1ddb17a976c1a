#!/bin/bash
# round 5 call J: run-start critical path of the queue kernel — parity of the
# 4-way run-end scan, D's phase timing, then a same-box A/B of the serial
# scan (round 4), the 4-way scan, and the 4-way scan + vector session loads.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05j
mkdir -p $O
cd $R
export TLSGPU_BALANCE=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_batch_digests.py > $O/tests.log 2>&1 || exit $?
TLSGPU_LIBRARY=$R/_variants/lib_vsl.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 \
  --timeout-method thread tests/test_gpu_batch_digests.py tests/test_evp_doorbell.py > $O/tests_vsl.log 2>&1 || exit $?
TLSGPU_PHASE_STATS=1 timeout -k 10 300 python bench.py --config D --steps 10 --no-cpu-baseline > $O/phaseD.txt 2>&1 || exit 1
bash scripts/ab_bench.sh r05j/abD 3 "_variants/lib_serial.so _variants/lib_new.so _variants/lib_vsl.so" --config D \
  > $O/abD.txt 2>&1 || exit $?
bash scripts/ab_bench.sh r05j/abB 2 "_variants/lib_serial.so _variants/lib_new.so _variants/lib_vsl.so" --config B \
  > $O/abB.txt 2>&1 || exit $?
