#!/bin/bash
# round 5 call W: ChaCha staged kernel step order (TLSGPU_CC_ORDER 0/1/2):
# parity of the two new orders, then a same-box A/B on config C and wire C.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05w
mkdir -p $O
cd $R
for ord in 1 2; do
  TLSGPU_CC_ORDER=$ord timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_batch_digests.py tests/test_gpu_parity.py tests/test_wire_reference.py -m gpu -k "chacha or C or wire or reference" \
    > $O/tests_ord$ord.log 2>&1 || exit $?
done
bash scripts/env_ab.sh r05w/abC 3 "TLSGPU_CC_ORDER=0|TLSGPU_CC_ORDER=1|TLSGPU_CC_ORDER=2" --config C > $O/abC.txt 2>&1 || exit $?
bash scripts/env_ab.sh r05w/abW 2 "TLSGPU_CC_ORDER=0|TLSGPU_CC_ORDER=1|TLSGPU_CC_ORDER=2" --config C --mode wire > $O/abW.txt 2>&1 || exit $?
