#!/bin/bash
# round 5 call AA: workgroups per CU (TLSGPU_WG_PER_CU) for the GCM queue
# kernels — parity at 2 and 4, then same-box A/B on B and D.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05aa
mkdir -p $O
cd $R
for k in 2 4; do
  TLSGPU_WG_PER_CU=$k timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_batch_digests.py tests/test_gpu_parity.py -m gpu -k "batch" \
    > $O/tests_k$k.log 2>&1 || exit $?
done
bash scripts/env_ab.sh r05aa/abB 2 "TLSGPU_WG_PER_CU=1|TLSGPU_WG_PER_CU=2|TLSGPU_WG_PER_CU=3|TLSGPU_WG_PER_CU=4" > $O/abB.txt 2>&1 || exit $?
bash scripts/env_ab.sh r05aa/abD 2 "TLSGPU_WG_PER_CU=1|TLSGPU_WG_PER_CU=2|TLSGPU_WG_PER_CU=3|TLSGPU_WG_PER_CU=4" --config D > $O/abD.txt 2>&1 || exit $?
