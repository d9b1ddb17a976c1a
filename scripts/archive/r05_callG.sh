#!/bin/bash
# round 5 call G: work-balanced ranges for the fused queue kernel — parity
# (fused prologue cases, balanced / unbalanced child runs, full-size digests),
# then a same-box A/B of config D (TLSGPU_BALANCE=0 vs the default) and the
# kernel-trace stats of both.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05g
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py -k "fused" tests/test_gpu_batch_digests.py tests/test_evp_deferred_install.py \
  > $O/tests.log 2>&1 || exit $?
bash scripts/env_ab.sh r05g/abD 4 "TLSGPU_BALANCE=0|-" --config D > $O/abD.txt 2>&1 || exit $?
bash scripts/env_ab.sh r05g/abB 2 "TLSGPU_BALANCE=0|TLSGPU_BALANCE=2" --config B > $O/abB.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
for b in 0 1; do
  TLSGPU_BALANCE=$b timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kD$b -o run -- \
    python3 $R/bench.py --config D --steps 10 --warmup 2 --no-cpu-baseline > $O/kD$b.log 2>&1 || exit 1
done
