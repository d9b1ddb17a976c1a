#!/bin/bash
# round 5 call AS: randomized differential soak (300 seeds), kernel-trace stats
# of B / C / D with the warm-start bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05as
mkdir -p $O
cd $R
TLSGPU_FUZZ_SEEDS=300 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -m gpu -k random_differential > $O/soak.log 2>&1 || exit $?
bash scripts/kstats.sh r05as/kstats > $O/kstats.txt 2>&1 || exit $?
