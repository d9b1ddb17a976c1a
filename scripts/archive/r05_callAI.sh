#!/bin/bash
# round 5 call AI: final bench lines with the warm-start bench (default
# warm-up 30), smoke first; PMC/kernel stats unchanged from r05z (same kernels).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/r05ai
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05ai/smoke.log 2>&1 || exit $?
bash scripts/measure_set.sh r05ai --no-pmc > gpurun_out/r05ai_measure.txt 2>&1 || exit $?
