#!/bin/bash
# round 5 call Z (re-entry): the round's final measurement set after the ChaCha
# step-order change: bench lines, PMC for B / C / D, kernel-trace stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash scripts/measure_set.sh r05z > gpurun_out/r05z_measure.txt 2>&1 || exit $?
bash scripts/kstats.sh r05z/kstats > gpurun_out/r05z_kstats.txt 2>&1 || exit $?
