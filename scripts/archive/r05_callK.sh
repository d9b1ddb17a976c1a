#!/bin/bash
# round 5 call K: the round's measurement set (bench lines, PMC passes for
# B / C / D) and kernel-trace stats of the same configs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash scripts/measure_set.sh r05k > gpurun_out/r05k_measure.txt 2>&1 || exit $?
bash scripts/kstats.sh r05k/kstats > gpurun_out/r05k_kstats.txt 2>&1 || exit $?
