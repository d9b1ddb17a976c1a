#!/bin/bash
# round 5 call AZ: the final measurement set of the final tree (bench lines
# of every config with the warm-start bench, warm PMC for B / C / D)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash scripts/measure_set.sh r05az > gpurun_out/r05az_measure.txt 2>&1 || exit $?
