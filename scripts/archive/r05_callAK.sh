#!/bin/bash
# round 5 call AK: PMC passes for B / C / D with the warm-start bench (warm-up
# 30, 10 timed steps; the summary keeps the timed launches)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for c in B C D; do
  bash scripts/pmc.sh r05ak/pmc$c --config $c > gpurun_out/r05ak_pmc$c.txt 2>&1 || exit $?
done
