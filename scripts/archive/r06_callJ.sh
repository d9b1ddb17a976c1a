#!/bin/bash
# round 6 call J: rocprofv3 kernel stats of B / C / D and the PMC passes of
# config B on the final kernels (the bench's settle + warm-up precede them)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash scripts/kstats.sh r06j/kstats || exit $?
bash scripts/pmc.sh r06j/pmcB --config B || exit $?
