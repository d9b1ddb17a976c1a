#!/bin/bash
# Round-4 measurement call B: the bench set (measure_set.sh without PMC:
# B, B at S = 1 / 65,536 / interleaved, C, D, host, PCIe, wire, group split)
# and the kernel-trace stats.  usage: scripts/r04_callB.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04i}
cd $R
bash scripts/measure_set.sh $TAG --no-pmc || exit $?
bash scripts/kstats.sh $TAG/kstats || exit $?
exit 0
