#!/bin/bash
# Round-4 call K: kernel-trace stats and PMC passes for configs B, C, D.
# usage: scripts/r04_callK.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04p}
cd $R
bash scripts/kstats.sh $TAG/kstats || exit $?
for c in B C D; do
  bash scripts/pmc.sh $TAG/pmc$c --config $c || exit $?
done
exit 0
