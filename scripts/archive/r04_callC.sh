#!/bin/bash
# Round-4 measurement call C: PMC passes (scripts/pmc.sh) for configs B, C, D.
# usage: scripts/r04_callC.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04i}
cd $R
for c in B C D; do
  bash scripts/pmc.sh $TAG/pmc$c --config $c || exit $?
done
exit 0
