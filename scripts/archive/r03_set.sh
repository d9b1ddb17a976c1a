#!/bin/bash
# Round-3 measurement set (GPU box): bench lines, kernel stats, PMC passes
# with their own bench lines, phase timing of B and D, install-kernel timing.
# usage: scripts/r03_set.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
bash scripts/measure_set.sh $TAG --no-pmc || exit $?
for c in B D; do
  TLSGPU_PHASE_STATS=1 timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --steps 10 \
    > $O/phase_$c.json 2> $O/phase_$c.err || exit 1
  echo "phase $c: $(grep -c phase $O/phase_$c.err) lines"
done
bash scripts/kstats.sh $TAG/kstats || exit $?
for c in B D C; do
  bash scripts/pmc.sh $TAG/pmc$c --config $c || exit $?
done
exit 0
