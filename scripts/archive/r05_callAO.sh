#!/bin/bash
# round 5 call AO: final check of the tree — whole GPU suite, smoke, the default
# bench lines B / C / D (warm start), warm PMC of C's default kernel
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ao
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/suite.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
for c in B C D; do
  timeout -k 10 300 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || exit $?
done
bash scripts/pmc.sh r05ao/pmcC --config C > $O/pmcC.txt 2>&1 || exit $?
