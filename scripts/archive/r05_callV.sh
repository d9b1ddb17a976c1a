#!/bin/bash
# round 5 call V (re-entry): the whole GPU suite and smoke on the current tree,
# then the default bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05v
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/suite.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
