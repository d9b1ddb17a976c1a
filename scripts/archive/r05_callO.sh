#!/bin/bash
# round 5 call O: the round-end sequence on the committed tree — smoke(),
# the whole GPU suite, the default bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05o
mkdir -p $O
cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  > $O/suite.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
