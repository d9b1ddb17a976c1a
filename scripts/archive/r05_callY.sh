#!/bin/bash
# round 5 call Y: whole GPU suite with the LATE_STORES ChaCha default and the
# randomized differential sweep.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05y
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/suite.log 2>&1 || exit $?
