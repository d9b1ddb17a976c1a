#!/bin/bash
# round 6 call S: ssl_batch tests with the split-wire phase (partial records
# kept across two batch reads)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06s
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_ssl_batch.py -x -v --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -12 $O/tests.log
