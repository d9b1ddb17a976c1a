#!/bin/bash
# round 6 call T: the consumer after folding its two pipelines into shared
# helpers — ssl_batch tests, then the read / write benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06t
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_ssl_batch.py -x -v --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash scripts/archive/r06_callQ.sh r06t
