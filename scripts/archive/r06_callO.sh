#!/bin/bash
# round 6 call O: the pipelined record-layer consumer (integration/ssl_batch.c:
# two wire slots, the GPU open of group k on a worker thread beside the
# delivery of k-1 and the gather of k+1) — its tests, then the 1,024-connection
# bench three times
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06o
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_ssl_batch.py -x -v --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for k in 1 2 3; do
  timeout -k 10 300 tests/ssl_batch/_build/batch_server -p tests/golden/server.pem -c ECDHE-RSA-AES128-GCM-SHA256 \
    -n 1024 -b -r 8 -l 16384 > $O/bench_$k.json 2> $O/bench_$k.err || exit $?
  cut -c1-600 $O/bench_$k.json
done
