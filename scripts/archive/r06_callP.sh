#!/bin/bash
# round 6 call P: the record-layer consumer's batched write side
# (tlsgpu_ssl_batch_write) against the reference's client SSL_read, all suites
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06p
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_ssl_batch.py -x -v --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 120 tests/ssl_batch/_build/batch_server -p tests/golden/server.pem -c ECDHE-RSA-AES256-GCM-SHA384 \
  -n 24 -t 5 > $O/write_aes256.json 2> $O/write_aes256.err || exit $?
cat $O/write_aes256.json
