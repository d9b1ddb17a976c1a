#!/bin/bash
# round 6 call Q: the record-layer consumer's read and write benches
# (1,024 connections x 8 x 16 KiB), three runs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r06q}
mkdir -p $O
cd $R
for k in 1 2 3; do
  timeout -k 10 300 tests/ssl_batch/_build/batch_server -p tests/golden/server.pem -c ECDHE-RSA-AES128-GCM-SHA256 \
    -n 1024 -b -r 8 -l 16384 > $O/bench_$k.json 2> $O/bench_$k.err || { cat $O/bench_$k.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/bench_$k.json').read()); print(d['ok'], d['bench']['batch_GiBps'], d['bench']['ssl_read_cpu1_GiBps'], d['write_bench'])"
done
