#!/bin/bash
# Pool-scratch root cause: tools/pool_probe over pool / plain
# memory (see its header for the arguments), then the engine's fresh-batch loop
# with the scratch from the pool (TLSGPU_PRE_POOL=1) and from hipMalloc.
# usage: scripts/pool_probe.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
P=$R/tools/pool_probe
: > $O/pool_probe.jsonl
: > $O/pool_probe_bad.log
for args in "pool 400 1 1 0 0" "plain 400 1 1 0 0" "pool_keep 400 1 1 0 1" "plain 400 1 1 0 1"; do
  echo "== $args" >> $O/pool_probe_bad.log
  timeout -k 10 60 $P $args >> $O/pool_probe.jsonl 2>> $O/pool_probe_bad.log || exit 1
done
cat $O/pool_probe.jsonl
grep -c . $O/pool_probe_bad.log; grep -m 12 'zero words\|==' $O/pool_probe_bad.log | cut -c1-600
ITERS=60 TLSGPU_PRE_POOL=1 timeout -k 10 300 python3 -u $R/scripts/dbg_open3.py > $O/dbg_pool.log 2>&1 || exit 1
echo "engine, pool scratch: $(grep -c 'bad \[\] 0' $O/dbg_pool.log) clean of $(grep -c '^iter' $O/dbg_pool.log)"
