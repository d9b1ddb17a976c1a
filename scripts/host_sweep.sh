#!/bin/bash
# tlsgpu_open_host chunk / stream sweep on config B (bench.py --mode host).
# usage: scripts/host_sweep.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
: > $O/host_sweep.jsonl
for cfg in "2 32 65536" "2 16 65536" "2 64 65536" "3 32 65536" "4 32 65536" "2 128 65536" "2 32 131072"; do
  set -- $cfg
  timeout -k 10 180 python3 $R/bench.py --mode host --no-cpu-baseline --steps 8 --warmup 2 \
    --host-streams $1 --host-chunk-mib $2 --records $3 | tail -1 >> $O/host_sweep.jsonl || exit 1
done
cat $O/host_sweep.jsonl
