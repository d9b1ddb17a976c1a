#!/bin/bash
# round 5 call AB: why two members on one GPU beat one engine — batch size per
# launch vs two concurrent streams (same box, 2 rounds).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ab
mkdir -p $O
cd $R
for k in 1 2; do
  for args in "" "--records 131072" "--records 32768" "--split group --devices 0,0" "--split group --devices 0" "--split group --devices 0,0 --records 32768"; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 $args > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
    echo "$k [$args] $(python3 -c "import json; d=json.loads(open('$O/b.json').read().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('member_device_ms_per_step',''))")"
  done
done
