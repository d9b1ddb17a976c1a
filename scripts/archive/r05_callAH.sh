#!/bin/bash
# round 5 call AH: config B / C / D step time by warm-up length and timed steps
# (the warm-up now follows the first step's verification directly)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ah
mkdir -p $O
cd $R
for args in "--warmup 3" "--warmup 10" "--warmup 30" "--warmup 60" "--warmup 30 --steps 80" "--warmup 100 --steps 80" "--warmup 30 --config C" "--warmup 30 --config D" "--warmup 60 --config D"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline $args > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  echo "[$args] $(python3 -c "import json; d=json.loads(open('$O/b.json').read().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done
