#!/bin/bash
# round 5 call AG: config B by timed steps, with the warm-up right before the
# timed region (no verification gap), then C and D once
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ag
mkdir -p $O
cd $R
for args in "--steps 10" "--steps 20" "--steps 80" "--steps 20 --warmup 10" "" "--config C" "--config D" "--steps 80 --config C" "--steps 80 --config D"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline $args > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  echo "[$args] $(python3 -c "import json; d=json.loads(open('$O/b.json').read().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done
