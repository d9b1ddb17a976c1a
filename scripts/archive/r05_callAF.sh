#!/bin/bash
# round 5 call AF: config B step time by steps timed and records per launch
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05af
mkdir -p $O
cd $R
for args in "--steps 10" "--steps 20" "--steps 80" "--steps 10 --records 131072" "--steps 40 --records 131072" "--steps 20 --warmup 30" "--steps 20"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline $args > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  echo "[$args] $(python3 -c "import json; d=json.loads(open('$O/b.json').read().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done
