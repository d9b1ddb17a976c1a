#!/bin/bash
# Same-box A/B of library builds (box-to-box variance is ~7 %): runs bench.py
# with each library (TLSGPU_LIBRARY) in turn, ROUNDS times, for the given
# bench arguments.  usage: scripts/ab_bench.sh TAG ROUNDS "lib1 lib2 ..." [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; shift
ROUNDS=$1; shift
LIBS=$1; shift
mkdir -p $O
cd $R
for k in $(seq $ROUNDS); do
  for lib in $LIBS; do
    TLSGPU_LIBRARY=$R/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 "$@" > $O/ab.json 2>$O/ab.err || exit 1
    echo "$k $lib $(python3 -c "import json; d=json.loads(open('$O/ab.json').read().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
  done
done
