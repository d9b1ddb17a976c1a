#!/bin/bash
# Same-box A/B of engine settings read from the environment at library load
# (TLSGPU_*): runs bench.py once per setting, ROUNDS times.
# usage: scripts/env_ab.sh TAG ROUNDS "SET1|SET2|..." [bench args]
#   each SET is a space-separated list of VAR=value ("-" = no extra setting)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; shift
ROUNDS=$1; shift
IFS='|' read -ra SETS <<< "$1"; shift
mkdir -p $O
cd $R
for k in $(seq $ROUNDS); do
  for set in "${SETS[@]}"; do
    [ "$set" = "-" ] && set=""
    env $set timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 "$@" > $O/ab.json 2>$O/ab.err || { tail -5 $O/ab.err; exit 1; }
    echo "$k [$set] $(python3 -c "import json; d=json.loads(open('$O/ab.json').read().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
  done
done
