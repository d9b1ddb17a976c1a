#!/bin/bash
# Round-4 call T: line-aligned record slots (bench.py --slot-align 128) vs the
# default 16-B layout, configs C, B, D (C twice, alternating).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04y}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for r in 1 2; do
  for a in 16 128; do
    timeout -k 10 300 python bench.py --config C --no-cpu-baseline --slot-align $a > $O/C_a$a.r$r.json 2> $O/C_a$a.r$r.err || exit $?
    echo "C align $a r$r $(python3 -c 'import json,sys;d=json.load(open(sys.argv[1]));print(d["value"], d["ms_per_step"])' $O/C_a$a.r$r.json)"
  done
done
for c in B D; do
  for a in 16 128; do
    timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --slot-align $a > $O/${c}_a$a.json 2> $O/${c}_a$a.err || exit $?
    echo "$c align $a $(python3 -c 'import json,sys;d=json.load(open(sys.argv[1]));print(d["value"], d["ms_per_step"])' $O/${c}_a$a.json)"
  done
done
TLSGPU_CC_DIAG=4 timeout -k 10 240 python tools/cc_diag.py > $O/cc_diag4_a16.json 2>&1 || exit $?
echo "diag4 (16) $(cat $O/cc_diag4_a16.json)"
exit 0
