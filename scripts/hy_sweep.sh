#!/bin/bash
# Sweep hybrid-kernel knobs on bench config B.  usage: scripts/hy_sweep.sh TAG "FLAGS:RESERVE ..."
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O; cd $R
for fr in $2; do
  f=${fr%%:*}; r=${fr##*:}
  TLSGPU_HY_FLAGS=$f TLSGPU_BS_RESERVE=$r timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/b_${f}_${r}.json 2>$O/b_${f}_${r}.err || exit 1
  echo "flags=$f reserve=$r $(grep -o '"value": [0-9.]*' $O/b_${f}_${r}.json)"
done
