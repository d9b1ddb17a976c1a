#!/bin/bash
# round 6 call V: where the wave-priority pass's +2 % on B comes from —
# default, no tail priority (TG_NO_TAIL_PRIO), the pass (wp), both; B and D
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06v
mkdir -p $O
cd $R
L="talos_amd/libtlsgpu.so _variants/lib_ntp.so _variants/lib_wp.so _variants/lib_wpntp.so"
bash scripts/ab_bench.sh r06v/abB 4 "$L" > $O/abB.txt 2>&1 || exit $?
cat $O/abB.txt
bash scripts/ab_bench.sh r06v/abD 2 "$L" --config D > $O/abD.txt 2>&1 || exit $?
cat $O/abD.txt
