#!/bin/bash
# round 6 call AB: the per-record finish (close chain, Shoup weights, tag) at
# priority 2 / 1 (TG_FINISH_PRIO) against the kept build; B and D
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06ab
mkdir -p $O
cd $R
L="talos_amd/libtlsgpu.so _variants/lib_fp2.so _variants/lib_fp1.so"
bash scripts/ab_bench.sh r06ab/abB 3 "$L" > $O/abB.txt 2>&1 || exit $?
cat $O/abB.txt
bash scripts/ab_bench.sh r06ab/abD 3 "$L" --config D > $O/abD.txt 2>&1 || exit $?
cat $O/abD.txt
