#!/bin/bash
# round 6 call AD: the x2 loop's next-group loads issued at priority 2
# (TG_LOAD_PRIO) against the kept build; B and D, 4 rounds
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06ad
mkdir -p $O
cd $R
L="talos_amd/libtlsgpu.so _variants/lib_lp2.so"
bash scripts/ab_bench.sh r06ad/abB 4 "$L" > $O/abB.txt 2>&1 || exit $?
cat $O/abB.txt
bash scripts/ab_bench.sh r06ad/abD 3 "$L" --config D > $O/abD.txt 2>&1 || exit $?
cat $O/abD.txt
