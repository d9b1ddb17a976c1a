#!/bin/bash
# round 6 call AE: config C with the staged kernel's memory phase (scatter +
# next gather) at priority 2 / 1 (TG_CC_MEM_PRIO) against the kept build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06ae
mkdir -p $O
cd $R
L="talos_amd/libtlsgpu.so _variants/lib_cm2.so _variants/lib_cm1.so"
bash scripts/ab_bench.sh r06ae/abC 4 "$L" --config C > $O/abC.txt 2>&1 || exit $?
cat $O/abC.txt
