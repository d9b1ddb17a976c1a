#!/bin/bash
# round 6 call AA: two more compiler options on top of the kept build —
# -misched-cluster=false (nc), -amdgpu-scalarize-global-loads=false (nsc); B, D, C
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06aa
mkdir -p $O
cd $R
L="talos_amd/libtlsgpu.so _variants/lib_nc.so _variants/lib_nsc.so"
bash scripts/ab_bench.sh r06aa/abB 3 "$L" > $O/abB.txt 2>&1 || exit $?
cat $O/abB.txt
bash scripts/ab_bench.sh r06aa/abD 2 "$L" --config D > $O/abD.txt 2>&1 || exit $?
cat $O/abD.txt
bash scripts/ab_bench.sh r06aa/abC 2 "$L" --config C > $O/abC.txt 2>&1 || exit $?
cat $O/abC.txt
