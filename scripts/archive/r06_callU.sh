#!/bin/bash
# round 6 call U: compiler scheduling variants of the whole library, same box:
# -amdgpu-use-amdgpu-trackers (tr), -amdgpu-set-wave-priority (wp),
# -amdgpu-sched-strategy=max-ilp (ilp) against the default, configs B, C, D
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06u
mkdir -p $O
cd $R
L="talos_amd/libtlsgpu.so _variants/lib_tr.so _variants/lib_wp.so _variants/lib_ilp.so"
bash scripts/ab_bench.sh r06u/abB 3 "$L" > $O/abB.txt 2>&1 || exit $?
cat $O/abB.txt
bash scripts/ab_bench.sh r06u/abD 2 "$L" --config D > $O/abD.txt 2>&1 || exit $?
cat $O/abD.txt
bash scripts/ab_bench.sh r06u/abC 2 "$L" --config C > $O/abC.txt 2>&1 || exit $?
cat $O/abC.txt
