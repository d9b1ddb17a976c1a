#!/bin/bash
# round 6 call Y: with the wave-priority pass, the tail-priority window —
# default (last 48 claims), every claim (TG_TAIL_WIN=1000), last 16 (=1); B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06y
mkdir -p $O
cd $R
L="talos_amd/libtlsgpu.so _variants/lib_tw1000.so _variants/lib_tw1.so"
bash scripts/ab_bench.sh r06y/abB 4 "$L" > $O/abB.txt 2>&1 || exit $?
cat $O/abB.txt
