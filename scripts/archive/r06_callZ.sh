#!/bin/bash
# round 6 call Z: D with a raised priority from each claim (pack or long
# record) to the wave-priority pass's first drop (TG_PACK_START_PRIO)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06z
mkdir -p $O
cd $R
L="talos_amd/libtlsgpu.so _variants/lib_dsp.so"
bash scripts/ab_bench.sh r06z/abD 4 "$L" --config D > $O/abD.txt 2>&1 || exit $?
cat $O/abD.txt
