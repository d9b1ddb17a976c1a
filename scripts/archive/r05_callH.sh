#!/bin/bash
# round 5 call H: per-workgroup timing of the queue kernel (TLSGPU_WG_TIMES)
# for config D with equal-count and work-balanced ranges, and config B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05h
mkdir -p $O
cd $R
export TLSGPU_WG_TIMES=1
for b in 0 1; do
  TLSGPU_BALANCE=$b timeout -k 10 180 python tools/wg_times.py --config D --launches 3 >> $O/wg_times.jsonl 2> $O/err_D$b.txt || exit 1
done
TLSGPU_BALANCE=0 timeout -k 10 180 python tools/wg_times.py --config B --launches 2 >> $O/wg_times.jsonl 2> $O/err_B.txt || exit 1
