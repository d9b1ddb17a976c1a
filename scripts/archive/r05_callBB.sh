#!/bin/bash
# round 5 call BB: the no-pack queue kernel's tail-priority window (last 32 /
# 48 / 80 claims of a run) on config B, warm bench, same box
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05bb
mkdir -p $O
cd $R
bash scripts/ab_bench.sh r05bb/abB 3 "_variants/lib_w3.so _variants/lib_w2.so _variants/lib_w5.so" > $O/abB.txt 2>&1 || exit $?
