#!/bin/bash
# round 5 call AN: config C occupancy with the warm-start bench: round-4 order
# at 4 waves/SIMD (default), LATE_STORES at 3 waves/SIMD, round-4 order at 3
# waves/SIMD (LDS pad)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05an
mkdir -p $O
cd $R
bash scripts/env_ab.sh r05an/abC 3 "-|TLSGPU_CC_ORDER=1|TLSGPU_CC_LDS_PAD=1024" --config C > $O/abC.txt 2>&1 || exit $?
