#!/bin/bash
# round 5 call AM: earlier A/Bs again with the warm-start bench (they were
# measured in the clock dip): workgroups per CU (B, D), ChaCha step order (C),
# longest-first pieces (D)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05am
mkdir -p $O
cd $R
bash scripts/env_ab.sh r05am/abB 3 "TLSGPU_WG_PER_CU=1|TLSGPU_WG_PER_CU=2" > $O/abB.txt 2>&1 || exit $?
bash scripts/env_ab.sh r05am/abC 3 "TLSGPU_CC_ORDER=0|TLSGPU_CC_ORDER=2" --config C > $O/abC.txt 2>&1 || exit $?
bash scripts/env_ab.sh r05am/abD 3 "-|TLSGPU_WG_PER_CU=2|TLSGPU_PIECES=0" --config D > $O/abD.txt 2>&1 || exit $?
