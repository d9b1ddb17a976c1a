#!/bin/bash
# round 5 call M: the staged ChaCha kernel at 3 waves per SIMD on one side
# only (TLSGPU_CC_LDS_PAD_OPEN / _SEAL = 1024 B of unused LDS per workgroup),
# same-box A/B of config C and wire C (open only).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05m
mkdir -p $O
cd $R
bash scripts/env_ab.sh r05m/abC 3 "-|TLSGPU_CC_LDS_PAD_OPEN=1024|TLSGPU_CC_LDS_PAD_SEAL=1024" --config C > $O/abC.txt 2>&1 || exit $?
bash scripts/env_ab.sh r05m/abW 2 "-|TLSGPU_CC_LDS_PAD_OPEN=1024" --config C --mode wire > $O/abW.txt 2>&1 || exit $?
