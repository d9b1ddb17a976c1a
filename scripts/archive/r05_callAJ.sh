#!/bin/bash
# round 5 call AJ: PMC pass 1 + LDS pass for B with the warm-start bench
# (warm-up 30): the working clock and LDS busy of warm launches
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05aj
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $O/p$i -o pmc -- \
    python3 $R/bench.py --steps 10 --no-cpu-baseline > $O/p$i.log 2>&1 || exit 1
done
