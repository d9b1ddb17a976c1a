#!/bin/bash
# Quick PMC passes (SQ groups only) over a short bench.py run.
# usage: scripts/pmc_quick.sh TAG [bench args]   (env PMC_GROUPS overrides the counter groups, ';'-separated)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
G=${PMC_GROUPS:-"SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE;SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM"}
i=0
IFS=';' read -ra GRPS <<< "$G"
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $O/pmc$i -o pmc -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > $O/pmc$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
