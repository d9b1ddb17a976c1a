#!/bin/bash
# PMC passes over bench.py (one rocprofv3 process per counter group, kernel
# trace only; the bench's default 30-step warm-up, then 10 timed steps, whose
# launches scripts/pmc_summary.py keeps with LAST=10 / 20 for C; round 5), kernel
# trace only: no sys/runtime tracing with --pmc).  usage: scripts/pmc.sh TAG [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
[ -n "$LIST" ] && (timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || true)
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" \
           "TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_64B_sum" ${EXTRA_GROUPS}; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $O/pmc$i -o pmc -- \
    python3 $R/bench.py --steps 10 --no-cpu-baseline "$@" > $O/pmc$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
