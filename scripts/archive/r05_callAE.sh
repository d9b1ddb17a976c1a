#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ae
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for r in 65536 131072; do
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d $O/p$r -o pmc -- \
    python3 $R/bench.py --steps 6 --warmup 2 --no-cpu-baseline --records $r > $O/p$r.log 2>&1 || exit 1
done
