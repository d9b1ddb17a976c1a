#!/bin/bash
# rocprofv3 kernel-trace --stats of bench.py for configs B, C, D (kernel
# durations per step: prep pass, status memset, main kernel).
# usage: scripts/kstats.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in B C D; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k$c -o run -- \
    python3 $R/bench.py --config $c --steps 10 --no-cpu-baseline > $O/k$c.log 2>&1 || exit 1
  tail -1 $O/k$c.log | cut -c1-160
done
