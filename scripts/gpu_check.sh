#!/bin/bash
# One GPU-box round trip: parity tests, then a bench line (+ optional rocprof).
# usage: scripts/gpu_check.sh TAG [bench args...]   (PROF=1 adds a kernel-trace pass)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py "$@" > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cat $O/bench.json; tail -3 $O/bench.err
[ $rc -ne 0 ] && exit $rc
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o prof -- \
    python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@" > $O/prof.log 2>&1
  rc=$?; echo "prof rc=$rc"; cat $O/prof/prof_kernel_stats.csv 2>/dev/null | head -5
fi
exit $rc
