#!/bin/bash
# One GPU-box round trip (round 3): parity suite, a list of bench lines, then
# optional kernel-trace stats and PMC passes.
# usage: scripts/gpu_run.sh TAG [--no-tests] [--kstats "B D"] [--pmc "B C"] -- NAME:ARGS ...
#   e.g. scripts/gpu_run.sh r03f --pmc B -- B: "B_nohints:--no-hints" "D:--config D"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
TESTS=1; KSTATS=""; PMC=""
while [ $# -gt 0 ] && [ "$1" != "--" ]; do
  case $1 in
    --no-tests) TESTS=0;;
    --kstats) KSTATS=$2; shift;;
    --pmc) PMC=$2; shift;;
  esac
  shift
done
[ "$1" = "--" ] && shift
if [ $TESTS = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
  [ $rc -ne 0 ] && exit $rc
fi
for spec in "$@"; do
  n=${spec%%:*}; a=${spec#*:}
  timeout -k 10 300 python bench.py $a > $O/bench_$n.json 2> $O/bench_$n.err
  rc=$?; echo "bench $n rc=$rc $(cut -c1-150 $O/bench_$n.json)"
  [ $rc -ne 0 ] && exit $rc
done
for c in $KSTATS; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $O/k$c -o run -- python3 $R/bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline \
    > $O/k$c.log 2>&1) || exit 1
  echo "kstats $c: $(tail -1 $O/k$c.log | cut -c1-120)"
done
for c in $PMC; do
  bash scripts/pmc.sh $TAG/pmc$c --config $c || exit $?
done
exit 0
