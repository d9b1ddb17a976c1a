#!/bin/bash
# GPU parity suite, then bench lines B / D / C / B at S = 65,536 (no CPU baseline).
# usage: scripts/quick_bench.sh TAG [skip-tests]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1
  rc=$?; tail -2 $O/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
fi
for cfg in "B" "D --config D" "C --config C" "S65536 --sessions 65536"; do
  set -- $cfg
  n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/bench_$n.json 2> $O/bench_$n.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/bench_$n.json').read().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'])"
done
