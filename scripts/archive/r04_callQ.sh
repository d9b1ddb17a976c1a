#!/bin/bash
# Round-4 call Q (end of round): GPU suite, smoke(), the default bench line.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04v}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -v --timeout 120 --timeout-method thread -m gpu > $O/suite.log 2>&1
rc=$?; echo "suite rc=$rc $(tail -1 $O/suite.log)"; grep -E "FAILED|ERROR" $O/suite.log | head -20
[ $rc -ge 124 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 $O/smoke.log)"
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
echo "bench rc=$? $(cut -c1-400 $O/bench.json)"
exit 0
