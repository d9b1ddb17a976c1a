#!/bin/bash
# Round-4 call S: the GPU suite with the doorbell on for every test (new exit
# drain), then in the default environment, then smoke().
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04x}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
PYTHONFAULTHANDLER=1 TLSGPU_EVP_DOORBELL=64 timeout -k 10 700 python -u -m pytest tests -v --timeout 120 \
  --timeout-method thread -m gpu > $O/suite_doorbell.log 2>&1
rc=$?; echo "suite (doorbell=64) rc=$rc $(tail -1 $O/suite_doorbell.log)"; grep -E "FAILED|ERROR" $O/suite_doorbell.log | head
[ $rc -ge 124 ] && exit $rc
timeout -k 10 700 python -u -m pytest tests -v --timeout 120 --timeout-method thread -m gpu > $O/suite.log 2>&1
rc=$?; echo "suite (default) rc=$rc $(tail -1 $O/suite.log)"; grep -E "FAILED|ERROR" $O/suite.log | head
[ $rc -ge 124 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "smoke rc=$? $(tail -1 $O/smoke.log)"
exit 0
