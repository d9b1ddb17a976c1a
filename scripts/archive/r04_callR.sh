#!/bin/bash
# Round-4 call R: GPU suite + smoke() in the default environment (doorbell
# off), then one run of the two-engine EVP test with the doorbell on and the
# Python fault handler, for the exit-time SIGSEGV seen once in r04v.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04w}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -v --timeout 120 --timeout-method thread -m gpu > $O/suite.log 2>&1
rc=$?; echo "suite rc=$rc $(tail -1 $O/suite.log)"; grep -E "FAILED|ERROR" $O/suite.log | head -20
[ $rc -ge 124 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 $O/smoke.log)"
[ $rc -ge 124 ] && exit $rc
PYTHONFAULTHANDLER=1 TLSGPU_EVP_DOORBELL=64 timeout -k 10 200 python -u -m pytest tests/test_evp_multi_device.py -v \
  --timeout 120 --timeout-method thread -m gpu > $O/multi_doorbell.log 2>&1
echo "multi-device with doorbell rc=$? $(tail -1 $O/multi_doorbell.log)"
exit 0
