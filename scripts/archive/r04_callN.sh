#!/bin/bash
# Round-4 call N: the whole GPU suite with the doorbell on for every EVP
# per-call path (TLSGPU_EVP_DOORBELL=64), then smoke().
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04s}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
TLSGPU_EVP_DOORBELL=64 timeout -k 10 700 python -u -m pytest tests -v --timeout 120 --timeout-method thread -m gpu \
  > $O/suite_doorbell.log 2>&1
echo "suite (doorbell=64) rc=$? $(tail -1 $O/suite_doorbell.log)"
grep -E "FAILED|ERROR" $O/suite_doorbell.log | head -20
TLSGPU_EVP_DOORBELL=64 timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "smoke rc=$? $(tail -1 $O/smoke.log)"
exit 0
