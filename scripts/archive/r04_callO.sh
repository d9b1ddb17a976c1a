#!/bin/bash
# Round-4 call O (final check): the GPU suite and smoke() in the default
# environment (doorbell on), then the per-call bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04t}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -v --timeout 120 --timeout-method thread -m gpu > $O/suite.log 2>&1
rc=$?; echo "suite rc=$rc $(tail -1 $O/suite.log)"; grep -E "FAILED|ERROR" $O/suite.log | head -20
[ $rc -ge 124 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 $O/smoke.log)"
[ $rc -ge 124 ] && exit $rc
timeout -k 10 480 scripts/evp_doorbell_bench.sh "$O/doorbell_bench.jsonl" > $O/doorbell_bench.log 2>&1
echo "doorbell bench rc=$?"
python3 - "$O/doorbell_bench.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); n = d.get("records", d.get("contexts"))
    print(f'{d["lib"][10:]:30s} {d["aead"]:18s} {d["rec_len"]:6d} T={d["threads"]:3d} {n/d["seconds"]/1e3:8.1f} K/s fail={d["failures"]}')
PY
exit 0
