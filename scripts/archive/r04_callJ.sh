#!/bin/bash
# Round-4 call J: doorbell parity and per-call bench after the relaunch fix.
# usage: scripts/r04_callJ.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04o}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_evp_doorbell.py tests/test_evp_churn.py tests/test_gpu_parity.py -x -v \
  --timeout 120 --timeout-method thread -m gpu -k "doorbell or churn or split_jobs or chacha_wave or aeadtests" \
  > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
timeout -k 10 480 scripts/evp_doorbell_bench.sh "$O/doorbell_bench.jsonl" > $O/doorbell_bench.log 2>&1
echo "doorbell bench rc=$?"
python3 - "$O/doorbell_bench.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); n = d.get("records", d.get("contexts"))
    print(f'{d["lib"][10:]:30s} {d["aead"]:18s} {d["rec_len"]:6d} T={d["threads"]:3d} {n/d["seconds"]/1e3:8.1f} K/s fail={d["failures"]} s={d["seconds"]}')
PY
exit 0
