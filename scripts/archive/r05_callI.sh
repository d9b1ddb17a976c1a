#!/bin/bash
# round 5 call I: snapped work cuts (TLSGPU_BALANCE_SNAP) — parity, then
# per-workgroup timing and a same-box bench A/B of config D.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05i
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py -k "balanced" > $O/tests.log 2>&1 || exit $?
for set in "TLSGPU_BALANCE=0" "TLSGPU_BALANCE=1 TLSGPU_BALANCE_SNAP=0" "TLSGPU_BALANCE_SNAP=64" \
           "TLSGPU_BALANCE_SNAP=128" "TLSGPU_BALANCE_SNAP=256" "TLSGPU_BALANCE_SNAP=512"; do
  echo "## $set" >> $O/wg_times.jsonl
  env $set TLSGPU_WG_TIMES=1 timeout -k 10 180 python tools/wg_times.py --config D --launches 3 \
    >> $O/wg_times.jsonl 2> $O/err.txt || exit 1
done
bash scripts/env_ab.sh r05i/abD 3 "TLSGPU_BALANCE=0|TLSGPU_BALANCE_SNAP=128|TLSGPU_BALANCE_SNAP=256" --config D \
  > $O/abD.txt 2>&1 || exit $?
