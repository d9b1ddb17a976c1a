#!/bin/bash
# round 5 call R: whole-piece balance (TLSGPU_PIECES), one-pass prologue — parity (fused cases,
# full-size digests with pieces on), per-workgroup timing, same-box A/B of D
# and B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05r
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py -k "fused" tests/test_gpu_batch_digests.py > $O/tests.log 2>&1 || exit $?
TLSGPU_PIECES=2 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_batch_digests.py tests/test_gpu_parity.py -k "fused or batch_seal_open or pack or digest" \
  > $O/tests_pieces.log 2>&1 || exit $?
for p in 0 1; do
  echo "## TLSGPU_PIECES=$p" >> $O/wg_times.jsonl
  TLSGPU_PIECES=$p TLSGPU_WG_TIMES=1 timeout -k 10 180 python tools/wg_times.py --config D --launches 3 \
    >> $O/wg_times.jsonl 2> $O/err.txt || exit 1
done
bash scripts/env_ab.sh r05r/abD 4 "TLSGPU_PIECES=0|TLSGPU_PIECES=1" --config D > $O/abD.txt 2>&1 || exit $?
bash scripts/env_ab.sh r05r/abB 2 "TLSGPU_PIECES=0|TLSGPU_PIECES=2" --config B > $O/abB.txt 2>&1 || exit $?
