#!/bin/bash
# ChaCha parity tests under each variant library, then a same-box A/B on C.
# usage: scripts/ab_cc_variants.sh TAG "lib ..." [rounds]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
for lib in $2; do
  TLSGPU_LIBRARY=$R/$lib timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "chacha or C" \
    --timeout 120 --timeout-method thread > $O/tests_$(basename $lib).log 2>&1
  rc=$?; echo "tests $lib rc=$rc $(tail -1 $O/tests_$(basename $lib).log)"
  [ $rc -ne 0 ] && exit $rc
done
bash scripts/ab_bench.sh $1/ab ${3:-3} "$2" --config C
