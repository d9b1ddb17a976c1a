#!/bin/bash
# Parity suite under each library (in-tree first), then a same-box A/B of the
# libraries on the given configs.  usage: scripts/ab_variants.sh TAG "lib ..." "B D" [rounds]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
for lib in $2; do
  TLSGPU_LIBRARY=$R/$lib timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
    --timeout 120 --timeout-method thread > $O/tests_$(basename $lib).log 2>&1
  rc=$?; echo "tests $lib rc=$rc $(tail -1 $O/tests_$(basename $lib).log)"
  [ $rc -ne 0 ] && exit $rc
done
for c in $3; do
  bash scripts/ab_bench.sh $1/ab$c ${4:-3} "$2" --config $c || exit 1
done
