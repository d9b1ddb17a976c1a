#!/bin/bash
# GCM: parity suite on the in-tree build, then a same-box A/B of library
# variants on configs B and D.  usage: scripts/ab_gcm.sh TAG "lib ..." [rounds]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -ne 0 ] && exit $rc
bash scripts/ab_bench.sh $1/abB ${3:-3} "$2" || exit 1
bash scripts/ab_bench.sh $1/abD ${3:-3} "$2" --config D
