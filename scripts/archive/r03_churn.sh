#!/bin/bash
# Parity suite, connection churn (contexts/s) and the EVP kernel profile.
# usage: scripts/r03_churn.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -ne 0 ] && exit $rc
bash scripts/churn_bench.sh $O/churn.jsonl > /dev/null || exit 1
python3 -c "
import json
for l in open('$O/churn.jsonl'):
    d=json.loads(l); print(d['lib'], d['threads'], round(d['contexts_per_s']), d['us_per_context_per_thread'])"
bash scripts/evp_kernel_profile.sh $1/evp > $O/evp_profile.txt 2>&1 || exit 1
for d in $O/evp/*/; do python3 scripts/rocpd_summary.py $d/run_results.db | grep -i install; done
exit 0
