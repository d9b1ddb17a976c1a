#!/bin/bash
# Config C check (GPU box): parity suite, bench C and wire C, PMC passes of C.
# usage: scripts/r03_cc.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
for m in "C --config C" "wire_C --mode wire --config C --no-cpu-baseline"; do
  set -- $m; n=$1; shift
  timeout -k 10 300 python bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err || exit 1
  echo "bench $n $(cut -c1-160 $O/bench_$n.json)"
done
LIST=1 bash scripts/pmc.sh $TAG/pmcC --config C || exit $?
python3 scripts/pmc_summary.py $O/pmcC "void tg::chacha_tls_kernel" $O/pmcC.json "r03 staged ChaCha, 4 waves/SIMD" > /dev/null
python3 -c "import json;d=json.load(open('$O/pmcC.json'));print({k:d.get(k) for k in ('mean_duration_ns_profiled','hbm_read_bytes_per_launch','hbm_write_bytes_per_launch','bench_lines_of_these_passes')})"
# request-size counters (calibration of FETCH_SIZE on this access pattern); tolerated if absent
cd /tmp && export TMPDIR=/tmp
for grp in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_BUBBLE_sum TCC_EA0_WRREQ_sum" "TCC_EA0_WRREQ_64B_sum TCC_REQ_sum"; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $O/cal_${grp%% *} -o pmc -- \
    python3 $R/bench.py --config C --steps 3 --warmup 1 --no-cpu-baseline > $O/cal_${grp%% *}.log 2>&1
  echo "cal $grp rc=$?"
done
exit 0
