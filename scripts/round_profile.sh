#!/bin/bash
# Round-end measurement set (run on the GPU box via gpurun):
#   bench lines for configs B (metric), C, D; rocprofv3 kernel-trace stats of B,
#   C, D; FETCH_SIZE / WRITE_SIZE PMC passes of B (separate runs, MI355X_MICROARCH.md
#   HBM section) summarised into profiles/pmc_configB.json for bench.py's roofline.traffic.
# usage: scripts/round_profile.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for c in B C D; do
  timeout -k 10 400 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err
  rc=$?; echo "bench $c rc=$rc"; cat $O/bench_$c.json
  [ $rc -ne 0 ] && exit $rc
done
cd /tmp && export TMPDIR=/tmp
for c in B C D; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o prof -- \
    python3 $R/bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > $O/prof_$c.log 2>&1
  rc=$?; echo "prof $c rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $O/pmcB/pmc$i -o pmc -- \
    python3 $R/bench.py --config B --steps 3 --warmup 1 --no-cpu-baseline > $O/pmcB_$i.log 2>&1
  rc=$?; echo "pmc $grp rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
