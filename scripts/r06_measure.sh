#!/bin/bash
# round 6 final measurement set: bench lines (the driver's flags for B / C / D,
# the other modes as measure_set.sh runs them), rocprofv3 kernel stats of B / C
# / D, and PMC passes for config B; outputs under gpurun_out/$TAG.
# usage: scripts/r06_measure.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err
  local rc=$?
  echo "bench $n rc=$rc $(cut -c1-220 $O/bench_$n.json)"
  return $rc
}
run B_driver --gpus 1 --steps 20 --warmup 5 &&
run B_driver2 --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline &&
run C_driver --config C --steps 20 --warmup 5 --no-cpu-baseline &&
run D_driver --config D --steps 20 --warmup 5 --no-cpu-baseline &&
run B --no-cpu-baseline &&
run B_S1 --sessions 1 --no-cpu-baseline &&
run B_S65536 --sessions 65536 --no-cpu-baseline &&
run B_inter1024 --sessions 1024 --interleave --no-cpu-baseline &&
run C --config C &&
run D --config D &&
run copy --mode copy --steps 20 &&
run host_B --mode host --no-cpu-baseline --steps 8 --warmup 2 &&
run pcie --mode pcie &&
run wire_B --mode wire --no-cpu-baseline &&
run wire_C --mode wire --config C --no-cpu-baseline &&
run wire_D --mode wire --config D --no-cpu-baseline &&
run group_dev00 --gpus 2 --devices 0,0 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
[ "$2" = "--no-prof" ] && exit 0
bash scripts/kstats.sh $TAG/kstats || exit $?
LAST=10 bash scripts/pmc.sh $TAG/pmcB --config B || exit $?
exit 0
