#!/bin/bash
# Measurement set for a round (run on the GPU box via gpurun):
#   bench lines: B (metric), B at S = 1 / 65,536 sessions and interleaved, C, D,
#   the box's copy bandwidth, host-resident B (tlsgpu_open_host), the pinned
#   PCIe rates, wire B / C / D (tlsgpu_open_wire); then PMC passes (scripts/pmc.sh) for
#   B, C and D.
# usage: scripts/measure_set.sh TAG [--no-pmc]
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
  echo "bench $n rc=$rc $(cut -c1-200 $O/bench_$n.json)"
  return $rc
}
run copy --mode copy --steps 20 &&
run B &&
run B_S1 --sessions 1 --no-cpu-baseline &&
run B_S65536 --sessions 65536 --no-cpu-baseline &&
run B_inter1024 --sessions 1024 --interleave --no-cpu-baseline &&
run C --config C &&
run D --config D &&
run host_B --mode host --no-cpu-baseline --steps 8 --warmup 2 &&
run pcie --mode pcie &&
run wire_B --mode wire --no-cpu-baseline &&
run wire_C --mode wire --config C --no-cpu-baseline &&
run wire_D --mode wire --config D --no-cpu-baseline &&
run group_dev0 --split group --devices 0 --no-cpu-baseline &&
run group_dev00 --split group --devices 0,0 --no-cpu-baseline || exit $?
[ "$2" = "--no-pmc" ] && exit 0
for c in B C D; do
  bash scripts/pmc.sh $TAG/pmc$c --config $c || exit $?
done
exit 0
