#!/bin/bash
# round 6 call N: the committed tree as the driver runs it — the GPU suite and
# smoke(), then bench.py with the driver's flags (config B), C and D
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06n
mkdir -p $O
cd $R
bash scripts/gpu_suite.sh r06n/suite || { tail -30 $O/suite_tests.log; exit 1; }
tail -2 $O/suite_tests.log; tail -3 $O/suite_smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_B.json 2> $O/bench_B.err || exit $?
cut -c1-300 $O/bench_B.json
for c in C D; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 > $O/bench_$c.json 2> $O/bench_$c.err || exit $?
  cut -c1-200 $O/bench_$c.json
done
