#!/bin/bash
# The round-end driver's sequence on the committed tree: GPU suite + smoke(),
# then bench.py as the driver runs it (N = 1), and the N = 2 group path on one
# GPU (devices 0,0).  usage: scripts/final_check.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
bash scripts/gpu_suite.sh $1/suite || { tail -30 $O/suite_tests.log; exit 1; }
tail -1 $O/suite_tests.log; tail -1 $O/suite_smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_B.json 2> $O/bench_B.err || exit $?
cut -c1-200 $O/bench_B.json
timeout -k 10 300 python bench.py --gpus 2 --devices 0,0 --steps 20 --warmup 5 --no-cpu-baseline \
  > $O/bench_group00.json 2> $O/bench_group00.err || exit $?
cut -c1-200 $O/bench_group00.json
