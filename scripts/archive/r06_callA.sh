#!/bin/bash
# round 6 call A: GPU suite + smoke on the round-6 tree (AES-NI host image),
# the driver's bench command, the N > 1 bench plumbing on a 1-GPU box
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06a
mkdir -p $O
cd $R
bash scripts/gpu_suite.sh r06a/suite || exit $?
tail -3 $O/suite_tests.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_B.json 2> $O/bench_B.err || exit $?
cut -c1-400 $O/bench_B.json
# --gpus 2 on a one-GPU box must refuse (exit non-zero), not measure one GPU
timeout -k 10 120 python bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_g2.json 2> $O/bench_g2.err
rc=$?; echo "gpus2 rc=$rc (want 1)"; tail -2 $O/bench_g2.err
[ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -gt 128 ] && exit $rc
timeout -k 10 300 python bench.py --gpus 2 --devices 0,0 --steps 20 --warmup 5 > $O/bench_g00.json 2> $O/bench_g00.err || exit $?
cut -c1-600 $O/bench_g00.json
timeout -k 10 300 python bench.py --config D --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_D.json 2> $O/bench_D.err || exit $?
timeout -k 10 300 python bench.py --config C --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_C.json 2> $O/bench_C.err || exit $?
cut -c1-200 $O/bench_D.json $O/bench_C.json
