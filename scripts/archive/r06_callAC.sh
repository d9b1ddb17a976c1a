#!/bin/bash
# round 6 call AC: soaks on the final build — the batch path's randomized
# differential with 300 seeds, the doorbell per-call path with 300 contexts
# per thread — and a long B run (200 timed steps, the driver's warm-up)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06ac
mkdir -p $O
cd $R
TLSGPU_FUZZ_SEEDS=300 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q \
  -k random_differential --timeout 1000 --timeout-method thread > $O/soak_random_differential.log 2>&1 || exit $?
tail -1 $O/soak_random_differential.log
TLSGPU_SOAK_ITERS=300 timeout -k 10 900 python -u -m pytest tests/test_evp_doorbell.py -x -v \
  -k matches_oracle --timeout 1000 --timeout-method thread > $O/soak_doorbell.log 2>&1 || exit $?
tail -1 $O/soak_doorbell.log
timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 5 > $O/bench_B_200.json 2> $O/bench_B_200.err || exit $?
cut -c1-260 $O/bench_B_200.json
