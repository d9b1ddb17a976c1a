#!/bin/bash
# round 6 call K: soaks on the final tree — the doorbell per-call path with
# 300 contexts per thread (1 and 12 threads), the batch path's randomized
# differential with 300 seeds — and multi-GPU rehearsals on one GPU: an
# 8-member group on device 0 and a 2-rank torch.distributed.run launch
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06k
mkdir -p $O
cd $R
TLSGPU_SOAK_ITERS=300 timeout -k 10 900 python -u -m pytest tests/test_evp_doorbell.py -x -v \
  -k matches_oracle --timeout 1000 --timeout-method thread > $O/soak_doorbell.log 2>&1 || exit $?
tail -3 $O/soak_doorbell.log
TLSGPU_FUZZ_SEEDS=300 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q \
  -k random_differential --timeout 1000 --timeout-method thread > $O/soak_random_differential.log 2>&1 || exit $?
tail -3 $O/soak_random_differential.log
timeout -k 10 300 python bench.py --gpus 8 --devices 0,0,0,0,0,0,0,0 --steps 10 --warmup 2 --no-cpu-baseline \
  > $O/bench_group8_dev0.json 2> $O/bench_group8_dev0.err || exit $?
cut -c1-700 $O/bench_group8_dev0.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --devices 0,0 --steps 10 --warmup 2 \
  > $O/bench_torchrun2_dev00.json 2> $O/bench_torchrun2_dev00.err || exit $?
cut -c1-400 $O/bench_torchrun2_dev00.json
