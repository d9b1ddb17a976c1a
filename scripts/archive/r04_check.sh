#!/bin/bash
# Round-4 GPU check: new parity tests, group split bench, ubench set4.
set -o pipefail
O=gpurun_out/${1:-r04c}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_wire_reference.py tests/test_group.py -x -v \
  --timeout 120 --timeout-method thread -m gpu > ${O}_tests.log 2>&1 &&
timeout -k 10 200 python -u bench.py --no-cpu-baseline > ${O}_bench_B.json 2> ${O}_bench_B.err &&
timeout -k 10 200 python -u bench.py --split group --devices 0 --no-cpu-baseline > ${O}_group1.json 2> ${O}_group1.err &&
timeout -k 10 200 python -u bench.py --split group --devices 0,0 --no-cpu-baseline > ${O}_group00.json 2> ${O}_group00.err &&
timeout -k 10 300 tools/ubench set4 > ${O}_ubench_set4.jsonl 2>&1
