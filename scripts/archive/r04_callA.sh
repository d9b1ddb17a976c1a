#!/bin/bash
# Round-4 GPU call A: the doorbell parity test and per-call bench, then the
# whole GPU suite and smoke().  A step that times out, aborts or faults ends
# the script (status >= 124); an ordinary failure (1) does not stop the rest.
O=gpurun_out/${1:-r04h}
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "${O}_${name}.log" 2>&1
  local rc=$?
  echo "step $name rc=$rc"
  [ $rc -ge 124 ] && exit $rc
  return 0
}
step ubench5 60 tools/ubench set5
step chacha_wave 200 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu -k "chacha_wave or aeadtests"
step doorbell_test 240 python -u -m pytest tests/test_evp_doorbell.py -x -v --timeout 120 --timeout-method thread -m gpu
step doorbell_bench 400 scripts/evp_doorbell_bench.sh "${O}_doorbell_bench.jsonl"
step suite 700 python -u -m pytest tests -v --timeout 120 --timeout-method thread -m gpu
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
