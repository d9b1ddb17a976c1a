#!/bin/bash
# Round-4 doorbell check: probe floor, parity test, per-call bench, then the
# whole GPU suite.  A step that times out, aborts or faults ends the script
# (exit status >= 124); an ordinary test failure (1) does not stop the rest.
O=gpurun_out/${1:-r04f}
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "${O}_${name}.log" 2>&1
  local rc=$?
  echo "step $name rc=$rc"
  [ $rc -ge 124 ] && exit $rc   # timed out, killed, aborted or faulted: stop here
  return 0
}
step probe 60 tools/doorbell_probe
step abC 400 bash scripts/ab_bench.sh "$(basename $O)_abC" 3 "variants/libtlsgpu_base.so talos_amd/libtlsgpu.so" --config C
step doorbell_test 240 python -u -m pytest tests/test_evp_doorbell.py -x -v --timeout 120 --timeout-method thread -m gpu
step doorbell_bench 400 scripts/evp_doorbell_bench.sh "${O}_doorbell_bench.jsonl"
step copy 120 tools/ubench copy
