#!/bin/bash
# round 5 call C: the whole GPU suite on the working tree (shutdown contract,
# write-aligned ChaCha windows, fused queue prologue), then same-box A/B of
# B and C (base = HEAD 3fcaf41 kernels), then the exit-order probe.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05c
mkdir -p $O
cd $R
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/suite.log 2>&1 || exit $?
ab() {  # tag, bench args...
  local tag=$1; shift
  for k in 1 2 3; do
    for v in base new new0; do
      lib=_variants/lib_$v.so; env=""
      [ $v = new0 ] && lib=_variants/lib_new.so && env="TLSGPU_FUSED=0 TLSGPU_CC_ALIGN=0"
      env $env TLSGPU_LIBRARY=$R/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 "$@" > $O/ab.json 2>$O/ab.err || return 1
      echo "$tag $k $v $(python3 -c "import json; d=json.loads(open('$O/ab.json').read().splitlines()[-1]); print(d['value'], d['ms_per_step'])")" >> $O/ab.txt
    done
  done
}
ab B --config B && ab C --config C && ab D --config D || exit 1
cd tools
timeout -k 10 60 ./exit_order_probe nohip > ../gpurun_out/r05c/probe_nohip.txt 2>&1; echo "rc=$?" >> ../gpurun_out/r05c/probe_nohip.txt
timeout -k 10 60 ./exit_order_probe hip > ../gpurun_out/r05c/probe_hip.txt 2>&1; echo "rc=$?" >> ../gpurun_out/r05c/probe_hip.txt
