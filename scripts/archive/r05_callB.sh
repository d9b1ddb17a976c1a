#!/bin/bash
# round 5 call B: shutdown-contract tests + exit-order probe (call A), then the
# ChaCha write-aligned windows: parity under the aligned library, C digest,
# and a same-box A/B of C (base vs aligned vs aligned-with-TLSGPU_CC_ALIGN=0).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05b
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread \
  tests/test_evp_shutdown.py tests/test_evp_doorbell.py tests/test_evp_multi_device.py > $O/tests_shutdown.log 2>&1 || exit $?
TLSGPU_LIBRARY=$R/_variants/lib_cc_align.so timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread \
  tests/test_gpu_batch_digests.py tests/test_gpu_parity.py tests/test_wire.py tests/test_seal_wire.py tests/test_wire_reference.py \
  -k "chacha or C or CHACHA or wire" > $O/tests_cc.log 2>&1 || exit $?
for k in 1 2 3; do
  for v in base align align0; do
    lib=_variants/lib_cc_$v.so; env=""
    [ $v = align0 ] && lib=_variants/lib_cc_align.so && env="TLSGPU_CC_ALIGN=0"
    env $env TLSGPU_LIBRARY=$R/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --config C > $O/ab.json 2>$O/ab.err || exit 1
    echo "$k $v $(python3 -c "import json; d=json.loads(open('$O/ab.json').read().splitlines()[-1]); print(d['value'], d['ms_per_step'])")" >> $O/ab.txt
  done
done
cd tools
timeout -k 10 60 ./exit_order_probe nohip > ../gpurun_out/r05b/probe_nohip.txt 2>&1; echo "rc=$?" >> ../gpurun_out/r05b/probe_nohip.txt
timeout -k 10 60 ./exit_order_probe hip > ../gpurun_out/r05b/probe_hip.txt 2>&1; echo "rc=$?" >> ../gpurun_out/r05b/probe_hip.txt
