#!/bin/bash
# round 5 call U: the draft ChaCha wave job MACs from the LDS stage — parity,
# then per-call rates.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05u
mkdir -p $O
cd $R
export TLSGPU_CRASH_TRACE=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_evp_chacha_old_wave.py tests/test_evp_doorbell.py tests/test_gpu_parity.py -k "old or doorbell or evp" \
  > $O/tests.log 2>&1 || exit $?
OUT=$O/percall.jsonl; : > $OUT
for t in 1 16 64; do
  for aead in chacha20-poly1305-old chacha20-poly1305; do
    timeout -k 10 60 oracle/_ref/cpubench talos_amd/libtlsgpu.so $aead seal 1400 $((t * 8)) $t 2 \
      | sed "s/^{/{\"lib\": \"libtlsgpu (default)\", /" >> $OUT || exit 1
    timeout -k 10 60 oracle/_ref/cpubench talos_amd/libtlsgpu.so $aead open 1400 $((t * 8)) $t 2 \
      | sed "s/^{/{\"lib\": \"libtlsgpu (default)\", /" >> $OUT || exit 1
  done
done
