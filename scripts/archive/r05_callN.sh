#!/bin/bash
# round 5 call N: the draft ChaCha20-Poly1305 AEAD on one wave (doorbell op 21,
# launched one-wave kernel) — parity, then per-call rates for it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05n
mkdir -p $O
cd $R
export TLSGPU_CRASH_TRACE=1
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_evp_chacha_old_wave.py tests/test_evp_doorbell.py tests/test_evp_deferred_install.py \
  tests/test_gpu_parity.py -k "evp or old or doorbell or deferred" > $O/tests.log 2>&1 || exit $?
OUT=$O/percall.jsonl; : > $OUT
for t in 1 16; do
  for db in 64 0; do
    TLSGPU_EVP_DOORBELL=$db timeout -k 10 60 oracle/_ref/cpubench talos_amd/libtlsgpu.so \
      chacha20-poly1305-old seal 1400 $((t * 8)) $t 2 | sed "s/^{/{\"lib\": \"libtlsgpu doorbell=$db\", /" >> $OUT || exit 1
  done
done
