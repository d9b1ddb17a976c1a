#!/bin/bash
# EVP per-call path: staged through HBM (TLSGPU_EVP_ZEROCOPY=0) vs zero-copy
# (default), AES-128-GCM seal, 1 / 16 / 64 threads, 1,400 B and 16 KiB.
# usage: scripts/evp_percall_ab.sh OUT.jsonl
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${1:-$R/gpurun_out/evp_percall.jsonl}
: > "$OUT"
for len in 1400 16384; do
  for t in 1 16 64; do
    n=$((t * 8))
    for zc in 0 1; do
      TLSGPU_EVP_DOORBELL=0 TLSGPU_EVP_ZEROCOPY=$zc timeout -k 10 60 "$R/oracle/_ref/cpubench" "$R/talos_amd/libtlsgpu.so" \
        aes-128-gcm seal $len $n $t 2 | sed "s/^{/{\"lib\": \"libtlsgpu per call zerocopy=$zc\", /" >> "$OUT" || exit 1
      [ -n "$QUEUE" ] && { TLSGPU_EVP_BATCH_US=50 TLSGPU_EVP_ZEROCOPY=$zc timeout -k 10 60 "$R/oracle/_ref/cpubench" \
        "$R/talos_amd/libtlsgpu.so" aes-128-gcm seal $len $n $t 2 \
        | sed "s/^{/{\"lib\": \"libtlsgpu queue 50us zerocopy=$zc\", /" >> "$OUT" || exit 1; }
    done
  done
done
python3 -c "
import json
for l in open('$OUT'):
    d=json.loads(l); print(d['lib'], d['rec_len'], d['threads'], round(d['records']/d['seconds']), 'calls/s', d['gib_per_s'], 'GiB/s')"
