#!/bin/bash
# Per-call EVP rate, launched path vs the doorbell server (round 4):
# AES-128-GCM (and ChaCha20-Poly1305 at 1,400 B) seal through oracle/_ref/cpubench dlopen()ing libtlsgpu.so,
# 1,400 B and 16 KiB, 1 / 16 / 64 threads; plus connection churn (init).
# usage: scripts/evp_doorbell_bench.sh OUT.jsonl
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${1:-$R/gpurun_out/evp_doorbell.jsonl}
: > "$OUT"
for len in 1400 16384; do
  for t in 1 16 64; do
    n=$((t * 8))
    TLSGPU_EVP_DOORBELL=0 TLSGPU_EVP_SPIN=1 timeout -k 10 60 "$R/oracle/_ref/cpubench" "$R/talos_amd/libtlsgpu.so" \
      aes-128-gcm seal $len $n $t 2 | sed "s/^{/{\"lib\": \"libtlsgpu per call launch+eventspin\", /" >> "$OUT" || exit 1
    for db in 0 16 64; do
      TLSGPU_EVP_DOORBELL=$db timeout -k 10 60 "$R/oracle/_ref/cpubench" "$R/talos_amd/libtlsgpu.so" \
        aes-128-gcm seal $len $n $t 2 | sed "s/^{/{\"lib\": \"libtlsgpu per call doorbell=$db\", /" >> "$OUT" || exit 1
    done
  done
done
for t in 1 16; do
  TLSGPU_EVP_DOORBELL=0 TLSGPU_EVP_SPIN=1 timeout -k 10 60 "$R/oracle/_ref/cpubench" "$R/talos_amd/libtlsgpu.so" \
    chacha20-poly1305 seal 1400 $((t * 8)) $t 2 | sed "s/^{/{\"lib\": \"libtlsgpu per call launch+eventspin\", /" >> "$OUT" || exit 1
  for db in 0 16; do
    TLSGPU_EVP_DOORBELL=$db timeout -k 10 60 "$R/oracle/_ref/cpubench" "$R/talos_amd/libtlsgpu.so" \
      chacha20-poly1305 seal 1400 $((t * 8)) $t 2 | sed "s/^{/{\"lib\": \"libtlsgpu per call doorbell=$db\", /" >> "$OUT" || exit 1
  done
done
for t in 1 16; do
  for db in 0 16; do
    TLSGPU_EVP_DOORBELL=$db timeout -k 10 60 "$R/oracle/_ref/cpubench" "$R/talos_amd/libtlsgpu.so" \
      aes-128-gcm init 1400 $t $t 2 | sed "s/^{/{\"lib\": \"libtlsgpu churn doorbell=$db\", /" >> "$OUT" || exit 1
  done
done
