#!/bin/bash
# Connection churn: contexts/s of
# EVP_AEAD_CTX_init + one 1,400-B seal + EVP_AEAD_CTX_cleanup per connection
# direction, reference (oracle/_ref/libref.so, AES-NI) vs libtlsgpu per call
# and with the coalescing queue, at 1/16/64 threads.  usage: churn_bench.sh OUT.jsonl
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${1:-$R/gpurun_out/churn.jsonl}
: > "$OUT"
for t in 1 16 64; do
  timeout -k 10 60 "$R/oracle/_ref/cpubench" "$R/oracle/_ref/libref.so" aes-128-gcm init 1400 $t $t 2 \
    | sed "s/^{/{\"lib\": \"reference\", /" >> "$OUT" || exit 1
  TLSGPU_EVP_DOORBELL=0 timeout -k 10 60 "$R/oracle/_ref/cpubench" "$R/talos_amd/libtlsgpu.so" aes-128-gcm init 1400 $t $t 2 \
    | sed "s/^{/{\"lib\": \"libtlsgpu per call\", /" >> "$OUT" || exit 1
  TLSGPU_EVP_BATCH_US=50 timeout -k 10 60 "$R/oracle/_ref/cpubench" "$R/talos_amd/libtlsgpu.so" aes-128-gcm init 1400 $t $t 2 \
    | sed "s/^{/{\"lib\": \"libtlsgpu queue 50us\", /" >> "$OUT" || exit 1
done
cat "$OUT"
