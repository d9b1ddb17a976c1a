#!/bin/bash
# round 5 call AT: per-call and churn rates of the final build (default
# settings: doorbell on) beside the reference, as call P measured them
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/r05at
OUT=$R/gpurun_out/r05at/evp.jsonl; : > $OUT
cd $R
for aead in aes-128-gcm chacha20-poly1305 chacha20-poly1305-old; do
  for t in 1 16 64; do
    timeout -k 10 60 oracle/_ref/cpubench talos_amd/libtlsgpu.so $aead seal 1400 $((t * 8)) $t 2 \
      | sed "s/^{/{\"lib\": \"libtlsgpu (default)\", /" >> $OUT || exit 1
  done
done
for t in 1 16 64; do
  timeout -k 10 60 oracle/_ref/cpubench talos_amd/libtlsgpu.so aes-128-gcm init 1400 $t $t 2 \
    | sed "s/^{/{\"lib\": \"libtlsgpu (default)\", /" >> $OUT || exit 1
  timeout -k 10 60 oracle/_ref/cpubench oracle/_ref/libref.so aes-128-gcm init 1400 $t $t 2 \
    | sed "s/^{/{\"lib\": \"reference\", /" >> $OUT || exit 1
  timeout -k 10 60 oracle/_ref/cpubench oracle/_ref/libref.so aes-128-gcm seal 1400 $((t * 8)) $t 2 \
    | sed "s/^{/{\"lib\": \"reference\", /" >> $OUT || exit 1
done
