#!/bin/bash
# round 5 call P: the final measurement set of the round (bench lines, PMC
# for B / C / D, kernel-trace stats), then per-call and churn rates with the
# default (doorbell on) settings beside the reference.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash scripts/measure_set.sh r05p > gpurun_out/r05p_measure.txt 2>&1 || exit $?
bash scripts/kstats.sh r05p/kstats > gpurun_out/r05p_kstats.txt 2>&1 || exit $?
OUT=gpurun_out/r05p/evp.jsonl; : > $OUT
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
