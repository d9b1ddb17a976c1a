#!/bin/bash
# Round-4 call D: doorbell latency breakdown (TLSGPU_EVP_DOORBELL_TRACE) and
# the config C occupancy A/B (TLSGPU_CC_LDS_PAD: 4 vs 3 waves per SIMD).
# usage: scripts/r04_callD.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04j}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
B="$R/oracle/_ref/cpubench $R/talos_amd/libtlsgpu.so"
for spec in "aes-128-gcm 1400 1 1" "aes-128-gcm 1400 8 1" "aes-128-gcm 1400 16 16" \
            "aes-128-gcm 16384 1 1" "chacha20-poly1305 1400 1 1" "chacha20-poly1305 1400 16 16"; do
  set -- $spec
  TLSGPU_EVP_DOORBELL=16 TLSGPU_EVP_DOORBELL_TRACE=1 timeout -k 10 60 $B $1 seal $2 $3 $4 2 \
    >> $O/trace.jsonl 2>> $O/trace.err || exit $?
  echo "trace $spec: $(tail -1 $O/trace.err)"
done
for r in 1 2; do
  for pad in 0 1024; do
    TLSGPU_CC_LDS_PAD=$pad timeout -k 10 300 python bench.py --config C --no-cpu-baseline \
      > $O/C_pad$pad.r$r.json 2> $O/C_pad$pad.r$r.err || exit $?
    echo "C pad=$pad r$r $(python3 -c 'import json,sys;d=json.load(open(sys.argv[1]));print(d["value"])' $O/C_pad$pad.r$r.json)"
  done
done
exit 0
