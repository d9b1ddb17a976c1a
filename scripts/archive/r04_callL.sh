#!/bin/bash
# Round-4 call L: doorbell yield threshold A/B (64 / 16 / 1 threads, 1,400 B).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04q}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
B="$R/oracle/_ref/cpubench $R/talos_amd/libtlsgpu.so"
for r in 1 2; do
  for y in 100 20 5 0; do
    for t in 64 16 1; do
      TLSGPU_EVP_DOORBELL=64 TLSGPU_EVP_DOORBELL_YIELD_US=$y timeout -k 10 60 $B aes-128-gcm seal 1400 $((t * 8)) $t 2 \
        | sed "s/^{/{\"yield_us\": $y, \"round\": $r, /" >> $O/yield.jsonl || exit $?
    done
  done
done
python3 - "$O/yield.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["round"], "yield", d["yield_us"], "T", d["threads"], round(d["records"] / d["seconds"] / 1e3, 1), "K/s fail", d["failures"])
PY
exit 0
