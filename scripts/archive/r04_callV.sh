#!/bin/bash
# Round-4 call V: bank-conflict-free GCM table load (load_session_tables):
# GCM / EVP / doorbell parity tests, then one-thread doorbell traces with a key
# change on every call and per-call A/B against ab/libtlsgpu_head.so.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04za}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_evp_doorbell.py tests/test_gpu_parity.py tests/test_evp_queue.py tests/test_evp_churn.py \
  > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for lib in ab/libtlsgpu_head.so talos_amd/libtlsgpu.so; do
  echo "== trace $lib"
  TLSGPU_EVP_DOORBELL=64 TLSGPU_EVP_DOORBELL_TRACE=1 timeout -k 10 60 oracle/_ref/cpubench $R/$lib \
    aes-128-gcm seal 1400 8 1 2 > $O/trace_1t.txt 2>&1 || exit 1
  grep doorbell $O/trace_1t.txt
done
: > $O/ab.jsonl
for r in 1 2; do
  for lib in ab/libtlsgpu_head.so talos_amd/libtlsgpu.so; do
    for t in 1 16; do
      TLSGPU_EVP_DOORBELL=64 timeout -k 10 60 oracle/_ref/cpubench $R/$lib aes-128-gcm seal 1400 $((t * 8)) $t 2 \
        | sed "s#^{#{\"lib\": \"$lib\", \"round\": $r, #" >> $O/ab.jsonl || exit 1
    done
    TLSGPU_EVP_DOORBELL=64 timeout -k 10 60 oracle/_ref/cpubench $R/$lib aes-256-gcm open 1400 8 1 2 \
      | sed "s#^{#{\"lib\": \"$lib\", \"round\": $r, #" >> $O/ab.jsonl || exit 1
  done
done
python3 - $O/ab.jsonl <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    j = json.loads(l)
    d[(j["lib"].split("/")[-1], j["aead"], j["op"], j["threads"])].append(round(j["records"] / j["seconds"]))
for k in sorted(d): print(k, d[k])
PY
exit 0
