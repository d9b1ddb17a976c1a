#!/bin/bash
# Round-4 call U: the slot input area (a short job's input read with its
# slot): doorbell tests, then per-call A/B against the previous library
# (ab/libtlsgpu_head.so), AES-128-GCM seal / open 1,400 B, 1 / 16 / 64
# threads, doorbell=64, two alternating rounds; one trace run at 1 thread.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04z}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_evp_doorbell.py > $O/doorbell_tests.txt 2>&1 || { tail -30 $O/doorbell_tests.txt; exit 1; }
tail -3 $O/doorbell_tests.txt
: > $O/ab.jsonl
for r in 1 2; do
  for lib in ab/libtlsgpu_head.so ab/libtlsgpu_pre2k.so talos_amd/libtlsgpu.so; do
    for op in seal open; do
      for t in 1 16 64; do
        TLSGPU_EVP_DOORBELL=64 timeout -k 10 60 oracle/_ref/cpubench $R/$lib aes-128-gcm $op 1400 $((t * 8)) $t 2 \
          | sed "s#^{#{\"lib\": \"$lib\", \"round\": $r, #" >> $O/ab.jsonl || exit 1
      done
    done
  done
done
python3 - $O/ab.jsonl <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    j = json.loads(l)
    k = (j["lib"].split("/")[-1], j["op"], j["threads"])
    d[k].append(round(j["records"] / j["seconds"]))
for k in sorted(d): print(k, d[k])
PY
for lib in ab/libtlsgpu_head.so ab/libtlsgpu_pre2k.so talos_amd/libtlsgpu.so; do
  echo "== trace $lib"
  TLSGPU_EVP_DOORBELL=64 TLSGPU_EVP_DOORBELL_TRACE=1 timeout -k 10 60 oracle/_ref/cpubench $R/$lib \
    aes-128-gcm seal 1400 8 1 2 > $O/trace_1t.txt 2>&1 || exit 1
  grep doorbell $O/trace_1t.txt
done
exit 0
