#!/bin/bash
# Round-4 call F: the whole GPU suite and smoke(), the doorbell trace and
# per-call bench, and bench lines B / C / D.  A step that times out, aborts
# or faults ends the script.  usage: scripts/r04_callF.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04l}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "step $name rc=$rc $(tail -1 $O/$name.log | cut -c1-200)"
  [ $rc -ge 124 ] && exit $rc
  return 0
}
step suite 600 python -u -m pytest tests -v --timeout 120 --timeout-method thread -m gpu
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
B="$R/oracle/_ref/cpubench $R/talos_amd/libtlsgpu.so"
for spec in "aes-128-gcm seal 1400 1 1" "aes-128-gcm seal 1400 8 1" "aes-128-gcm seal 1400 16 16" \
            "chacha20-poly1305 seal 1400 1 1"; do
  set -- $spec
  TLSGPU_EVP_DOORBELL=16 TLSGPU_EVP_DOORBELL_TRACE=1 timeout -k 10 60 $B $1 $2 $3 $4 $5 2 \
    >> $O/trace.jsonl 2>> $O/trace.err || exit $?
  echo "trace $spec: $(tail -2 $O/trace.err | tr '\n' ' ')"
done
step doorbell_bench 420 scripts/evp_doorbell_bench.sh "$O/doorbell_bench.jsonl"
for c in B C D; do
  step bench_$c 300 python bench.py --config $c --no-cpu-baseline
done
exit 0
