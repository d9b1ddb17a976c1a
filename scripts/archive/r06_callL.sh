#!/bin/bash
# round 6 call L: where config B's session-run boundaries go (phase stats at
# S = 1,024 and S = 1, and D), then a same-box A/B of the run-boundary table
# prefetch (TG_RUN_PREFETCH: the next session's GHASH tables fetched into
# registers before the run-start barrier) on B and D, and the GPU suite on it
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06l
mkdir -p $O
cd $R
for lib in talos_amd/libtlsgpu.so _variants/lib_pf.so; do
  n=$(basename $lib .so)
  for cfg in "B" "B --sessions 1" "D"; do
    t=$(echo $cfg | tr -d ' -')
    TLSGPU_LIBRARY=$R/$lib TLSGPU_PHASE_STATS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 \
      --config $cfg > $O/phase_${n}_$t.json 2> $O/phase_${n}_$t.txt || exit $?
  done
done
grep -h "phase" $O/phase_*.txt | head -0
bash scripts/ab_bench.sh r06l/abB 3 "talos_amd/libtlsgpu.so _variants/lib_pf.so" > $O/abB.txt 2>&1 || exit $?
cat $O/abB.txt
bash scripts/ab_bench.sh r06l/abD 3 "talos_amd/libtlsgpu.so _variants/lib_pf.so" --config D > $O/abD.txt 2>&1 || exit $?
cat $O/abD.txt
TLSGPU_LIBRARY=$R/_variants/lib_pf.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 \
  --timeout-method thread > $O/tests_pf.log 2>&1 || exit $?
tail -2 $O/tests_pf.log
