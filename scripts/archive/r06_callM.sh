#!/bin/bash
# round 6 call M: split session-run tails (TG_TAIL_SPLIT: a run's last
# records taken as two half-record claims) — the GPU suite on the variant,
# then a same-box A/B of 8 / 16 / 24 split records against the default on B,
# and B's phase stats with 16
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06m
mkdir -p $O
cd $R
TLSGPU_LIBRARY=$R/_variants/lib_ts16.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 \
  --timeout-method thread > $O/tests_ts16.log 2>&1 || { tail -30 $O/tests_ts16.log; exit 1; }
tail -2 $O/tests_ts16.log
bash scripts/ab_bench.sh r06m/abB 3 "talos_amd/libtlsgpu.so _variants/lib_ts8.so _variants/lib_ts16.so _variants/lib_ts24.so" > $O/abB.txt 2>&1 || exit $?
cat $O/abB.txt
TLSGPU_LIBRARY=$R/_variants/lib_ts16.so TLSGPU_PHASE_STATS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 \
  > $O/phase_ts16_B.json 2> $O/phase_ts16_B.txt || exit $?
grep phase $O/phase_ts16_B.txt
