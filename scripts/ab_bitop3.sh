#!/bin/bash
# r03c: GPU parity, A/B of two library builds on config B, phase stats of D.
set -o pipefail
O=gpurun_out/r03c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 160 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  for v in old new; do
    if [ $v = old ]; then L=variants/libtlsgpu_perm.so; else L=talos_amd/libtlsgpu.so; fi
    TLSGPU_LIBRARY=$L timeout -k 10 120 python bench.py --no-cpu-baseline > $O/ab_${v}_$i.json 2> $O/ab_${v}_$i.err || exit 1
    echo "$v $i $(python -c "import json;print(json.load(open('$O/ab_${v}_$i.json'))['value'])")"
  done
done
TLSGPU_PHASE_STATS=1 timeout -k 10 300 python bench.py --config D --no-cpu-baseline --steps 10 > $O/phase_D.json 2> $O/phase_D.err || exit 1
grep phase $O/phase_D.err
exit 0
