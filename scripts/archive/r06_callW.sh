#!/bin/bash
# round 6 call W: the wave-priority pass on the queue kernels as the default —
# GPU suite + smoke on it, then the driver's command alternating with the
# previous build (TLSGPU_LIBRARY=_variants/lib_nowp.so), three rounds, and D
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06w
mkdir -p $O
cd $R
bash scripts/gpu_suite.sh r06w/suite || { tail -30 $O/suite_tests.log; exit 1; }
tail -1 $O/suite_tests.log; tail -1 $O/suite_smoke.log
for k in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_B_$k.json 2> $O/bench_B_$k.err || exit $?
  TLSGPU_LIBRARY=$R/_variants/lib_nowp.so timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 \
    > $O/bench_B_nowp_$k.json 2> $O/bench_B_nowp_$k.err || exit $?
  python3 -c "import json; a=json.loads(open('$O/bench_B_$k.json').read().splitlines()[-1]); b=json.loads(open('$O/bench_B_nowp_$k.json').read().splitlines()[-1]); print('$k', 'wp', a['value'], 'nowp', b['value'])"
done
timeout -k 10 300 python bench.py --config D --steps 20 --warmup 5 > $O/bench_D.json 2> $O/bench_D.err || exit $?
cut -c1-160 $O/bench_D.json
