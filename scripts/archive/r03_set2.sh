#!/bin/bash
# Round-3 GPU set 2: parity suite; same-box A/B of non-temporal output stores
# on config C (+ request-size PMC of both); PMC of the experimental bitsliced
# wave role (B16W = 4) on config B; EVP per-call / queue kernel profile; churn.
# usage: scripts/r03_set2.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -ne 0 ] && exit $rc
bash scripts/ab_bench.sh $TAG/ab_cc 3 "talos_amd/libtlsgpu.so variants/libtlsgpu_ccnt.so" --config C || exit 1
for lib in talos_amd/libtlsgpu.so variants/libtlsgpu_ccnt.so; do
  for grp in "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "WRITE_SIZE"; do
    (cd /tmp && TMPDIR=/tmp TLSGPU_LIBRARY=$R/$lib timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp \
      --output-format csv -d $O/cc_$(basename $lib .so)_${grp%%_sum*} -o pmc -- \
      python3 $R/bench.py --config C --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>&1) || exit 1
  done
done
echo "cc pmc done"
# bitsliced wave role: bench + PMC passes (kernel trace in the same runs)
TLSGPU_LIBRARY=$R/variants/libtlsgpu_exp.so TLSGPU_BS16_MIN=1024 timeout -k 10 300 python bench.py \
  --no-cpu-baseline > $O/bench_B_b16.json 2> $O/bench_B_b16.err || exit 1
echo "b16 bench $(cut -c1-120 $O/bench_B_b16.json)"
TLSGPU_LIBRARY=$R/variants/libtlsgpu_exp.so TLSGPU_BS16_MIN=1024 bash scripts/pmc.sh $TAG/pmcB_b16 || exit 1
bash scripts/evp_kernel_profile.sh $TAG/evp > $O/evp_profile.txt 2>&1 || exit 1
echo "evp profile done"
bash scripts/churn_bench.sh $O/churn.jsonl > /dev/null || exit 1
echo "churn done"
exit 0
