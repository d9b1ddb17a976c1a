set -o pipefail
bash scripts/ab_bench.sh r03h 3 "talos_amd/libtlsgpu.so variants/libtlsgpu_ccnt.so" --config C || exit 1
cd /tmp && export TMPDIR=/tmp
for lib in talos_amd/libtlsgpu.so variants/libtlsgpu_ccnt.so; do
  for grp in "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "WRITE_SIZE"; do
    TLSGPU_LIBRARY=$GRAFT_REPO_ROOT/$lib timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r03h/p_$(basename $lib .so)_${grp%%_sum*} -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py --config C --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>&1 || exit 1
  done
done
echo done
