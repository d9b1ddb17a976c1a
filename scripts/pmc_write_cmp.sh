set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmcw; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
for im in ttable queue; do
  TLSGPU_GCM_IMPL=$im timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/$im -o pmc -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/$im.log 2>&1 || exit 1
done
