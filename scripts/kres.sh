#!/bin/bash
# Print VGPRs / VGPR spills / occupancy per kernel of the given HIP sources.
# usage: scripts/kres.sh [extra hipcc flags] -- file.hip ...
flags=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do flags+=("$1"); shift; done; shift
for f in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result "${flags[@]}" \
    -c "$f" -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  awk '/Function Name:/{n=$NF=="[-Rpass-analysis=kernel-resource-usage]"?$(NF-1):$NF}
       / VGPRs: /{v=$(NF-1)} /Occupancy/{o=$(NF-1)} /VGPRs Spill:/{print n, "vgpr=" v, "spill=" $(NF-1), "occ=" o}'
done
