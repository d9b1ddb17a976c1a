#!/usr/bin/env python3
"""Print mean per-launch PMC counters per kernel from a pmc_quick.sh run dir."""
import collections, csv, glob, os, sys
run = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
durs = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(run, "pmc*", "pmc_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        vals[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in sorted(glob.glob(os.path.join(run, "pmc*", "pmc_kernel_trace.csv"))):
    for r in csv.DictReader(open(f)):
        durs[r["Kernel_Name"][:60]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, d in vals.items():
    ds = durs.get(k, [])
    print(k, "launches", len(ds), "mean_ns", sum(ds) / max(1, len(ds)))
    for c, v in sorted(d.items()):
        print(f"   {c:24s} {sum(v)/len(v):16.1f}")
