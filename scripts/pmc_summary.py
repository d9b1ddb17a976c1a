#!/usr/bin/env python3
"""Summarise a scripts/pmc.sh run into profiles/pmc_<name>.json.

HBM traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE (KB) come from separate --pmc passes; on gfx950 FETCH_SIZE reports
half the bytes of a wide coalesced streaming read, so it is doubled.
usage: pmc_summary.py RUN_DIR KERNEL_PREFIX OUT_JSON [label]
"""
import collections
import csv
import glob
import json
import os
import sys

run, prefix, out = sys.argv[1], sys.argv[2], sys.argv[3]
label = sys.argv[4] if len(sys.argv) > 4 else ""
# LAST=N (round 5): only each pass's last N launches of the kernel — the timed
# steps of a warm-start bench run (the warm-up's launches ramp the clock)
last = int(os.environ.get("LAST", "0"))
vals = collections.defaultdict(list)
durs = []
for f in sorted(glob.glob(os.path.join(run, "pmc*", "pmc_counter_collection.csv"))):
    rows = [r for r in csv.DictReader(open(f)) if r["Kernel_Name"].startswith(prefix)]
    ids = sorted({int(r["Dispatch_Id"]) for r in rows})
    keep = set(ids[-last:]) if last else set(ids)
    for r in rows:
        if int(r["Dispatch_Id"]) in keep:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in sorted(glob.glob(os.path.join(run, "pmc*", "pmc_kernel_trace.csv"))):
    rows = sorted((r for r in csv.DictReader(open(f)) if r["Kernel_Name"].startswith(prefix)),
                  key=lambda r: int(r["Start_Timestamp"]))
    for r in (rows[-last:] if last else rows):
        durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
mean = {k: sum(v) / len(v) for k, v in vals.items()}
# the bench line each profiled pass printed (same process as its PMC and kernel trace)
bench = []
for f in sorted(glob.glob(os.path.join(run, "pmc*.log"))):
    for line in open(f):
        if line.startswith("{") and '"ms_per_step"' in line:
            d = json.loads(line)
            bench.append({"pass": os.path.basename(f), "value": d["value"],
                          "ms_per_step": d["ms_per_step"]})
res = {"kernel": prefix, "label": label, "launches_sampled": len(durs),
       "last_launches_per_pass": last or None,
       "mean_duration_ns_profiled": sum(durs) / len(durs) if durs else None,
       "counters_per_launch_mean": mean, "bench_lines_of_these_passes": bench}
if durs and bench:  # the main kernel must fit in the step it was timed in
    res["kernel_ms_le_step_ms"] = all(sum(durs) / len(durs) / 1e6 <= b["ms_per_step"] for b in bench)
if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
    res["hbm_read_bytes_per_launch"] = mean["FETCH_SIZE"] * 1024 * 2
    res["hbm_write_bytes_per_launch"] = mean["WRITE_SIZE"] * 1024
    res["hbm_bytes_per_launch"] = res["hbm_read_bytes_per_launch"] + res["hbm_write_bytes_per_launch"]
    res["correction"] = "FETCH_SIZE x2 (gfx950 half-count of wide streaming reads), KB x1024"
# calibrated read bytes: the L2's memory-side read requests by size (the
# FETCH_SIZE x2 rule holds for 128-B requests only; partial-line accesses
# issue 64-B and 32-B requests)
if "TCC_EA0_RDREQ_128B_sum" in mean and "TCC_EA0_RDREQ_64B_sum" in mean:
    rd = (128 * mean["TCC_EA0_RDREQ_128B_sum"] + 64 * mean["TCC_EA0_RDREQ_64B_sum"] +
          32 * mean.get("TCC_EA0_RDREQ_32B_sum", 0.0))
    res["hbm_read_bytes_per_launch_by_request_size"] = rd
    if "WRITE_SIZE" in mean:
        res["hbm_bytes_per_launch_by_request_size"] = rd + mean["WRITE_SIZE"] * 1024
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
