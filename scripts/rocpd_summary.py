"""Per-kernel duration summary of rocprofv3 rocpd databases (run_results.db):
name, launches, average and median microseconds.  usage: rocpd_summary.py DB..."""
import collections
import sqlite3
import sys

for f in sys.argv[1:]:
    c = sqlite3.connect(f)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    ni = cols.index("name") if "name" in cols else cols.index("kernel_name")
    si, ei = cols.index("start"), cols.index("end")
    d = collections.defaultdict(list)
    for r in c.execute("select * from kernels"):
        d[r[ni][:80]].append((r[ei] - r[si]) / 1e3)
    print(f)
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        v.sort()
        print(f"  {k:80s} n={len(v):6d} avg={sum(v) / len(v):8.1f}us med={v[len(v) // 2]:8.1f}us")
