"""Per-workgroup timing of the queue kernel on a bench config (diagnostic).

Runs config D's (or another config's) open batch with TLSGPU_WG_TIMES=1 and
prints, per launch, the kernel span, the spread of workgroup start / end
times, and how each workgroup's duration follows its bytes and records —
whether the batch's equal-count (or work-balanced, TLSGPU_BALANCE) ranges
leave the slowest CU with more work than the others.
usage: TLSGPU_WG_TIMES=1 python tools/wg_times.py [--config D] [--launches 3]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="D")
    ap.add_argument("--launches", type=int, default=3)
    ap.add_argument("--records", type=int, default=0, help="override the config's records")
    ap.add_argument("--sustained", type=int, default=0,
                    help="launch this many batches back to back before each timed one")
    args = ap.parse_args()
    os.environ.setdefault("TLSGPU_WG_TIMES", "1")
    import bench
    import talos_amd as ta
    from talos_amd.workload import Workload, zipf_lengths
    kind_name, per_gpu, sessions, rec_len, seed, op = bench.CONFIGS[args.config]
    if args.records:
        sessions = max(1, sessions * args.records // per_gpu)
        per_gpu = args.records
    ta.load_library()
    eng = ta.Engine(0)
    kind = ta.AEAD_NAMES[kind_name]
    lengths = None if rec_len else zipf_lengths(per_gpu, seed)
    wl = Workload(eng, kind, per_gpu, sessions, seed, lengths=lengths, record_len=rec_len or 0,
                  tamper_every=1024)
    desc_len = wl.lengths + ta.EXPLICIT_NONCE_LEN[kind] + ta.TAG_LEN
    wl.table.hint(ta.batch_hints(desc_len, wl.session, seal=False))
    groups = eng.num_cus                  # engine.cpp groups_for
    if groups * 16 > per_gpu:
        groups = (per_gpu + 15) // 16
    rpg = (per_gpu + groups - 1) // groups
    groups = (per_gpu + rpg - 1) // rpg
    wl.open(None)
    eng.sync()
    for it in range(args.launches):
        for _ in range(args.sustained):   # the timed launch then follows without a gap
            wl.open(None)
        wl.open(None)
        eng.sync()
        t = np.array(ta.debug_wg_times(eng, groups), dtype=np.int64)
        st, en, recs, work = t[:, 0], t[:, 1], t[:, 2].astype(np.float64), t[:, 3]
        dur = (en - st) / 100.0          # us
        nbytes = (work - 256 * recs).astype(np.float64)   # work = bytes + 256 per record
        runs = np.zeros(len(st))
        span = (en.max() - st.min()) / 100.0
        out = {
            "launch": it, "records": per_gpu, "sustained": args.sustained, "balance": os.environ.get("TLSGPU_BALANCE", "default"), "pieces": os.environ.get("TLSGPU_PIECES", "0"),
            "span_us": round(span, 1),
            "start_spread_us": round((st.max() - st.min()) / 100.0, 1),
            "end_spread_us": round((en.max() - en.min()) / 100.0, 1),
            "dur_us": {"mean": round(dur.mean(), 1), "max": round(dur.max(), 1), "min": round(dur.min(), 1)},
            "bytes_max_over_mean": round(nbytes.max() / nbytes.mean(), 3),
            "dur_max_over_mean": round(dur.max() / dur.mean(), 3),
            "corr_dur_bytes": round(float(np.corrcoef(dur, nbytes)[0, 1]), 3),
            "corr_dur_records": round(float(np.corrcoef(dur, recs)[0, 1]), 3),
            "records_per_group": {"mean": round(recs.mean(), 1), "max": int(recs.max())},
            # ns per byte from a least-squares fit dur = a + b * bytes + c * runs
        }
        A = np.stack([np.ones_like(dur), nbytes, recs], 1)
        coef, *_ = np.linalg.lstsq(A, dur, rcond=None)
        out["fit_us"] = {"const": round(coef[0], 1), "per_MiB": round(coef[1] * (1 << 20), 1),
                         "per_record": round(coef[2], 3)}
        print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
