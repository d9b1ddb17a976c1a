#!/usr/bin/env python3
"""EVP drop-in throughput: T threads x M EVP_AEAD_CTX_seal calls of L bytes
(AES-128-GCM), per-call path vs the coalescing queue (--batch-us > 0).
Prints one JSON line.  usage: evp_bench.py [--threads T] [--calls M] [--len L] [--batch-us W]"""
import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import talos_amd as ta  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--threads", type=int, default=16)
ap.add_argument("--calls", type=int, default=200)
ap.add_argument("--len", type=int, default=1400)
ap.add_argument("--batch-us", type=int, default=0)
args = ap.parse_args()
ta.load_library()
if args.batch_us:
    ta.evp_set_batching(args.batch_us, 0, 256)
ctxs = [ta.EvpAead(ta.AES_128_GCM, bytes([t]) * 16) for t in range(args.threads)]
pt, ad = bytes(args.len), bytes(13)
for c in ctxs:  # warm-up (engine, kernels, staging)
    c.seal(bytes(12), pt, ad)
barrier = threading.Barrier(args.threads + 1)


def worker(c):
    barrier.wait()
    for i in range(args.calls):
        ok, _, _ = c.seal(i.to_bytes(12, "little"), pt, ad)
        assert ok == 1


ths = [threading.Thread(target=worker, args=(c,)) for c in ctxs]
for t in ths:
    t.start()
barrier.wait()
t0 = time.perf_counter()
for t in ths:
    t.join()
dt = time.perf_counter() - t0
calls = args.threads * args.calls
b, j = ta.evp_batch_stats()
print(json.dumps({"metric": "EVP_AEAD_CTX_seal calls/s (AES-128-GCM, drop-in ABI)",
                  "threads": args.threads, "len": args.len, "batch_us": args.batch_us,
                  "calls_per_s": round(calls / dt, 1), "gib_per_s": round(calls * args.len / dt / 2**30, 4),
                  "batches": b, "jobs": j}))
