#!/usr/bin/env python3
"""Micro-benchmark of the bitsliced AES core alone (tlsgpu_aes_ecb_bitsliced):
blocks/s and the VALU-issue ceiling it implies for the CTR keystream."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import talos_amd as ta  # noqa: E402

eng = ta.Engine(0)
tab = ta.SessionTable(eng, 2)
tab.install(0, [ta.SessionParams(ta.AEAD_NAMES["aes-128-gcm"], bytes(range(16)), bytes(4)),
                ta.SessionParams(ta.AEAD_NAMES["aes-256-gcm"], bytes(range(32)), bytes(4))])
n = 64 << 20   # blocks (1 GiB)
d_in = ta.DeviceBuffer(eng, 16 * n)
d_out = ta.DeviceBuffer(eng, 16 * n)
eng.fill_synthetic(d_in.ptr, 0, 16 * n, 1, 7)
e0, e1 = ta.Event(eng), ta.Event(eng)
for sid, name in ((0, "aes-128"), (1, "aes-256")):
    ta.aes_ecb_bitsliced(tab, sid, d_in.ptr, d_out.ptr, n)
    eng.sync()
    e0.record()
    for _ in range(5):
        ta.aes_ecb_bitsliced(tab, sid, d_in.ptr, d_out.ptr, n)
    e1.record()
    eng.sync()
    ms = e0.elapsed_ms(e1) / 5
    print(f"{name} bitsliced ECB: {ms:.3f} ms per 1 GiB -> {16 * n / ms / 1e6:.1f} GB/s, "
          f"{n / ms / 1e6:.2f} Gblocks/s", flush=True)
