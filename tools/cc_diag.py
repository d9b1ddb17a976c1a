"""Config C time split (diagnostic, not a benchmark): times the staged
ChaCha20-Poly1305 kernels' seal and open over config C's batch (1 Mi x 1,400-B
records, 4,096 sessions) with the TLSGPU_CC_DIAG bits the library read at
load (1 = no gather loads, 2 = no scatter stores, 4 = no ChaCha / Poly1305
work; chacha_kernels.hip) and the TLSGPU_CC_LDS_PAD occupancy knob.  Outputs
are not verified: with any bit set they are wrong by construction.
usage: TLSGPU_CC_DIAG=<bits> python tools/cc_diag.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import talos_amd as ta  # noqa: E402
from talos_amd.workload import Workload  # noqa: E402


def main():
    ta.load_library()
    eng = ta.Engine(0)
    kind = ta.AEAD_NAMES["chacha20-poly1305"]
    wl = Workload(eng, kind, 1 << 20, 4096, 0x5EED0002, record_len=1400)
    wl.table.hint(ta.batch_hints(wl.lengths, wl.session, seal=True))
    res = {"diag": os.environ.get("TLSGPU_CC_DIAG", "0"),
           "lds_pad": os.environ.get("TLSGPU_CC_LDS_PAD", "0")}
    for name, fn in (("seal", wl.seal), ("open", wl.open)):
        for _ in range(2):
            fn()
        eng.sync()
        e0, e1 = ta.Event(eng), ta.Event(eng)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        eng.sync()
        res[name + "_ms"] = round(e0.elapsed_ms(e1) / 10, 4)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
