"""The drop-in EVP surface spread over several GPUs (SURVEY.md §8e for the
per-call path and the coalescing queue).

EVP_AEAD_CTX_init hands new contexts to the EVP devices in turn; each device
has its own engine, call streams and (batching on) queue and session pool.  On
a one-GPU box TLSGPU_DEVICES=0,0 makes two EVP devices of device 0 — two
engines, two queues — which runs exactly the code of two GPUs.  Every call is
checked against the oracle (evp_aead.c / e_aes.c / e_chacha20poly1305.c
semantics: outputs, return values, zero-fill on a bad tag), and the per-device
counters must show both devices serving contexts and calls.
"""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

_CHILD = r"""
import faulthandler; faulthandler.enable()
import os, random, sys, threading
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, os.path.join(sys.argv[1], "oracle"))
import talos_amd as ta, pyoracle as po
ta.load_library()
orc = po.Oracle()
kinds = [po.AES_128_GCM, po.AES_256_GCM, po.CHACHA20_POLY1305, po.CHACHA20_POLY1305_OLD]
errors = []
def worker(t):
    rnd = random.Random(500 + t)
    kind = kinds[t % 4]
    key = bytes(rnd.randrange(256) for _ in range(po.KEY_LEN[kind]))
    ctx, octx = ta.EvpAead(kind, key), orc.aead(kind, key)
    nlen = 8 if kind == po.CHACHA20_POLY1305_OLD else 12
    try:
        assert ctx.ok == 1
        for i in range(10):
            nonce = bytes(rnd.randrange(256) for _ in range(nlen))
            pt = bytes(rnd.randrange(256) for _ in range(rnd.choice([0, 1, 16, 100, 1400, 5000])))
            ad = bytes(rnd.randrange(256) for _ in range(rnd.choice([0, 13, 40])))
            ok, exp = orc.seal(octx, nonce, pt, ad)
            ok2, got, ol = ctx.seal(nonce, pt, ad)
            assert ok == ok2 == 1 and got == exp and ol == len(exp), (t, i)
            ok3, back, _ = ctx.open(nonce, got, ad)
            assert ok3 == 1 and back == pt, (t, i)
            if got:
                bad = bytearray(got); bad[rnd.randrange(len(bad))] ^= 2
                ok4, z, ol4 = ctx.open(nonce, bytes(bad), ad)
                assert ok4 == 0 and z == bytes(len(bad)) and ol4 == 0, (t, i)
    except Exception as exc:
        errors.append(repr(exc))
    finally:
        ctx.cleanup()
ths = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
[th.start() for th in ths]; [th.join() for th in ths]
assert not errors, errors[:3]
st = ta.evp_device_stats()
assert len(st) == 2 and all(d == 0 for d, _, _ in st), st
assert all(c == 4 for _, c, _ in st), st            # 8 contexts dealt round-robin
assert all(n >= 4 * 10 * 2 for _, _, n in st), st   # every device served its contexts' calls
b, j = ta.evp_batch_stats()
print("OK", st, b, j)
"""


@pytest.mark.parametrize("batch_us", [None, "200"])
def test_evp_two_devices(batch_us):
    env = dict(os.environ, TLSGPU_DEVICES="0,0", TLSGPU_CRASH_TRACE="1")
    env.pop("TLSGPU_DEVICE", None)
    if batch_us:
        env["TLSGPU_EVP_BATCH_US"] = batch_us
    else:
        env.pop("TLSGPU_EVP_BATCH_US", None)
    r = subprocess.run([sys.executable, "-c", _CHILD, ROOT], env=env, capture_output=True,
                       text=True, timeout=150)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
    if batch_us:
        jobs = int(r.stdout.split()[-1])
        assert jobs > 0, r.stdout    # the calls went through the two queues
