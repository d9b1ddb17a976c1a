"""Connection churn on the drop-in EVP surface:
EVP_AEAD_CTX_init does not wait for its device key install and
EVP_AEAD_CTX_cleanup does not wait for its scrub (round 3) — the slot's event
orders the install before the context's first call and the scrub before the
slot's next install.  Threads cycle init / seal / open / cleanup with a fresh
key every time, so slots are reused while scrubs and installs of other
threads are still queued; every output must equal the oracle's
(e_aes.c / e_chacha20poly1305.c semantics), per call and with the coalescing
queue."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

_CHILD = r"""
import os, random, sys, threading
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, os.path.join(sys.argv[1], "oracle"))
import talos_amd as ta, pyoracle as po
ta.load_library()
orc = po.Oracle()
kinds = [po.AES_128_GCM, po.AES_256_GCM, po.CHACHA20_POLY1305, po.CHACHA20_POLY1305_OLD]
errors = []
def worker(t):
    rnd = random.Random(900 + t)
    try:
        for i in range(40):
            kind = kinds[(t + i) % 4]
            key = bytes(rnd.randrange(256) for _ in range(po.KEY_LEN[kind]))
            ctx, octx = ta.EvpAead(kind, key), orc.aead(kind, key)
            assert ctx.ok == 1
            nlen = 8 if kind == po.CHACHA20_POLY1305_OLD else 12
            nonce = bytes(rnd.randrange(256) for _ in range(nlen))
            pt = bytes(rnd.randrange(256) for _ in range(rnd.choice([0, 1, 100, 1400])))
            ad = bytes(rnd.randrange(256) for _ in range(13))
            ok, exp = orc.seal(octx, nonce, pt, ad)
            ok2, got, ol = ctx.seal(nonce, pt, ad)
            assert ok == ok2 == 1 and got == exp and ol == len(exp), (t, i, kind)
            ok3, back, _ = ctx.open(nonce, got, ad)
            assert ok3 == 1 and back == pt, (t, i, kind)
            ctx.cleanup()
    except Exception as exc:
        errors.append(repr(exc))
# contexts created on one thread and cleaned up on another without any call:
# the scrub must not overtake the install queued on the creating thread's stream
handoff = []
def create(t):
    rnd = random.Random(700 + t)
    for i in range(30):
        kind = kinds[(t + i) % 4]
        c = ta.EvpAead(kind, bytes(rnd.randrange(256) for _ in range(po.KEY_LEN[kind])))
        assert c.ok == 1
        handoff.append(c)
ths = [threading.Thread(target=create, args=(t,)) for t in range(4)]
[th.start() for th in ths]; [th.join() for th in ths]
def destroy(part):
    for c in part:
        c.cleanup()
ths = [threading.Thread(target=destroy, args=(handoff[k::4],)) for k in range(4)]
[th.start() for th in ths]; [th.join() for th in ths]
ths = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
[th.start() for th in ths]; [th.join() for th in ths]
assert not errors, errors[:3]
print("OK")
"""


@pytest.mark.parametrize("batch_us", [None, "100"])
def test_evp_context_churn(batch_us):
    env = dict(os.environ)
    if batch_us:
        env["TLSGPU_EVP_BATCH_US"] = batch_us
    else:
        env.pop("TLSGPU_EVP_BATCH_US", None)
    r = subprocess.run([sys.executable, "-c", _CHILD, ROOT], env=env, capture_output=True,
                       text=True, timeout=150)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


_SCRUB_CHILD = r"""
import ctypes as C, os, sys
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, os.path.join(sys.argv[1], "oracle"))
import talos_amd as ta, pyoracle as po
lib = ta.load_library()
for kind in (po.AES_128_GCM, po.AES_256_GCM, po.CHACHA20_POLY1305):
    key = bytes(range(1, 1 + po.KEY_LEN[kind]))
    ctx = ta.EvpAead(kind, key)
    assert ctx.ok == 1
    ok, ct, _ = ctx.seal(bytes(12), b"x" * 100, b"")
    assert ok == 1
    t, slot = C.c_void_p(), C.c_uint32()
    assert lib.tlsgpu_evp_context_slot(C.byref(ctx.ctx), C.byref(t), C.byref(slot)) == 0
    n = 1024 + 4096
    live = (C.c_uint8 * n)()
    assert lib.tlsgpu_sessions_debug_read(t, slot.value, live, n) == 0
    assert any(bytes(live)), "installed slot reads all zero"
    ctx.cleanup()          # returns before the scrub has run on the device
    after = (C.c_uint8 * n)()
    assert lib.tlsgpu_sessions_debug_read(t, slot.value, after, n) == 0
    assert not any(bytes(after)), (kind, "key material left after cleanup")
print("SCRUBBED")
"""


def test_evp_cleanup_scrubs_device_key():
    """EVP_AEAD_CTX_cleanup's asynchronous scrub (explicit_bzero analogue,
    e_aes.c:1415-1422): once the slot's queued work has finished, the context's
    DevSession and GCM tables read back as zeros."""
    r = subprocess.run([sys.executable, "-c", _SCRUB_CHILD, ROOT], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0 and "SCRUBBED" in r.stdout, r.stdout + r.stderr
