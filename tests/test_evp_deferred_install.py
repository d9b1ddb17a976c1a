"""Deferred session install for EVP contexts (round 5; VERDICT r04 next-round 6;
engine.cpp defer_install, evp_server.hip install / scrub ops).

With the doorbell on (the round-5 default), EVP_AEAD_CTX_init builds the
session image on the host (session_host.cpp: the key schedule, H and the GHASH
tables that aead_aes_gcm_init / CRYPTO_gcm128_init derive, e_aes.c:1372-1413,
gcm128.c:681-747) and launches nothing; the context's first call installs it —
inside its doorbell job, or with one upload kernel ahead of a launched job —
and EVP_AEAD_CTX_cleanup scrubs the slot through the server
(e_aes.c:1415-1422).  Every output is checked against the oracle:

* many threads making the FIRST call on one shared context at once (one
  installs, the others wait for it; EVP contexts may be used concurrently,
  evp.h:1273-1274);
* contexts initialised and cleaned up without any call (nothing reaches the
  device), then their slots reused by contexts that do call;
* more calling threads than doorbell slots (TLSGPU_EVP_DOORBELL=1: 8 slots),
  so some first calls install on the launched path;
* the slot reads back zero after cleanup (scrub job), and holds the key while
  the context lives.
"""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

_CHILD = r"""
import ctypes as C, faulthandler, os, random, sys, threading
faulthandler.enable()
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, os.path.join(sys.argv[1], "oracle"))
import talos_amd as ta, pyoracle as po
lib = ta.load_library()
lib.tlsgpu_session_image.restype = C.c_int
lib.tlsgpu_session_image.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
IMG = 1024 + 2048 + 65 * 256 + 15 * 512
orc = po.Oracle()
errors = []
def check(ctx, octx, rnd, kind):
    nonce = bytes(rnd.randrange(256) for _ in range(12))
    pt = bytes(rnd.randrange(256) for _ in range(rnd.choice([0, 1, 100, 1400, 5000])))
    ad = bytes(rnd.randrange(256) for _ in range(13))
    ok, exp = orc.seal(octx, nonce, pt, ad)
    ok2, got, _ = ctx.seal(nonce, pt, ad)
    assert ok == ok2 == 1 and got == exp, (kind, len(pt))
    ok3, back, _ = ctx.open(nonce, got, ad)
    assert ok3 == 1 and back == pt, ("open", kind, len(pt), ok3, threading.current_thread().name)
kinds = [po.AES_128_GCM, po.AES_256_GCM, po.CHACHA20_POLY1305]

# 1. concurrent first calls on one shared context
for kind in kinds:
    key = bytes(range(3, 3 + po.KEY_LEN[kind]))
    ctx, octx = ta.EvpAead(kind, key), orc.aead(kind, key)
    bar = threading.Barrier(8)
    def first(t):
        try:
            bar.wait()
            check(ctx, octx, random.Random(t), kind)
        except Exception as exc:
            errors.append(repr(exc))
    ths = [threading.Thread(target=first, args=(t,)) for t in range(8)]
    [t.start() for t in ths]; [t.join() for t in ths]
    assert not errors, errors[:2]
    t_, slot = C.c_void_p(), C.c_uint32()
    assert lib.tlsgpu_evp_context_slot(C.byref(ctx.ctx), C.byref(t_), C.byref(slot)) == 0
    buf = (C.c_uint8 * 2048)()
    assert lib.tlsgpu_sessions_debug_read(t_, slot.value, buf, 2048) == 0
    assert any(bytes(buf)), "installed slot reads zero"
    # round 6: the doorbell install builds the slot's Shoup tables on the
    # device from H^e; the slot must hold exactly the host image's bytes
    used = 1024 + (2048 + 65 * 256 if kind != po.CHACHA20_POLY1305 else 0)
    full = (C.c_uint8 * used)()
    assert lib.tlsgpu_sessions_debug_read(t_, slot.value, full, used) == 0
    img = (C.c_uint8 * IMG)()
    prm = ta.SessionParams(kind, key, b"", tag_len=16, version=0x0303).to_c()
    assert lib.tlsgpu_session_image(C.byref(prm), img, IMG) == 0
    assert bytes(full) == bytes(img)[:used], (kind, "doorbell-installed slot differs from the host image")
    ctx.cleanup()
    assert lib.tlsgpu_sessions_debug_read(t_, slot.value, buf, 2048) == 0
    assert not any(bytes(buf)), (kind, "key material left after cleanup")

# 2. init / cleanup without a call, slots then reused by calling contexts
rnd = random.Random(7)
idle = [ta.EvpAead(kinds[i % 3], bytes([i + 1]) * po.KEY_LEN[kinds[i % 3]]) for i in range(20)]
for c in idle:
    c.cleanup()
for i in range(20):
    kind = kinds[i % 3]
    key = bytes(rnd.randrange(256) for _ in range(po.KEY_LEN[kind]))
    c, oc = ta.EvpAead(kind, key), orc.aead(kind, key)
    check(c, oc, rnd, kind)
    c.cleanup()

# 2b. one thread (one slot, one server workgroup): a ChaCha install between two
#     calls of a GCM context must not leave the GCM context's session copy stale
for gk in kinds[:2]:
    g = ta.EvpAead(gk, bytes([0x5A]) * po.KEY_LEN[gk]); og = orc.aead(gk, bytes([0x5A]) * po.KEY_LEN[gk])
    check(g, og, rnd, gk)
    c = ta.EvpAead(kinds[2], bytes([0xA5]) * 32); oc = orc.aead(kinds[2], bytes([0xA5]) * 32)
    check(c, oc, rnd, kinds[2])
    check(g, og, rnd, gk)
    c.cleanup()
    check(g, og, rnd, gk)
    g.cleanup()

# 3. many threads cycling contexts (more threads than doorbell slots when
#    TLSGPU_EVP_DOORBELL=1)
def churn(t):
    r = random.Random(100 + t)
    try:
        for i in range(12):
            kind = kinds[(t + i) % 3]
            key = bytes(r.randrange(256) for _ in range(po.KEY_LEN[kind]))
            c, oc = ta.EvpAead(kind, key), orc.aead(kind, key)
            check(c, oc, r, kind)
            if i % 4 == 1:
                check(c, oc, r, kind)
            c.cleanup()
    except Exception as exc:
        errors.append(repr(exc))
ths = [threading.Thread(target=churn, args=(t,)) for t in range(int(sys.argv[2]))]
[t.start() for t in ths]; [t.join() for t in ths]
assert not errors, errors[:2]
j, l = ta.evp_doorbell_stats()
print("OK", j, l)
"""


@pytest.mark.parametrize("groups,threads", [("64", 8), ("1", 12)])
def test_deferred_install_and_doorbell_scrub(groups, threads):
    env = dict(os.environ, TLSGPU_EVP_DOORBELL=groups, TLSGPU_CRASH_TRACE="1")
    env.pop("TLSGPU_EVP_BATCH_US", None)
    r = subprocess.run([sys.executable, "-c", _CHILD, ROOT, str(threads)], env=env,
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
    jobs = int(r.stdout.split()[-2])
    assert jobs > 0, r.stdout


_CHILD_FAIL = r"""
import os, random, sys, threading, time
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, os.path.join(sys.argv[1], "oracle"))
import talos_amd as ta, pyoracle as po
orc = po.Oracle()
res, errors = [], []
for kind in (po.AES_128_GCM, po.CHACHA20_POLY1305):
    key = bytes(range(9, 9 + po.KEY_LEN[kind]))
    ctx, octx = ta.EvpAead(kind, key), orc.aead(kind, key)
    bar = threading.Barrier(8)
    def first(t):
        try:
            rnd = random.Random(t)
            nonce, pt, ad = rnd.randbytes(12), rnd.randbytes(1400), rnd.randbytes(13)
            bar.wait()
            ok, got, _ = ctx.seal(nonce, pt, ad)
            if ok:
                assert (1, got) == orc.seal(octx, nonce, pt, ad)[:2], kind
            res.append(ok)
        except Exception as exc:
            errors.append(repr(exc))
    t0 = time.time()
    ths = [threading.Thread(target=first, args=(t,)) for t in range(8)]
    [t.start() for t in ths]; [t.join() for t in ths]
    print("kind", kind, "calls", len(res), "ok", sum(res), "s", round(time.time() - t0, 2))
    ctx.cleanup()
assert not errors, errors[:2]
print("OK", sum(res), len(res))
"""


def test_failed_install_claim_is_retaken_by_waiters():
    """the call that claims a context's deferred install
    fails (test hook TLSGPU_TEST_FAIL_INSTALLS=1: the first claim only) while
    seven other first callers wait on it.  The waiters must take the install
    over at once — not spin until their 2^34-iteration cap — and every call
    but the failed one must return the oracle's bytes."""
    env = dict(os.environ, TLSGPU_EVP_DOORBELL="64", TLSGPU_TEST_FAIL_INSTALLS="1")
    env.pop("TLSGPU_EVP_BATCH_US", None)
    r = subprocess.run([sys.executable, "-c", _CHILD_FAIL, ROOT], env=env,
                       capture_output=True, text=True, timeout=90)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
    ok, calls = map(int, r.stdout.split()[-2:])
    assert calls == 16 and ok == 15, r.stdout       # exactly the one forced failure
