"""The doorbell server for per-call EVP jobs (round 4, talos_amd/csrc/evp_server.hip,
include/tlsgpu.h tlsgpu_evp_set_doorbell): with TLSGPU_EVP_DOORBELL set, a
synchronous EVP_AEAD_CTX_seal / _open on an AES-GCM or RFC 7539
ChaCha20-Poly1305 context is posted to a resident server workgroup instead of
launching a kernel.  Every output must
be the oracle's (e_aes.c:1424-1510 through evp_aead.c:89-144: tag, zero-fill
and return 0 on a bad tag, odd nonce lengths, truncated tags), with threads
cycling init / seal / open / cleanup so session slots are re-keyed while the
server runs, across server relaunches (short lifetime), and the server must
stop by itself when the calls stop.  ChaCha jobs (RFC 7539, and since round
5 the draft suite) run on the server's wave 0 (chacha_wave.h) between GCM
jobs, whose LDS table cache they must leave intact.  A GCM job's input up to 4 KiB is staged into LDS by the server's
idle waves 12-15 while waves 0-1 parse: the lengths cover both sides of that
limit for seal (4,096 B of plaintext) and open (4,080 + 16 B of ciphertext
and tag)."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

_CHILD = r"""
import faulthandler; faulthandler.enable()
import os, random, sys, threading, time
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, os.path.join(sys.argv[1], "oracle"))
import talos_amd as ta, pyoracle as po
ta.load_library()
orc = po.Oracle()
kinds = [po.AES_128_GCM, po.AES_256_GCM, po.CHACHA20_POLY1305, po.CHACHA20_POLY1305_OLD]
errors = []
def worker(t):
    rnd = random.Random(4100 + t)
    try:
        for i in range(int(os.environ.get("TLSGPU_SOAK_ITERS", "30"))):
            kind = kinds[(t + i) % len(kinds)]
            key = bytes(rnd.randrange(256) for _ in range(po.KEY_LEN[kind]))
            chacha = kind in (po.CHACHA20_POLY1305, po.CHACHA20_POLY1305_OLD)
            tag_len = rnd.choice([16, 16, 12]) if not chacha else 16
            ctx, octx = ta.EvpAead(kind, key, tag_len), orc.aead(kind, key, tag_len)
            assert ctx.ok == 1
            for _ in range(3):
                nlen = (12 if kind == po.CHACHA20_POLY1305 else 8 if kind == po.CHACHA20_POLY1305_OLD
                        else rnd.choice([12, 12, 1, 8, 16, 60]))
                nonce = bytes(rnd.randrange(256) for _ in range(nlen))
                pt = bytes(rnd.randrange(256) for _ in range(rnd.choice([0, 1, 15, 100, 1400, 4080, 4081, 4096, 16384, 40000])))
                ad = bytes(rnd.randrange(256) for _ in range(rnd.choice([0, 13, 100])))
                ok, exp = orc.seal(octx, nonce, pt, ad)
                ok2, got, ol = ctx.seal(nonce, pt, ad)
                assert ok == ok2 == 1 and got == exp and ol == len(exp), (t, i, kind, len(pt))
                ok3, back, _ = ctx.open(nonce, got, ad)
                assert ok3 == 1 and back == pt, (t, i, kind, len(pt))
                if got:
                    bad = bytearray(got); bad[rnd.randrange(len(bad))] ^= 1 << rnd.randrange(8)
                    ok4, z, _ = ctx.open(nonce, bytes(bad), ad)
                    assert ok4 == 0 and not any(z), (t, i, "tampered record accepted or not zero-filled")
            ctx.cleanup()
            if i % 7 == 3:
                time.sleep(0.03)   # past half a lifetime: the next call relaunches the server
    except Exception as exc:
        errors.append(repr(exc))
ths = [threading.Thread(target=worker, args=(t,)) for t in range(int(sys.argv[2]))]
[th.start() for th in ths]; [th.join() for th in ths]
assert not errors, errors[:3]
jobs, launches = ta.evp_doorbell_stats()
assert jobs > 0 and launches >= 2, (jobs, launches)
time.sleep(0.2)   # every instance has passed its lifetime: none may still be running
print("OK", jobs, launches)
"""


@pytest.mark.parametrize("threads", [1, 12])
def test_evp_doorbell_matches_oracle(threads):
    """TLSGPU_SOAK_ITERS=N: N contexts per thread instead of 30 (a soak run;
    profiles/r06*_soak_doorbell*)."""
    env = dict(os.environ, TLSGPU_EVP_DOORBELL="4", TLSGPU_EVP_DOORBELL_MS="40", TLSGPU_CRASH_TRACE="1")
    env.pop("TLSGPU_EVP_BATCH_US", None)
    iters = int(os.environ.get("TLSGPU_SOAK_ITERS", "30"))
    r = subprocess.run([sys.executable, "-c", _CHILD, ROOT, str(threads)], env=env,
                       capture_output=True, text=True, timeout=110 + iters * 3)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


_BUSY_CHILD = r"""
import faulthandler; faulthandler.enable()
import os, sys, threading, time
sys.path.insert(0, sys.argv[1])
import talos_amd as ta
ta.load_library()
stop = threading.Event()
lat = []
def busy():   # keeps its own server workgroup busy far past the 20 ms lifetime
    ctx = ta.EvpAead(ta.AES_128_GCM, bytes(16))
    while not stop.is_set():
        ok, out, _ = ctx.seal(bytes(12), b"x" * 1400, b"")
        assert ok == 1
    ctx.cleanup()
def late():   # starts after the first instance's lifetime has passed
    time.sleep(0.1)
    ctx = ta.EvpAead(ta.AES_256_GCM, bytes(32))
    for _ in range(20):
        t = time.perf_counter()
        ok, out, _ = ctx.seal(bytes(12), b"y" * 100, b"")
        lat.append(time.perf_counter() - t)
        assert ok == 1
    ctx.cleanup()
a, b = threading.Thread(target=busy), threading.Thread(target=late)
a.start(); b.start(); b.join(); stop.set(); a.join()
print("OK", max(lat))
"""


def test_evp_doorbell_busy_workgroup_yields_to_next_instance():
    """A workgroup whose thread never stops calling must still leave at its
    lifetime (evp_server.hip checks the clock before every poll): otherwise it
    holds the next instance, queued behind it on the same stream, off the GPU,
    and a thread whose workgroup has already exited waits for the busy thread
    to pause.  The late thread's calls must stay far below the 10 s timeout."""
    env = dict(os.environ, TLSGPU_EVP_DOORBELL="2", TLSGPU_EVP_DOORBELL_MS="20", TLSGPU_CRASH_TRACE="1")
    env.pop("TLSGPU_EVP_BATCH_US", None)
    r = subprocess.run([sys.executable, "-c", _BUSY_CHILD, ROOT], env=env,
                       capture_output=True, text=True, timeout=100)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
    worst = float(r.stdout.split()[-1])
    assert worst < 0.5, f"a call waited {worst:.3f} s behind a busy workgroup"


_CHILD_SCRUB = r"""
import os, random, sys, threading, time
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, os.path.join(sys.argv[1], "oracle"))
import talos_amd as ta, pyoracle as po
ta.load_library()
orc = po.Oracle()
N = 8
errors, ctxs = [], [None] * N
b1, b2 = threading.Barrier(N), threading.Barrier(N)
def worker(t):
    rnd = random.Random(900 + t)
    try:
        for rnd_i in range(6):
            kind = [po.AES_128_GCM, po.AES_256_GCM][(t + rnd_i) % 2]
            key = rnd.randbytes(po.KEY_LEN[kind])
            ctx, octx = ta.EvpAead(kind, key), orc.aead(kind, key)
            t_end = time.time() + 0.05   # past a few 20-ms server lifetimes: one workgroup per slot
            while True:
                nonce, pt, ad = rnd.randbytes(12), rnd.randbytes(1400), rnd.randbytes(13)
                ok, got, _ = ctx.seal(nonce, pt, ad)
                assert (ok, got) == tuple(orc.seal(octx, nonce, pt, ad)[:2]), (t, rnd_i)
                if time.time() > t_end:
                    break
            ctxs[t] = ctx
            b1.wait()
            ctxs[(t + 1) % N].cleanup()   # scrub a context another thread's workgroup cached
            b2.wait()
    except Exception as exc:
        errors.append(repr(exc))
        b1.abort(); b2.abort()
ths = [threading.Thread(target=worker, args=(t,)) for t in range(N)]
[t.start() for t in ths]; [t.join() for t in ths]
assert not errors, errors[:2]
time.sleep(0.1)                # idle workgroups look at the ring every 16 polls
scrubs, flushes = ta.evp_doorbell_scrub_stats()
print("SCRUBS", scrubs, "FLUSHES", flushes)
"""


def test_scrub_reaches_other_server_workgroups():
    """EVP_AEAD_CTX_cleanup's scrub job zeroes the serving
    workgroup's LDS copies of the key; the other server workgroups that cached
    the same key's tables zero theirs through the scrub ring (evp_server.hip,
    kSrvFlush).  Eight threads each use a context on their own doorbell slot
    (one workgroup each, once an instance is launched for 8 callers), then
    each cleans up its neighbour's context: at least one of those scrubs runs
    on a workgroup other than the one holding the key, and that one flushes."""
    env = dict(os.environ, TLSGPU_EVP_DOORBELL="64", TLSGPU_EVP_DOORBELL_MS="20")
    env.pop("TLSGPU_EVP_BATCH_US", None)
    r = subprocess.run([sys.executable, "-c", _CHILD_SCRUB, ROOT], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "SCRUBS" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
    w = r.stdout.split()
    scrubs, flushes = int(w[w.index("SCRUBS") + 1]), int(w[w.index("FLUSHES") + 1])
    assert scrubs >= 6 * 8 and flushes >= 1, r.stdout
