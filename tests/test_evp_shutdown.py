"""The doorbell server's shutdown contract (round 5, VERDICT r04 next-round 1;
DESIGN.md §4.7b; include/tlsgpu.h tlsgpu_evp_shutdown).

A server instance (evp_server.hip) reads and writes pinned host memory for as
long as it runs: its slots, its stop page, the callers' staging.  The HIP
runtime frees every pinned allocation when it tears down at exit, so every
instance ever launched — running, or still queued behind other work on a
shared hardware queue — must have left before that.  The library stops and
drains the servers first thing in exit() (the main thread's thread-local exit
guard), with no HIP call and no silent cap.  Each child process here exits in
one of the states that can race the runtime's teardown and must end with
status 0, its result line, and the drain's own report:

* right after a call, the instance mid-lifetime (2 s lifetime: the drain must
  stop it, not wait it out);
* two EVP devices on one GPU (TLSGPU_DEVICES=0,0): two servers, the r04v
  configuration;
* a server instance queued behind a long kernel on the same hardware queue
  (GPU_MAX_HW_QUEUES=1, a warm-up launch behind ~0.3 s of fill kernels);
* an explicit tlsgpu_evp_shutdown() mid-process, after which calls must take
  the launched path and still equal the oracle;
* a caller descheduled between its relaunch check and its post for longer
  than the lifetime (the wait loop relaunches past the deadline).

Children run with faulthandler enabled and TLSGPU_CRASH_TRACE=1, so a fault
at exit reports the exit phase and a native backtrace.
"""
import json
import os
import subprocess
import sys
import time

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

_PRE = r"""
import faulthandler, os, random, sys, threading, time
faulthandler.enable()
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, os.path.join(sys.argv[1], "oracle"))
import talos_amd as ta, pyoracle as po
ta.load_library()
orc = po.Oracle()
def check_calls(kind, rnd, n=4, sizes=(0, 17, 1400, 5000)):
    key = bytes(rnd.randrange(256) for _ in range(po.KEY_LEN[kind]))
    ctx, octx = ta.EvpAead(kind, key), orc.aead(kind, key)
    assert ctx.ok == 1
    for i in range(n):
        nonce = bytes(rnd.randrange(256) for _ in range(12))
        pt = bytes(rnd.randrange(256) for _ in range(rnd.choice(sizes)))
        ad = bytes(rnd.randrange(256) for _ in range(13))
        ok, exp = orc.seal(octx, nonce, pt, ad)
        ok2, got, _ = ctx.seal(nonce, pt, ad)
        assert ok == ok2 == 1 and got == exp, (kind, i, len(pt))
        ok3, back, _ = ctx.open(nonce, got, ad)
        assert ok3 == 1 and back == pt, (kind, i)
    return ctx
"""

_MID_LIFETIME = _PRE + r"""
rnd = random.Random(1)
for kind in (po.AES_128_GCM, po.CHACHA20_POLY1305):
    check_calls(kind, rnd).cleanup()
j, l = ta.evp_doorbell_stats()
assert j > 0 and l >= 1, (j, l)
print("OK", j, l, flush=True)
"""

_TWO_SERVERS = _PRE + r"""
errors = []
def worker(t):
    try:
        rnd = random.Random(70 + t)
        check_calls([po.AES_128_GCM, po.AES_256_GCM, po.CHACHA20_POLY1305][t % 3], rnd, n=6).cleanup()
    except Exception as exc:
        errors.append(repr(exc))
ths = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
[t.start() for t in ths]; [t.join() for t in ths]
assert not errors, errors[:2]
st = ta.evp_device_stats()
assert len(st) == 2 and all(c == 4 for _, c, _ in st), st
j, l = ta.evp_doorbell_stats()
assert j > 0, (j, l)
print("OK", j, l, flush=True)
"""

_QUEUED = _PRE + r"""
rnd = random.Random(2)
ctx = check_calls(po.AES_128_GCM, rnd, n=2)
import ctypes as C
eng = ta.Engine(0)
p = C.c_void_p()
# raw allocation, never freed: a hipFree during interpreter teardown would wait
# for the queue and let the instance run out before the exit hooks
assert eng.lib.tlsgpu_malloc(eng.handle, 1 << 30, C.byref(p)) == 0
# ~0.3 s of fill kernels on the engine stream; with one hardware queue per
# process the next server instance queues behind them
t = time.perf_counter()
for i in range(1000):
    eng.fill_synthetic(p.value, 1 << 30, 1 << 30, 1, 7 + i)
time.sleep(0.05)          # past half the 40 ms lifetime: warm launches a new instance
ta.evp_doorbell_warm()
j, l = ta.evp_doorbell_stats()
assert l >= 2, (j, l)
print("OK", j, l, round(time.perf_counter() - t, 3), flush=True)
# exit now: the warm instance is still queued behind the fills
"""

_EXPLICIT = _PRE + r"""
rnd = random.Random(3)
ctx = check_calls(po.AES_128_GCM, rnd)
j0, l0 = ta.evp_doorbell_stats()
assert j0 > 0
ta.evp_shutdown()
ta.evp_shutdown()          # idempotent
for _ in range(2):         # the same context, then fresh ones: launched path, still exact
    check_calls(po.AES_128_GCM, rnd)
ctx.cleanup()
check_calls(po.CHACHA20_POLY1305, rnd).cleanup()
j1, l1 = ta.evp_doorbell_stats()
assert (j1, l1) == (j0, l0), ((j0, l0), (j1, l1))   # no job posted, nothing launched
print("OK", j1, l1, flush=True)
"""

_POST_DELAY = _PRE + r"""
rnd = random.Random(4)
key = bytes(16)
ctx, octx = ta.EvpAead(po.AES_128_GCM, key), orc.aead(po.AES_128_GCM, key)
worst = 0.0
for i in range(8):
    nonce = bytes(rnd.randrange(256) for _ in range(12))
    pt = bytes(rnd.randrange(256) for _ in range(1400))
    t = time.perf_counter()
    ok, got, _ = ctx.seal(nonce, pt, b"")
    worst = max(worst, time.perf_counter() - t)
    assert ok == 1 and got == orc.seal(octx, nonce, pt, b"")[1], i
ctx.cleanup()
j, l = ta.evp_doorbell_stats()
assert j >= 7, (j, l)      # the first call of a context takes the launched path
print("OK", j, l, round(worst, 4), flush=True)
"""


def _run(code, extra_env, timeout=120):
    env = dict(os.environ, TLSGPU_EVP_SHUTDOWN_VERBOSE="1", TLSGPU_CRASH_TRACE="1")
    env.pop("TLSGPU_EVP_BATCH_US", None)
    env.pop("TLSGPU_DEVICES", None)
    env.update(extra_env)
    t = time.perf_counter()
    r = subprocess.run([sys.executable, "-c", code, ROOT], env=env, capture_output=True,
                       text=True, timeout=timeout)
    wall = time.perf_counter() - t
    assert r.returncode == 0 and "OK" in r.stdout, \
        f"rc={r.returncode}\n" + r.stdout[-2000:] + r.stderr[-3000:]
    drains = [json.loads(l)["evp_shutdown"] for l in r.stderr.splitlines()
              if l.startswith('{"evp_shutdown"')]
    assert len(drains) == 1, r.stderr[-2000:]   # drained exactly once (idempotent hooks)
    return r.stdout.split(), drains[0], wall


def test_exit_with_instance_mid_lifetime():
    out, drain, wall = _run(_MID_LIFETIME, {"TLSGPU_EVP_DOORBELL": "4",
                                            "TLSGPU_EVP_DOORBELL_MS": "2000"})
    assert drain["instances_waited"] >= 1, drain
    assert drain["ms"] < 1000, drain   # stopped by the stop word, not by its 2 s lifetime


def test_exit_with_two_servers_on_one_gpu():
    out, drain, wall = _run(_TWO_SERVERS, {"TLSGPU_EVP_DOORBELL": "8",
                                           "TLSGPU_EVP_DOORBELL_MS": "2000",
                                           "TLSGPU_DEVICES": "0,0"})
    assert drain["instances_waited"] >= 2, drain   # one per server at least


def test_exit_with_instance_queued_behind_long_kernel():
    out, drain, wall = _run(_QUEUED, {"TLSGPU_EVP_DOORBELL": "2",
                                      "TLSGPU_EVP_DOORBELL_MS": "40",
                                      "GPU_MAX_HW_QUEUES": "1"})
    assert drain["instances_waited"] >= 1, drain


def test_explicit_shutdown_then_launched_path():
    _run(_EXPLICIT, {"TLSGPU_EVP_DOORBELL": "4", "TLSGPU_EVP_DOORBELL_MS": "2000"})


def test_post_delayed_past_lifetime_is_served():
    """a caller descheduled for longer than the instance's
    lifetime between server_ensure and its post must not wait out the 10 s
    timeout — the wait loop relaunches once the deadline has passed."""
    out, drain, wall = _run(_POST_DELAY, {"TLSGPU_EVP_DOORBELL": "2",
                                          "TLSGPU_EVP_DOORBELL_MS": "2",
                                          "TLSGPU_TEST_DOORBELL_POST_DELAY_US": "5000"})
    worst = float(out[-1])
    assert worst < 0.5, f"a delayed post waited {worst:.3f} s"
