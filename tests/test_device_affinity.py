"""Multi-GPU device-affinity audit on the CPU (VERDICT r04 next-round 5;
DESIGN.md §6 "device affinity").

The group split (talos_amd/csrc/group.cpp) and the EVP device spread
(engine.cpp evp_pick) have only ever run with every member on device 0, where
a missing hipSetDevice cannot show.  Here the engine's unmodified host objects
run against tests/devstub/devstub.cpp — a recording stand-in for the HIP
runtime with TLSGPU_STUB_DEVICES fake GPUs (libtlsgpu_devstub.so, CPU only).
Each allocation, stream and event remembers the device current on its thread
when it was made; every kernel launch, async copy / memset and event record
must run with its stream's device current and may touch only that device's
memory (pinned host memory is mapped for all).  The child drives every path
that reaches a group member or an EVP device from a thread other than the
one that made its resources: group install / device batches / host pipelines
over members [2, 0, 1], an engine on device 2 alone (batches, host pipeline,
wire framing, fills), EVP contexts dealt over devices 0, 1, 2 from 6 threads
(per call and through the coalescing queue, init / seal / open / cleanup),
and asserts the stub recorded no violation.  The kernels do not run (the
stub's launchers only check), so results are not looked at here; the GPU
suite checks them on [0, 0].
"""
import os
import shutil
import subprocess
import sys

import pytest

from conftest import ROOT

STUB_DIR = os.path.join(ROOT, "tests", "devstub")
STUB_LIB = os.path.join(STUB_DIR, "libtlsgpu_devstub.so")

_CHILD = r"""
import ctypes as C, os, sys, threading
import numpy as np
sys.path.insert(0, sys.argv[1])
import talos_amd as ta
lib = ta.load_library()
lib.devstub_report.restype = C.c_int
lib.devstub_report.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]

def params(k):
    kinds = [ta.AES_128_GCM, ta.AES_256_GCM, ta.CHACHA20_POLY1305, ta.CHACHA20_POLY1305_OLD]
    kind = kinds[k % 4]
    klen = 16 if kind == ta.AES_128_GCM else 32
    ivlen = 4 if kind in (ta.AES_128_GCM, ta.AES_256_GCM) else (12 if kind == ta.CHACHA20_POLY1305 else 0)
    return ta.SessionParams(kind, bytes([k + 1]) * klen, bytes([k + 7]) * ivlen)

N, REC = 64, 1024
def records(seal):
    r = np.zeros(N, dtype=ta.RECORD_DTYPE)
    for i in range(N):
        body = REC + (0 if seal else 24)
        r[i] = (i * 2048, i * 2048 + 8, i, i % 4, (23 << 24) | body)
    return r
BUF = N * 2048 + 4096

def pinned(eng_h, n):
    p = C.c_void_p()
    assert lib.tlsgpu_host_alloc(eng_h, n, C.byref(p)) == 0
    return p.value

# --- group over devices [2, 0, 1]: install, device-resident batches, host pipelines
g = ta.Group([2, 0, 1])
gs = ta.GroupSessionTable(g, 8)
gs.install(0, [params(k) for k in range(4)])
shards = np.zeros(g.size, dtype=ta.SHARD_DTYPE)
for k in range(g.size):
    eng = ta.Engine.member(g, k)
    d_recs, d_in, d_out, d_st = (ta.DeviceBuffer(eng, n) for n in (32 * N, BUF, BUF, 4 * N))
    d_recs.upload(records(False).view(np.uint8))
    shards[k] = (d_recs.ptr, N, 0, d_in.ptr, BUF, d_out.ptr, BUF, d_st.ptr)
    globals().setdefault("_keep", []).extend([d_recs, d_in, d_out, d_st])
gs.batch(shards, seal=False)
gs.batch(shards, seal=True)
g.sync()
e0 = ta.Engine.member(g, 0).handle
for seal in (False, True):
    recs = records(seal)
    h_in, h_out, h_st = pinned(e0, BUF), pinned(e0, BUF + 4096), pinned(e0, 4 * N)
    (gs.seal_host if seal else gs.open_host)(recs.ctypes.data, N, h_in, BUF, h_out, BUF + 4096, h_st)

# --- one engine on device 2: batches, host pipeline, wire framing, fills
eng = ta.Engine(2)
tab = ta.SessionTable(eng, 8)
tab.install(0, [params(k) for k in range(4)])
d_recs, d_in, d_out, d_st = (ta.DeviceBuffer(eng, n) for n in (32 * N, BUF, BUF, 4 * N))
d_recs.upload(records(False).view(np.uint8))
ta.open_batch(tab, d_recs.ptr, N, d_in.ptr, BUF, d_out.ptr, BUF, d_st.ptr)
ta.seal_batch(tab, d_recs.ptr, N, d_in.ptr, BUF, d_out.ptr, BUF, d_st.ptr)
s2 = eng.new_stream()
ta.open_batch(tab, d_recs.ptr, N, d_in.ptr, BUF, d_out.ptr, BUF, d_st.ptr, s2)
eng.fill_synthetic(d_in.ptr, 2048, 1024, N, 5)
for seal in (False, True):
    recs = records(seal)
    h_in, h_out, h_st = pinned(eng.handle, BUF), pinned(eng.handle, BUF + 4096), pinned(eng.handle, 4 * N)
    (ta.seal_host if seal else ta.open_host)(tab, recs.ctypes.data, N, h_in, BUF, h_out, BUF + 4096, h_st)
ws = np.zeros(2, dtype=[("wire_off", "<u8"), ("wire_len", "<u4"), ("session", "<u4"), ("seq", "<u8"),
                        ("version", "<u2"), ("flags", "<u2"), ("pad", "<u4")])
d_ws, d_res, d_tot = ta.DeviceBuffer(eng, ws.nbytes), ta.DeviceBuffer(eng, 64 * 2), ta.DeviceBuffer(eng, 4)
d_ws.upload(ws.view(np.uint8))
ta.open_wire(tab, d_ws.ptr, 2, d_in.ptr, N, d_recs.ptr, d_st.ptr, d_res.ptr, d_tot.ptr)
eng.sync()

# --- EVP contexts dealt over devices 0, 1, 2 (TLSGPU_DEVICES), from 6 threads
def worker(t, calls):
    for i in range(calls):
        kind = [ta.AES_128_GCM, ta.AES_256_GCM, ta.CHACHA20_POLY1305][(t + i) % 3]
        ctx = ta.EvpAead(kind, bytes([t]) * (16 if kind == ta.AES_128_GCM else 32))
        ctx.seal(bytes(12), b"x" * 1400, b"ad")
        ctx.open(bytes(12), b"y" * 1416, b"ad")
        ctx.cleanup()
ths = [threading.Thread(target=worker, args=(t, 6)) for t in range(6)]
[t.start() for t in ths]; [t.join() for t in ths]
ta.evp_set_batching(50, 0, 64)
ths = [threading.Thread(target=worker, args=(t, 4)) for t in range(6)]
[t.start() for t in ths]; [t.join() for t in ths]
st = ta.evp_device_stats()
assert [d for d, _, _ in st] == [0, 1, 2], st
assert all(c > 0 for _, c, _ in st), st

g.close()
buf, chk, pc = C.create_string_buffer(1 << 16), C.c_uint64(), C.c_uint64()
nv = lib.devstub_report(buf, len(buf), C.byref(chk), C.byref(pc))
print("VIOLATIONS", nv, "CHECKED", chk.value, "PINNED_CROSS", pc.value)
print(buf.value.decode())
"""


@pytest.fixture(scope="module")
def stub_lib():
    if not shutil.which("hipcc") and not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc not available to build the stub library")
    subprocess.run(["make", "-C", STUB_DIR, "-s"], check=True, capture_output=True)
    return STUB_LIB


def test_every_member_call_reaches_its_device(stub_lib):
    # the stub runs no kernel, so no doorbell server could answer: launched path
    env = dict(os.environ, TLSGPU_LIBRARY=stub_lib, TLSGPU_STUB_DEVICES="3",
               TLSGPU_DEVICES="0,1,2", TLSGPU_EVP_DOORBELL="0")
    for k in ("TLSGPU_EVP_BATCH_US", "TLSGPU_DEVICE"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-c", _CHILD, ROOT], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    head = r.stdout.split("\n", 1)[0].split()
    nv, checked = int(head[1]), int(head[3])
    assert checked > 500, r.stdout[-2000:]   # the stub really saw the stream-ordered calls
    assert nv == 0, r.stdout[-4000:]


_NEGATIVE = r"""
import ctypes as C, sys
sys.path.insert(0, sys.argv[1])
import talos_amd as ta
lib = ta.load_library()
lib.devstub_report.restype = C.c_int
lib.devstub_report.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
eng = ta.Engine(2)
buf = ta.DeviceBuffer(eng, 256)
lib.hipSetDevice(0)              # a worker that forgot hipSetDevice(2)
lib.hipMemsetAsync(C.c_void_p(buf.ptr), 0, C.c_size_t(16), C.c_void_p(eng.stream))
p = C.c_void_p()
lib.hipMalloc(C.byref(p), C.c_size_t(64))   # lands on device 0
lib.hipSetDevice(2)
lib.hipMemsetAsync(p, 0, C.c_size_t(16), C.c_void_p(eng.stream))
out = C.create_string_buffer(4096)
print(lib.devstub_report(out, len(out), None, None))
print(out.value.decode())
"""


def test_stub_catches_a_missing_set_device(stub_lib):
    """The audit is not vacuous: a stream of device 2 used with device 0
    current, and device-0 memory touched by device-2 work, are both caught."""
    env = dict(os.environ, TLSGPU_LIBRARY=stub_lib, TLSGPU_STUB_DEVICES="3")
    r = subprocess.run([sys.executable, "-c", _NEGATIVE, ROOT], env=env, capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.splitlines()
    assert int(lines[0]) == 2, r.stdout
    assert "issued with device 0 current" in r.stdout and "memory of device 0" in r.stdout


_MEM_CHILD = r"""
import ctypes as C, os, sys, threading
sys.path.insert(0, sys.argv[1])
import talos_amd as ta
lib = ta.load_library()
lib.devstub_mem.restype = None
lib.devstub_mem.argtypes = [C.POINTER(C.c_uint64)] * 3
def mem():
    p, d, n = C.c_uint64(), C.c_uint64(), C.c_uint64()
    lib.devstub_mem(C.byref(p), C.byref(d), C.byref(n))
    return p.value, d.value, n.value
T = int(sys.argv[2])
def one_call(i):
    ctx = ta.EvpAead(ta.AES_128_GCM, bytes([i % 251 + 1]) * 16)
    ctx.seal(bytes(12), b"x" * 16384, b"a" * 13)   # the largest TLS record
    return ctx
one_call(0).cleanup()            # the process's shared setup (streams, slabs, servers)
p0, d0, n0 = mem()
def run_wave():
    bar = threading.Barrier(T)
    def w(i):
        ctx = one_call(i)
        bar.wait()               # every thread alive with its staging at once
        ctx.cleanup()
    ths = [threading.Thread(target=w, args=(i,)) for i in range(T)]
    [t.start() for t in ths]; [t.join() for t in ths]
    return mem()
p1, d1, n1 = run_wave()
p2, d2, n2 = run_wave()          # the exited threads' staging is reused
print("PINNED_PER_THREAD", (p1 - p0) / T, "DEVICE_PER_THREAD", (d1 - d0) / T,
      "PINNED_ALLOCS", n1 - n0, "SECOND_WAVE_PINNED_GROWTH", p2 - p1)
"""


def test_per_call_staging_is_bounded(stub_lib):
    """a thread-per-connection server's calling
    threads each hold at most 64 KiB of pinned staging and no device staging
    (zero-copy per-call path), carved from shared slabs (few pinned
    allocations), and a second wave of threads reuses the first wave's staging
    instead of growing.  1,024 threads, each sealing a 16 KiB record on the
    launched path under the recording HIP stub (no GPU)."""
    env = dict(os.environ, TLSGPU_LIBRARY=stub_lib, TLSGPU_STUB_DEVICES="1",
               TLSGPU_EVP_DOORBELL="0")
    for k in ("TLSGPU_EVP_BATCH_US", "TLSGPU_DEVICE", "TLSGPU_DEVICES"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-c", _MEM_CHILD, ROOT, "1024"], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    w = r.stdout.split()
    val = {w[i]: float(w[i + 1]) for i in range(0, len(w) - 1, 2)}
    assert val["PINNED_PER_THREAD"] <= 64 * 1024, r.stdout
    assert val["DEVICE_PER_THREAD"] == 0, r.stdout
    assert val["PINNED_ALLOCS"] <= 1024 / 32 + 8, r.stdout    # slabs, not one per thread
    assert val["SECOND_WAVE_PINNED_GROWTH"] == 0, r.stdout
