"""Multi-GPU batch split in the C ABI (include/tlsgpu.h tlsgpu_group_*,
SURVEY.md §8e, BASELINE configs[4]).

CPU: tlsgpu_split_by_bytes cuts exactly where talos_amd.dist.shard_by_bytes
(the bench's rank split) cuts.  GPU: a group of two engines on device 0 — two
streams, two worker threads, two session-table replicas, the code path of two
GPUs — seals and opens host-resident and device-resident batches; every record
is checked against the oracle's tls1_enc (ssl/t1_enc.c:832-975).  Also the
host pipeline's failure path: a failure in the middle of the
chunk loop returns only after the chunks already queued have finished.
"""
import ctypes as C
import os
import random
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle as po  # noqa: E402


@pytest.fixture(scope="module")
def ta():
    import talos_amd
    talos_amd.load_library()
    return talos_amd


def test_split_by_bytes_matches_dist(ta):
    from talos_amd.dist import shard_by_bytes
    from talos_amd.workload import zipf_lengths
    rng = np.random.default_rng(7)
    for n in (0, 1, 2, 9, 1000, 65536):
        for parts in (1, 2, 3, 4, 8):
            for lens in (np.full(n, 16384), zipf_lengths(n, 5) if n else np.zeros(0, int),
                         rng.integers(0, 3, n)):
                recs = np.zeros(n, dtype=ta.RECORD_DTYPE)
                recs["len_type"] = (23 << 24) | lens.astype(np.uint32)
                cuts = ta.split_by_bytes(recs, parts)
                want = [shard_by_bytes(lens, parts, k)[0] for k in range(parts)] + [n]
                assert cuts == want, (n, parts)
    recs = np.zeros(4, dtype=ta.RECORD_DTYPE)
    recs["len_type"] = 100
    assert ta.split_by_bytes(recs, 2) == [0, 2, 4]
    with pytest.raises(ta.TlsGpuError):
        ta.split_by_bytes(recs, 0)


def _params(ta, rnd, kinds):
    return [ta.SessionParams(k, bytes(rnd.getrandbits(8) for _ in range(po.KEY_LEN[k])),
                             bytes(rnd.getrandbits(8) for _ in range(po.FIXED_IV_LEN[k])))
            for k in kinds]


def _pinned(lib, eng, nbytes, keep):
    p = C.c_void_p()
    assert lib.tlsgpu_host_alloc(eng, max(nbytes, 1), C.byref(p)) == 0
    keep.append(p.value)
    return p.value


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["ascending", "shuffled"])
def test_group_host_two_engines(ta, oracle, layout):
    """tlsgpu_group_seal_host then tlsgpu_group_open_host over a 2-member group;
    the byte split gives each member about half the bytes (shuffled layout: one
    member takes the batch)."""
    rnd = random.Random(71)
    params = _params(ta, rnd, [po.AES_128_GCM, po.CHACHA20_POLY1305, po.AES_256_GCM,
                               po.CHACHA20_POLY1305_OLD])
    g = ta.Group([0, 0])
    assert g.size == 2
    gs = ta.GroupSessionTable(g, len(params))
    gs.install(0, params)
    osess = [oracle.tls_session(p.aead, p.key, p.fixed_iv) for p in params]
    n = 240
    recs = []
    for i in range(n):
        ln = rnd.choice([0, 1, 16, 17, 1400, 4096, 16384])
        sid = (i // 5) % len(params)
        recs.append((sid, rnd.getrandbits(64), bytes(rnd.getrandbits(8) for _ in range(ln))))
    order = list(range(n))
    if layout == "shuffled":
        rnd.shuffle(order)
    io, oo, ip, op = [0] * n, [0] * n, 0, 0
    for i in order:
        io[i] = ip
        ip += len(recs[i][2]) + (-len(recs[i][2])) % 16 + 16
        oo[i] = op
        op += len(recs[i][2]) + 8 + 16 + 16
    keep = []
    lib, e0 = g.lib, g.lib.tlsgpu_group_engine(g.handle, 0)
    in_bytes, out_bytes = ip + 64, op + 64
    h_pt = _pinned(lib, e0, in_bytes, keep)
    h_body = _pinned(lib, e0, out_bytes, keep)
    h_back = _pinned(lib, e0, in_bytes, keep)
    h_recs = _pinned(lib, e0, 32 * n, keep)
    h_status = _pinned(lib, e0, 4 * n, keep)
    descs = np.zeros(n, dtype=ta.RECORD_DTYPE)
    for i, (sid, seq, pt) in enumerate(recs):
        C.memmove(h_pt + io[i], pt, len(pt))
        descs[i] = (io[i], oo[i], seq, sid, ta.len_type(len(pt), 23))
    C.memmove(h_recs, descs.tobytes(), descs.nbytes)
    try:
        gs.seal_host(h_recs, n, h_pt, in_bytes, h_body, out_bytes, h_status)
        st = np.ctypeslib.as_array((C.c_int32 * n).from_address(h_status)).copy()
        bodies = []
        for i, (sid, seq, pt) in enumerate(recs):
            exp = oracle.tls_seal(osess[sid], seq, 23, pt)
            assert st[i] == len(exp) and C.string_at(h_body + oo[i], len(exp)) == exp, i
            bodies.append(exp)
        # tamper a few, then open out of place back into h_back
        odescs = descs.copy()
        for i, (sid, seq, pt) in enumerate(recs):
            odescs[i] = (oo[i], io[i], seq, sid, ta.len_type(len(bodies[i]), 23))
            if i % 37 == 3:
                C.memset(h_body + oo[i] + len(bodies[i]) - 1,
                         bodies[i][-1] ^ 1, 1)
        C.memmove(h_recs, odescs.tobytes(), odescs.nbytes)
        gs.open_host(h_recs, n, h_body, out_bytes, h_back, in_bytes, h_status)
        st = np.ctypeslib.as_array((C.c_int32 * n).from_address(h_status)).copy()
        for i, (sid, seq, pt) in enumerate(recs):
            if i % 37 == 3:
                assert st[i] == ta.REC_BAD_MAC and C.string_at(h_back + io[i], len(pt)) == bytes(len(pt))
            else:
                assert st[i] == len(pt) and C.string_at(h_back + io[i], len(pt)) == pt, i
    finally:
        for p in keep:
            lib.tlsgpu_host_free(e0, p)
        gs.close()
        g.close()


@pytest.mark.gpu
def test_group_device_batch_two_engines(ta, oracle):
    """tlsgpu_group_open_batch: each member opens its own slice from its own
    HBM buffers (per-GPU pools), asynchronously; tlsgpu_group_sync joins."""
    rnd = random.Random(73)
    params = _params(ta, rnd, [po.AES_128_GCM, po.AES_256_GCM, po.CHACHA20_POLY1305])
    g = ta.Group([0, 0])
    gs = ta.GroupSessionTable(g, len(params))
    gs.install(0, params)
    osess = [oracle.tls_session(p.aead, p.key, p.fixed_iv) for p in params]
    lib = g.lib
    shards = np.zeros(2, dtype=ta.SHARD_DTYPE)
    want, bufs = [], []

    def dmalloc(eng, nbytes):
        p = C.c_void_p()
        assert lib.tlsgpu_malloc(eng, max(nbytes, 1), C.byref(p)) == 0
        bufs.append((eng, p.value))
        return p.value

    for m in range(2):
        eng = lib.tlsgpu_group_engine(g.handle, m)
        recs, body, descs, pos = [], bytearray(), [], 0
        for i in range(150):
            ln = rnd.choice([0, 5, 64, 1000, 16384])
            sid = i % len(params)
            seq = rnd.getrandbits(64)
            pt = bytes(rnd.getrandbits(8) for _ in range(ln))
            b = oracle.tls_seal(osess[sid], seq, 23, pt)
            eiv = 8 if params[sid].aead != po.CHACHA20_POLY1305 else 0
            descs.append((pos, pos + eiv, seq, sid, ta.len_type(len(b), 23)))   # in place
            body += b + bytes((-len(b)) % 16)
            recs.append((pos + eiv, pt))
            pos = len(body)
        arr = np.array(descs, dtype=ta.RECORD_DTYPE)
        d_body, d_recs = dmalloc(eng, len(body)), dmalloc(eng, arr.nbytes)
        d_status = dmalloc(eng, 4 * len(descs))
        assert lib.tlsgpu_memcpy(eng, d_body, bytes(body), len(body), None) == 0
        assert lib.tlsgpu_memcpy(eng, d_recs, arr.ctypes.data, arr.nbytes, None) == 0
        assert lib.tlsgpu_engine_sync(eng) == 0
        shards[m] = (d_recs, len(descs), 0, d_body, len(body), d_body, len(body), d_status)
        want.append((eng, d_body, len(body), d_status, recs))
    try:
        gs.batch(shards, seal=False)
        g.sync()
        for eng, d_body, nbytes, d_status, recs in want:
            out = (C.c_uint8 * nbytes)()
            st = (C.c_int32 * len(recs))()
            assert lib.tlsgpu_memcpy(eng, out, d_body, nbytes, None) == 0
            assert lib.tlsgpu_memcpy(eng, st, d_status, 4 * len(recs), None) == 0
            assert lib.tlsgpu_engine_sync(eng) == 0
            raw = bytes(out)
            for k, (o, pt) in enumerate(recs):
                assert st[k] == len(pt) and raw[o:o + len(pt)] == pt, k
    finally:
        for eng, p in bufs:
            lib.tlsgpu_free(eng, p)
        gs.close()
        g.close()


_FAIL_CHILD = r"""
import ctypes as C, sys, numpy as np
sys.path.insert(0, sys.argv[1])
import talos_amd as ta
eng = ta.Engine(0)
t = ta.SessionTable(eng, 1)
key, fiv = bytes(range(16)), bytes(4)
t.install(0, [ta.SessionParams(ta.AES_128_GCM, key, fiv)])
n, L = 512, 16384
keep = []
def pinned(nb):
    p = C.c_void_p(); assert eng.lib.tlsgpu_host_alloc(eng.handle, nb, C.byref(p)) == 0
    keep.append(p.value); return p.value
h_in, h_out, h_recs, h_st = pinned(n * L), pinned(n * (L + 64)), pinned(32 * n), pinned(4 * n)
C.memset(h_in, 0x33, n * L); C.memset(h_out, 0x77, n * (L + 64))
d = np.zeros(n, dtype=ta.RECORD_DTYPE)
d["in_off"] = np.arange(n) * L; d["out_off"] = np.arange(n) * (L + 64); d["seq"] = np.arange(n)
d["len_type"] = ta.len_type(L, 23)
C.memmove(h_recs, d.tobytes(), d.nbytes)
ta.host_pipeline(eng, 2, 1 << 20)
try:
    ta.seal_host(t, h_recs, n, h_in, n * L, h_out, n * (L + 64), h_st)
    print("NO-ERROR")
except ta.TlsGpuError as exc:
    assert "injected" in str(exc), exc
    # chunk 0 (1 MiB = 64 records) was queued before the failure: the call
    # returned only after its copy back finished, so its fragments are final
    first = C.string_at(h_out, 8)
    assert first == (0).to_bytes(8, "big"), first     # explicit nonce = seq 0
    tail = C.string_at(h_out + 63 * (L + 64), L + 24)
    assert tail[:8] == (63).to_bytes(8, "big") and tail[8:] != b"\x77" * (L + 16)
    print("DRAINED")
"""


@pytest.mark.gpu
def test_host_pipeline_failure_drains(ta, tmp_path):
    """TLSGPU_TEST_HOST_FAIL_CHUNK=2: tlsgpu_seal_host fails after queueing
    chunk 2's copy in; chunks 0-1 are already running.  The error must come back
    only after they have drained (their sealed fragments are in h_out)."""
    env = dict(os.environ, TLSGPU_TEST_HOST_FAIL_CHUNK="2")
    r = subprocess.run([sys.executable, "-c", _FAIL_CHILD, ROOT], env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0 and "DRAINED" in r.stdout, r.stdout + r.stderr


_GROUP_FAIL_CHILD = r"""
import ctypes as C, sys, numpy as np
sys.path.insert(0, sys.argv[1])
import talos_amd as ta
g = ta.Group([0, 0])
gs = ta.GroupSessionTable(g, 1)
gs.install(0, [ta.SessionParams(ta.AES_128_GCM, bytes(range(16)), bytes(4))])
eng = g.lib.tlsgpu_group_engine(g.handle, 0)
n, L = 512, 16384
keep = []
def pinned(nb):
    p = C.c_void_p(); assert g.lib.tlsgpu_host_alloc(eng, nb, C.byref(p)) == 0
    keep.append(p.value); return p.value
h_in, h_out, h_recs, h_st = pinned(n * L), pinned(n * (L + 64)), pinned(32 * n), pinned(4 * n)
d = np.zeros(n, dtype=ta.RECORD_DTYPE)
d["in_off"] = np.arange(n) * L; d["out_off"] = np.arange(n) * (L + 64); d["seq"] = np.arange(n)
d["len_type"] = ta.len_type(L, 23)
C.memmove(h_recs, d.tobytes(), d.nbytes)
assert g.lib.tlsgpu_host_pipeline(eng, 2, 1 << 20) == 0
try:   # group-level argument failure
    gs.seal_host(h_recs, n, h_in, n * L, h_in, n * L, h_st)
    print("NO-ERROR-1")
except ta.TlsGpuError as exc:
    assert "in place" in str(exc), exc
try:   # a member's failure (on its worker thread) reaches this thread
    gs.seal_host(h_recs, n, h_in, n * L, h_out, n * (L + 64), h_st)
    print("NO-ERROR-2")
except ta.TlsGpuError as exc:
    assert "group member" in str(exc) and "injected" in str(exc), exc
    print("REASONS-OK")
"""


@pytest.mark.gpu
def test_group_errors_reach_caller(ta):
    """tlsgpu_last_error on the caller's thread carries the reason of a failed
    group call: a group-level argument check and a member's failure on its
    worker thread."""
    env = dict(os.environ, TLSGPU_TEST_HOST_FAIL_CHUNK="2")
    r = subprocess.run([sys.executable, "-c", _GROUP_FAIL_CHILD, ROOT], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "REASONS-OK" in r.stdout, r.stdout + r.stderr
