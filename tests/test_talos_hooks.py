"""TaLoS's TLS-processing interface on the engine.

libtlsgpu.so exports tls_processing_register_ssl_{read,write}_processing_cb &
co. with the reference signatures (src/talos/enclaveshim/
tls_processing_interface.h:23-49; include/tlsgpu_talos.h).

* CPU: the registry itself — a module's read callback gets (SSL*, data, len*),
  also when the caller passes the length BY VALUE as the TaLoS-patched
  s3_pkt.c does (s3_pkt.c.patch:13-14); and the reference's own nosgx build
  (oracle/_ref/ssl_loopback_talos: the TaLoS-patched tree, patch_libressl.sh
  applied by oracle/talos_tree.sh, with a logpoint-style module linked in)
  faults on exactly that mismatch as soon as the module reads *len.
* GPU: the same TaLoS-patched libssl with libtlsgpu.so LD_PRELOADed — the
  record ciphers run on the GPU, the hooks at s3_pkt.c.patch:19-33 (write) and
  :39-52 (read) bind to libtlsgpu's interface, and the module sees, per SSL
  object and direction, the exact plaintext of every application record.
* GPU: the engine's own host paths fire the registered callbacks with the SSL*
  set per session: tlsgpu_seal_host / tlsgpu_open_host, tlsgpu_deliver_host
  after tlsgpu_open_wire, tlsgpu_hook_write_streams before tlsgpu_seal_wire.
"""
import ctypes as C
import json
import os
import random
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle as po  # noqa: E402

LOOPBACK = os.path.join(ROOT, "oracle", "_ref", "ssl_loopback_talos")
PEM = os.path.join(ROOT, "tests", "golden", "server.pem")
LIB = os.path.join(ROOT, "talos_amd", "libtlsgpu.so")
CIPHERS = ["ECDHE-RSA-AES128-GCM-SHA256", "ECDHE-RSA-AES256-GCM-SHA384",
           "ECDHE-RSA-CHACHA20-POLY1305", "ECDHE-RSA-CHACHA20-POLY1305-OLD"]


@pytest.fixture(scope="module")
def ta():
    import talos_amd
    talos_amd.load_library()
    return talos_amd


def _loop(args, preload, env_extra=None, timeout=110):
    if not os.path.exists(LOOPBACK):
        pytest.skip("oracle/_ref/ssl_loopback_talos not built (reference tree absent at build time)")
    env = dict(os.environ)
    env.pop("LD_PRELOAD", None)
    if preload:
        env["LD_PRELOAD"] = LIB
    env.update(env_extra or {})
    return subprocess.run([LOOPBACK, "-p", PEM] + [str(a) for a in args], capture_output=True,
                          text=True, timeout=timeout, env=env)


def test_registry_by_value_and_pointer_lengths(ta):
    """tls_processing_ssl_read with len as a pointer (the interface) and as a
    value (the patched record layer's call): the callback reads *len both times."""
    lib = ta.load_library()
    seen = []

    def on_read(ssl, data, plen):
        seen.append((ssl, C.string_at(data, plen[0]), plen[0]))

    cbs = ta.talos_register(on_read, None)
    try:
        fn = lib.tls_processing_ssl_read
        fn.restype = None
        buf = C.create_string_buffer(b"GET / HTTP/1.1\r\n", 16)
        n = C.c_uint(16)
        r0, w0 = ta.talos_hook_stats()
        fn.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        fn(0x1234, buf, C.addressof(n))        # unsigned int *len
        fn(0x5678, buf, 5)                      # unsigned int len (s3_pkt.c.patch:13-14)
        assert seen == [(0x1234, b"GET / HTTP/1.1\r\n", 16), (0x5678, b"GET /", 5)]
        assert ta.talos_hook_stats() == (r0 + 2, w0)
    finally:
        ta.talos_register(None, None)
        del cbs


_LEN_MODE_CHILD = r"""
import ctypes as C, sys
sys.path.insert(0, sys.argv[1])
import talos_amd as ta
lib = ta.load_library()
seen = []
def on_read(ssl, data, plen):
    seen.append(plen[0])
cbs = ta.talos_register(on_read, None)
fn = lib.tls_processing_ssl_read
fn.restype = None
fn.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
buf = C.create_string_buffer(64)
n = C.c_uint(16)
if sys.argv[2] == "value":
    # by-value length with junk in the upper half of the register: only the low
    # 32 bits count
    fn(1, buf, (0xDEADBEEF << 32) | 7)
    fn(1, buf, 9)
else:
    fn(1, buf, C.addressof(n))
print(seen)
"""


@pytest.mark.parametrize("mode,want", [("value", "[7, 9]"), ("pointer", "[16]")])
def test_talos_len_mode_setting(mode, want):
    """TLSGPU_TALOS_LEN=value reads the low 32 bits of the third argument as the
    length (the patched record layer, any compiler); =pointer always dereferences
    it (tlsgpu_talos.h, process-wide)."""
    env = dict(os.environ, TLSGPU_TALOS_LEN=mode)
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([sys.executable, "-c", _LEN_MODE_CHILD, ROOT, mode], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip().splitlines()[-1] == want, r.stdout + r.stderr


def test_reference_nosgx_build_faults_with_logging_module():
    """The reference's own interface (tls_processing_interface.c:74-77) forwards
    the patched record layer's by-value length as a pointer; the module's *len
    read faults (SIGSEGV) — the latent bug SURVEY.md §8f-3 notes, live as soon
    as a module logs.  Without the module registered the build runs."""
    r = _loop(["-n", 8, "-m"], preload=False)
    assert r.returncode == -11, (r.returncode, r.stdout[-500:], r.stderr[-500:])
    r = _loop(["-n", 8], preload=False)
    assert r.returncode == 0 and json.loads(r.stdout.splitlines()[-1])["ok"]


@pytest.mark.gpu
@pytest.mark.parametrize("cipher", CIPHERS)
@pytest.mark.parametrize("queue", [False, True])
def test_talos_module_sees_every_record_with_engine(cipher, queue):
    """TaLoS-patched libssl + LD_PRELOAD=libtlsgpu.so + a registered module:
    every record cipher on the GPU, the module sees the plaintext of every
    application record at the patched call sites."""
    env = {"TLSGPU_EVP_BATCH_US": "100"} if queue else {}
    threads = 4 if queue else 2
    r = _loop(["-c", cipher, "-n", 200, "-r", 1024, "-t", threads, "-m"], preload=True,
              env_extra=env)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    m = d["talos_module"]
    assert d["ok"] and m["ok"] and d["tlsgpu_interposed"], d
    assert m["streams_ok"] == m["streams"] == 4 * threads
    assert m["new_connections"] == 2 * threads and m["tlsgpu_hooks"]
    assert d["tlsgpu_seal_calls"] == d["records_sealed_expected"]
    assert d["tlsgpu_open_calls"] == d["records_opened_expected"]
    # every hook call of the record layer went through libtlsgpu's interface:
    # at least one write per sealed record, one read per application record
    assert m["tlsgpu_hook_write_calls"] >= d["records_sealed_expected"]
    assert m["tlsgpu_hook_read_calls"] >= 2 * threads * 200


def _pinned(lib, eng, nbytes, keep):
    p = C.c_void_p()
    assert lib.tlsgpu_host_alloc(eng, max(nbytes, 1), C.byref(p)) == 0
    keep.append(p.value)
    return p.value


@pytest.mark.gpu
def test_engine_host_paths_fire_module_callbacks(ta, oracle):
    """tlsgpu_seal_host fires the write callback on each record (the module
    rewrites it in place and shortens one), tlsgpu_open_host the read callback
    on each delivered record (it shortens one delivery), with the SSL* owner of
    the record's session."""
    rnd = random.Random(79)
    eng = ta.Engine(0)
    kinds = [po.AES_128_GCM, po.CHACHA20_POLY1305, po.AES_256_GCM]
    params = [ta.SessionParams(k, bytes(rnd.getrandbits(8) for _ in range(po.KEY_LEN[k])),
                               bytes(rnd.getrandbits(8) for _ in range(po.FIXED_IV_LEN[k])))
              for k in kinds]
    table = ta.SessionTable(eng, len(params))
    table.install(0, params)
    owners = [0xA000 + 0x100 * i for i in range(len(params))]
    ta.set_session_owners(table, 0, owners)
    osess = [oracle.tls_session(p.aead, p.key, p.fixed_iv) for p in params]
    n, recs, ip, op = 90, [], 0, 0
    for i in range(n):
        ln = rnd.choice([1, 17, 1400, 4096, 16384])
        recs.append((i % 3, rnd.getrandbits(64), bytes(rnd.getrandbits(8) for _ in range(ln)), ip, op))
        ip += ln + 32
        op += ln + 64
    keep, lib = [], eng.lib
    in_bytes, out_bytes = ip + 64, op + 64
    h_in, h_out = _pinned(lib, eng.handle, in_bytes, keep), _pinned(lib, eng.handle, out_bytes, keep)
    h_back = _pinned(lib, eng.handle, in_bytes, keep)
    h_recs, h_status = _pinned(lib, eng.handle, 32 * n, keep), _pinned(lib, eng.handle, 4 * n, keep)
    descs = np.zeros(n, dtype=ta.RECORD_DTYPE)
    for i, (sid, seq, pt, io, oo) in enumerate(recs):
        C.memmove(h_in + io, pt, len(pt))
        descs[i] = (io, oo, seq, sid, ta.len_type(len(pt), 23))
    C.memmove(h_recs, descs.tobytes(), descs.nbytes)
    wrote, read = [], []

    def on_write(ssl, data, plen):
        k = len(wrote)
        wrote.append((ssl, plen[0]))
        for j in range(plen[0]):
            data[j] ^= 0x3C
        if k == 7:
            plen[0] = plen[0] // 2        # the module shortens record 7

    def on_read(ssl, data, plen):
        read.append((ssl, C.string_at(data, plen[0])))
        if len(read) == 5:
            plen[0] = 1                   # and delivers one byte of record 4

    cbs = ta.talos_register(on_read, on_write)
    try:
        ta.seal_host(table, h_recs, n, h_in, in_bytes, h_out, out_bytes, h_status)
        st = np.ctypeslib.as_array((C.c_int32 * n).from_address(h_status)).copy()
        assert wrote == [(owners[sid], len(pt)) for sid, _, pt, _, _ in recs]
        bodies, pts = [], []
        for i, (sid, seq, pt, io, oo) in enumerate(recs):
            xpt = bytes(b ^ 0x3C for b in pt)
            if i == 7:
                xpt = xpt[:len(pt) // 2]
            exp = oracle.tls_seal(osess[sid], seq, 23, xpt)
            assert st[i] == len(exp) and C.string_at(h_out + oo, len(exp)) == exp, i
            bodies.append(exp)
            pts.append(xpt)
        odescs = np.zeros(n, dtype=ta.RECORD_DTYPE)
        for i, (sid, seq, pt, io, oo) in enumerate(recs):
            odescs[i] = (oo, io, seq, sid, ta.len_type(len(bodies[i]), 23))
        C.memmove(h_recs, odescs.tobytes(), odescs.nbytes)
        ta.open_host(table, h_recs, n, h_out, out_bytes, h_back, in_bytes, h_status)
        st = np.ctypeslib.as_array((C.c_int32 * n).from_address(h_status)).copy()
        assert [r[0] for r in read] == [owners[sid] for sid, *_ in recs]
        assert [r[1] for r in read] == [pts[i][:1] if i == 4 else pts[i] for i in range(n)]
        assert all(st[i] == (1 if i == 4 else len(pts[i])) for i in range(n))
    finally:
        ta.talos_register(None, None)
        del cbs
        for p in keep:
            lib.tlsgpu_host_free(eng.handle, p)
        table.close()
        eng.close()


@pytest.mark.gpu
def test_wire_paths_host_delivery_hooks(ta, oracle):
    """Write side: tlsgpu_hook_write_streams on host data, upload,
    tlsgpu_seal_wire.  Read side: tlsgpu_open_wire in place, then
    tlsgpu_deliver_host: statuses and plaintext in host memory, the read
    callback once per record in stream order with the stream's SSL*."""
    rnd = random.Random(83)
    eng = ta.Engine(0)
    lib = eng.lib
    kinds = [po.AES_128_GCM, po.CHACHA20_POLY1305]
    params = [ta.SessionParams(k, bytes(rnd.getrandbits(8) for _ in range(po.KEY_LEN[k])),
                               bytes(rnd.getrandbits(8) for _ in range(po.FIXED_IV_LEN[k])))
              for k in kinds]
    table = ta.SessionTable(eng, 2)
    table.install(0, params)
    owners = [0xBEEF00, 0xBEEF80]
    ta.set_session_owners(table, 0, owners)
    lens = [40000, 0, 100, 16384]
    data = bytearray(rnd.getrandbits(8) for _ in range(sum(lens) + 64))
    streams = np.zeros(len(lens), dtype=ta.WRITE_STREAM_DTYPE)
    doff, woff = 0, 0
    for i, ln in enumerate(lens):
        sid = i % 2
        streams[i] = (doff, woff, 1000 * i, ln, sid, 0x0303, 23, 0, 0)
        doff += ln
        woff += ta.seal_wire_size(kinds[sid], ln)
    wire_bytes, nrec = woff, sum((ln + 16383) // 16384 for ln in lens)
    hdata = (C.c_uint8 * len(data)).from_buffer(data)
    wrote = []

    def on_write(ssl, ptr, plen):
        wrote.append((ssl, plen[0]))
        for j in range(plen[0]):
            ptr[j] ^= 0x11

    def on_read(ssl, ptr, plen):
        read.append((ssl, C.string_at(ptr, plen[0])))

    read = []
    cbs = ta.talos_register(on_read, on_write)
    bufs = []

    def dev(nbytes):
        b = ta.DeviceBuffer(eng, nbytes)
        bufs.append(b)
        return b

    try:
        ta.hook_write_streams(table, streams.ctypes.data, len(lens), C.addressof(hdata), len(data))
        assert wrote == [(owners[0], 16384), (owners[0], 16384), (owners[0], 7232),
                         (owners[0], 100), (owners[1], 16384)]
        d_data, d_wire = dev(len(data)), dev(wire_bytes + 64)
        d_streams, d_recs, d_st = dev(streams.nbytes), dev(32 * nrec), dev(4 * nrec)
        d_res, d_tot = dev(32 * len(lens)), dev(4)
        d_data.upload(bytes(data))
        d_streams.upload(streams.view(np.uint8))
        ta.seal_wire(table, d_streams.ptr, len(lens), d_data.ptr, len(data), d_wire.ptr,
                     wire_bytes, nrec, d_recs.ptr, d_st.ptr, d_res.ptr, d_tot.ptr)
        eng.sync()
        # read the sealed wire back, one read stream per write stream
        rstreams = np.zeros(len(lens), dtype=ta.WIRE_STREAM_DTYPE)
        for i in range(len(lens)):
            rstreams[i] = (int(streams[i]["wire_off"]), ta.seal_wire_size(kinds[i % 2], lens[i]),
                           i % 2, 1000 * i, 0x0303, 0, 0)
        d_rs = dev(rstreams.nbytes)
        d_rs.upload(rstreams.view(np.uint8))
        ta.open_wire(table, d_rs.ptr, len(lens), d_wire.ptr, nrec, d_recs.ptr, d_st.ptr, d_res.ptr,
                     d_tot.ptr)
        keep = []
        h_wire = _pinned(lib, eng.handle, wire_bytes + 64, keep)
        h_st = _pinned(lib, eng.handle, 4 * nrec, keep)
        ta.deliver_host(table, d_recs.ptr, d_st.ptr, nrec, d_wire.ptr, wire_bytes + 64, h_wire, h_st)
        st = list(np.ctypeslib.as_array((C.c_int32 * nrec).from_address(h_st)))
        assert st == [16384, 16384, 7232, 100, 16384]
        xdata = bytes(b for b in data)          # rewritten in place by on_write
        want, pos = [], 0
        for i, ln in enumerate(lens):
            for k in range(0, ln, 16384):
                want.append((owners[i % 2], xdata[pos + k:pos + min(ln, k + 16384)]))
            pos += ln
        # streams reserve their descriptor ranges in any order; within a
        # stream the records come in order
        assert sorted(read) == sorted(want)
        s0 = [read.index(w) for w in want[:3]]
        assert s0 == sorted(s0)
        for p in keep:
            lib.tlsgpu_host_free(eng.handle, p)
    finally:
        ta.talos_register(None, None)
        del cbs
        for b in bufs:
            b.free()
        table.close()
        eng.close()
