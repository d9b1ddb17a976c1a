"""Host-resident batch open (tlsgpu_open_host) against the
oracle: fragments and plaintext in pinned host memory, as ssl3_read_n's rbuf
and the application buffer would hold them (s3_pkt.c:134-267, :957).

Checked for every record: status and plaintext equal the oracle's tls1_enc(s, 0)
(ssl/t1_enc.c:832-975), tampered records bad_record_mac with zero-filled
plaintext, publicly invalid and out-of-bounds records rejected; with the batch
split over many small chunks and streams (ascending layout), in place, and with
a shuffled layout (one chunk).
"""
import ctypes as C
import os
import random
import sys

import numpy as np
import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle as po  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ta():
    import talos_amd
    talos_amd.load_library()
    return talos_amd


@pytest.fixture(scope="module")
def engine(ta):
    e = ta.Engine(0)
    yield e
    e.close()


def _pinned(engine, nbytes, keep):
    p = C.c_void_p()
    assert engine.lib.tlsgpu_host_alloc(engine.handle, max(nbytes, 1), C.byref(p)) == 0
    keep.append(p.value)
    return p.value


@pytest.mark.parametrize("layout", ["ascending", "in_place", "shuffled"])
def test_open_host_matches_oracle(ta, engine, oracle, layout):
    rnd = random.Random(61)
    kinds = [po.AES_128_GCM, po.AES_256_GCM, po.CHACHA20_POLY1305, po.AES_128_GCM]
    params = []
    for k in kinds:
        params.append(ta.SessionParams(k, bytes(rnd.getrandbits(8) for _ in range(po.KEY_LEN[k])),
                                       bytes(rnd.getrandbits(8) for _ in range(po.FIXED_IV_LEN[k]))))
    table = ta.SessionTable(engine, len(params))
    table.install(0, params)
    osess = [oracle.tls_session(p.aead, p.key, p.fixed_iv) for p in params]
    lengths = [rnd.choice([0, 1, 15, 16, 100, 1000, 1400, 4096, 16384]) for _ in range(300)]
    recs = []
    for i, ln in enumerate(lengths):
        sid = (i // 7) % len(params)
        seq = rnd.getrandbits(64)
        pt = bytes(rnd.getrandbits(8) for _ in range(ln))
        body = bytearray(oracle.tls_seal(osess[sid], seq, 23, pt))
        if i % 11 == 5:
            body[rnd.randrange(len(body))] ^= 0x10
        if i % 53 == 7:
            body = body[:5]     # shorter than explicit nonce / tag
        recs.append((sid, seq, pt, bytes(body)))
    order = list(range(len(recs)))
    if layout == "shuffled":
        rnd.shuffle(order)      # offsets no longer ascend with the record index
    # host layout: fragments packed in `order`, plaintext slots likewise
    in_off, out_off, ip, op = [0] * len(recs), [0] * len(recs), 0, 0
    for i in order:
        ip += (-ip) % 16 + 3
        in_off[i] = ip
        ip += len(recs[i][3])
        op += (-op) % 16
        out_off[i] = op
        op += len(recs[i][2]) + 1
    keep = []
    in_bytes, out_bytes = ip + 64, op + 64
    h_in = _pinned(engine, in_bytes, keep)
    h_out = h_in if layout == "in_place" else _pinned(engine, out_bytes, keep)
    h_recs = _pinned(engine, 32 * len(recs), keep)
    h_status = _pinned(engine, 4 * len(recs), keep)
    inbuf = (C.c_uint8 * in_bytes).from_address(h_in)
    descs = np.zeros(len(recs), dtype=ta.RECORD_DTYPE)
    for i, (sid, seq, pt, body) in enumerate(recs):
        C.memmove(h_in + in_off[i], body, len(body))
        eiv = 8 if params[sid].aead in (po.AES_128_GCM, po.AES_256_GCM) else 0
        o = in_off[i] + eiv if layout == "in_place" else out_off[i]
        descs[i] = (in_off[i], o, seq, sid, ta.len_type(len(body), 23))
    descs[3]["in_off"] = in_bytes - 4          # out of bounds
    C.memmove(h_recs, descs.tobytes(), descs.nbytes)
    if layout == "ascending":
        ta.host_pipeline(engine, 4, 64 << 10)      # many chunks over 4 streams
    try:
        ta.open_host(table, h_recs, len(recs), h_in, in_bytes, h_out,
                     in_bytes if layout == "in_place" else out_bytes, h_status)
    finally:
        ta.host_pipeline(engine, 2, 32 << 20)
    st = np.ctypeslib.as_array((C.c_int32 * len(recs)).from_address(h_status))
    for i, (sid, seq, pt, body) in enumerate(recs):
        if i == 3:
            assert st[i] == ta.REC_OUT_OF_BOUNDS
            continue
        est, exp = oracle.tls_open(osess[sid], seq, 23, body)
        want = len(exp) if est == 1 else (-1 if est == -1 else -2)
        assert st[i] == want, (i, st[i], want)
        if est == 0:
            continue
        o = int(descs[i]["out_off"])
        got = C.string_at(h_out + o, len(pt))
        assert got == (pt if est == 1 else bytes(len(pt))), i
    del inbuf
    for p in keep:
        engine.lib.tlsgpu_host_free(engine.handle, p)
    table.close()


def test_seal_host_matches_oracle(ta, engine, oracle):
    """tlsgpu_seal_host against the oracle's tls1_enc(s, 1), read back in place
    through tlsgpu_open_host.  (The TaLoS hooks these calls fire:
    tests/test_talos_hooks.py.)"""
    rnd = random.Random(67)
    kinds = [po.AES_128_GCM, po.CHACHA20_POLY1305, po.AES_256_GCM]
    params = [ta.SessionParams(k, bytes(rnd.getrandbits(8) for _ in range(po.KEY_LEN[k])),
                               bytes(rnd.getrandbits(8) for _ in range(po.FIXED_IV_LEN[k])))
              for k in kinds]
    table = ta.SessionTable(engine, len(params))
    table.install(0, params)
    osess = [oracle.tls_session(p.aead, p.key, p.fixed_iv) for p in params]
    recs, ip, op = [], 0, 0
    for i in range(120):
        ln = rnd.choice([0, 1, 17, 1400, 4096, 16384])
        sid = i % len(params)
        pt = bytes(rnd.getrandbits(8) for _ in range(ln))
        recs.append((sid, rnd.getrandbits(64), pt, ip, op))
        ip += ln + (-ln) % 16 + 5
        op += ln + 8 + 16 + (-(ln + 24)) % 16 + 16
    keep = []
    in_bytes, out_bytes = ip + 64, op + 64
    h_in, h_out = _pinned(engine, in_bytes, keep), _pinned(engine, out_bytes, keep)
    h_recs, h_status = _pinned(engine, 32 * len(recs), keep), _pinned(engine, 4 * len(recs), keep)
    descs = np.zeros(len(recs), dtype=ta.RECORD_DTYPE)
    for i, (sid, seq, pt, io, oo) in enumerate(recs):
        C.memmove(h_in + io, pt, len(pt))
        descs[i] = (io, oo, seq, sid, ta.len_type(len(pt), 23))
    C.memmove(h_recs, descs.tobytes(), descs.nbytes)
    ta.seal_host(table, h_recs, len(recs), h_in, in_bytes, h_out, out_bytes, h_status)
    st = np.ctypeslib.as_array((C.c_int32 * len(recs)).from_address(h_status)).copy()
    bodies = []
    for i, (sid, seq, pt, io, oo) in enumerate(recs):
        exp = oracle.tls_seal(osess[sid], seq, 23, pt)
        assert st[i] == len(exp), (i, st[i])
        assert C.string_at(h_out + oo, len(exp)) == exp, i
        bodies.append(exp)
    odescs = descs.copy()
    for i, (sid, seq, pt, io, oo) in enumerate(recs):
        eiv = 8 if params[sid].aead in (po.AES_128_GCM, po.AES_256_GCM) else 0
        odescs[i] = (oo, oo + eiv, seq, sid, ta.len_type(len(bodies[i]), 23))
    C.memmove(h_recs, odescs.tobytes(), odescs.nbytes)
    ta.open_host(table, h_recs, len(recs), h_out, out_bytes, h_out, out_bytes, h_status)
    st = np.ctypeslib.as_array((C.c_int32 * len(recs)).from_address(h_status)).copy()
    for i, (sid, seq, pt, io, oo) in enumerate(recs):
        eiv = 8 if params[sid].aead in (po.AES_128_GCM, po.AES_256_GCM) else 0
        assert st[i] == len(pt) and C.string_at(h_out + oo + eiv, len(pt)) == pt, i
    with pytest.raises(RuntimeError):
        ta.seal_host(table, h_recs, len(recs), h_in, in_bytes, h_in, in_bytes, h_status)
    for p in keep:
        engine.lib.tlsgpu_host_free(engine.handle, p)
    table.close()
