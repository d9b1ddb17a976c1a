"""GPU parity of tlsgpu_seal_wire (write-side framing) against
a model of ssl3_write_bytes + do_ssl3_write (ssl/s3_pkt.c:501-557, 560-762)
driving the oracle's tls1_enc(s, 1) (t1_enc.c:832-975).

Per connection the model splits the write at max_send_fragment (:531-536),
sends nothing for a zero-length write (:593-594), and emits per record the
5-byte header type || version || length (:662-677, :733; length = explicit
nonce + ciphertext + tag for the AEAD suites, :692-696) followed by the
sealed fragment, sequence numbers counting up from the stream's write
sequence (t1_enc.c:258-266).  Every wire byte must match; the sealed wire is
then read back by tlsgpu_open_wire (the device ssl3_get_record) and must
deliver the original application data.
"""
import os
import random
import sys

import numpy as np
import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle as po  # noqa: E402

TLS12 = 0x0303


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


def model_write(oracle, osess, data, seq, rtype, version, max_fragment):
    """ssl3_write_bytes(s, type, data, len) for an AEAD suite -> wire bytes."""
    frag = max_fragment or 16384
    out, k = bytearray(), 0
    for off in range(0, len(data), frag):       # len == 0: no record at all
        body = oracle.tls_seal(osess, seq + k, rtype, data[off:off + frag])
        out += bytes([rtype, version >> 8, version & 0xFF, len(body) >> 8, len(body) & 0xFF])
        out += body
        k += 1
    return bytes(out), k


@pytest.mark.gpu
@pytest.mark.parametrize("kind", [po.AES_128_GCM, po.AES_256_GCM, po.CHACHA20_POLY1305,
                                  po.CHACHA20_POLY1305_OLD])
def test_seal_wire_matches_do_ssl3_write(ta, engine, oracle, kind):
    rnd = random.Random(71 + kind)
    nsess = 6
    params = [ta.SessionParams(kind, bytes(rnd.getrandbits(8) for _ in range(po.KEY_LEN[kind])),
                               bytes(rnd.getrandbits(8) for _ in range(po.FIXED_IV_LEN[kind])))
              for _ in range(nsess)]
    table = ta.SessionTable(engine, nsess)
    table.install(0, params)
    osess = [oracle.tls_session(kind, p.key, p.fixed_iv) for p in params]
    sizes = [0, 1, 100, 1400, 16383, 16384, 16385, 40000, 65536, 3, 1024, 70000]
    frags = [0, 0, 0, 0, 0, 0, 0, 0, 4096, 512, 1000, 0]   # max_send_fragment (0 = 16384)
    data, streams, wire_off, data_off = bytearray(), [], 0, 0
    for i, (n, mf) in enumerate(zip(sizes, frags)):
        d = bytes(rnd.getrandbits(8) for _ in range(n))
        data_off += 3 if i % 2 else 0          # misaligned application data
        data += bytes(data_off - len(data)) + d
        sid = i % nsess
        seq = rnd.choice([0, 0xFF, 0xFFFFFFFF, rnd.getrandbits(64) & ~0xFFFF])
        rtype = 23 if i % 4 else 22
        size = ta.seal_wire_size(kind, n, mf)
        streams.append((data_off, wire_off, seq, n, sid, TLS12, rtype, 0, mf))
        data_off += n
        wire_off += size + (i % 3)            # gaps between streams' wire regions
    wire_bytes = wire_off + 16
    desc = np.array(streams, dtype=ta.WRITE_STREAM_DTYPE)
    max_records = 64
    bufs = [ta.DeviceBuffer(engine, x) for x in
            (len(data) + 16, wire_bytes, desc.nbytes, 32 * max_records, 4 * max_records,
             ta.WRITE_RESULT_DTYPE.itemsize * len(streams), 4)]
    d_data, d_wire, d_streams, d_recs, d_status, d_results, d_total = bufs
    d_data.upload(np.frombuffer(bytes(data) + bytes(16), np.uint8))
    d_wire.fill(0xA5)
    d_streams.upload(desc.view(np.uint8))
    ta.seal_wire(table, d_streams.ptr, len(streams), d_data.ptr, d_data.nbytes, d_wire.ptr,
                 wire_bytes, max_records, d_recs.ptr, d_status.ptr, d_results.ptr, d_total.ptr)
    engine.sync()
    wire = d_wire.download().tobytes()
    res = d_results.download().view(ta.WRITE_RESULT_DTYPE)
    st = d_status.download().view(np.int32)
    total = int(d_total.download().view(np.uint32)[0])
    assert total == sum(r["records"] for r in res)
    for i, (doff, woff, seq, n, sid, ver, rtype, _, mf) in enumerate(streams):
        exp, k = model_write(oracle, osess[sid], bytes(data[doff:doff + n]), seq, rtype, ver, mf)
        assert res[i]["records"] == k and res[i]["wire_len"] == len(exp), i
        assert res[i]["next_seq"] == seq + k
        assert wire[woff:woff + len(exp)] == exp, (i, n, mf)
        f = int(res[i]["first"])
        assert all(st[f + j] > 0 for j in range(k))
    # read it back with the device ssl3_get_record (tlsgpu_open_wire)
    ws = [(woff, int(res[i]["wire_len"]), sid, seq, ver, 0, 0)
          for i, (doff, woff, seq, n, sid, ver, rtype, _, mf) in enumerate(streams)]
    wdesc = np.array(ws, dtype=ta.WIRE_STREAM_DTYPE)
    d_ws = ta.DeviceBuffer(engine, wdesc.nbytes)
    d_ws.upload(wdesc.view(np.uint8))
    d_wres = ta.DeviceBuffer(engine, ta.WIRE_RESULT_DTYPE.itemsize * len(ws))
    ta.open_wire(table, d_ws.ptr, len(ws), d_wire.ptr, max_records, d_recs.ptr, d_status.ptr,
                 d_wres.ptr, d_total.ptr)
    engine.sync()
    plain = d_wire.download().tobytes()
    wres = d_wres.download().view(ta.WIRE_RESULT_DTYPE)
    recs = d_recs.download().view(ta.RECORD_DTYPE)
    st = d_status.download().view(np.int32)
    for i, (doff, woff, seq, n, sid, ver, rtype, _, mf) in enumerate(streams):
        assert wres[i]["alert"] == 0 and wres[i]["delivered"] == res[i]["records"]
        got = b"".join(plain[int(recs[int(wres[i]["first"]) + j]["out_off"]):
                             int(recs[int(wres[i]["first"]) + j]["out_off"]) +
                             int(st[int(wres[i]["first"]) + j])]
                       for j in range(int(wres[i]["records"])))
        assert got == bytes(data[doff:doff + n]), i
    for b in bufs + [d_ws, d_wres]:
        b.free()
    table.close()


def test_seal_wire_size(ta):
    """tlsgpu_seal_wire_size is host arithmetic (no GPU)."""
    assert ta.seal_wire_size(ta.AES_128_GCM, 0) == 0
    assert ta.seal_wire_size(ta.AES_128_GCM, 1) == 5 + 8 + 1 + 16
    assert ta.seal_wire_size(ta.CHACHA20_POLY1305, 16385) == 16385 + 2 * (5 + 16)
    assert ta.seal_wire_size(ta.AES_256_GCM, 10000, 4096) == 10000 + 3 * (5 + 8 + 16)
