"""Framing parity against bytes made by the reference's own record layer.

tests/golden/wire_ref.json holds, for the four AEAD suites, what LibreSSL
2.4.1's unmodified libssl (oracle/_ref/libssl_ref.so, compiled from the
reference sources) put on the wire after a real handshake: do_ssl3_write ->
tls1_enc(s, 1) -> EVP_AEAD_CTX_seal (ssl/s3_pkt.c:560-762, ssl/t1_enc.c:832-975),
for a list of application writes in each direction (1 B ... 40,000 B, the last
one fragmented at 16 KiB by ssl3_write_bytes, s3_pkt.c:531-536), together with
the record state it used: the key given to EVP_AEAD_CTX_init, the
SSL_AEAD_CTX fields fixed_nonce / xor_fixed_nonce / variable_nonce_in_record
(ssl/ssl_locl.h:527-543) and s3->write_sequence.  The peer SSL object of the
same run SSL_read() every byte back (oracle/wire_capture.c).

These tests feed those exact bytes to the engine and the oracle:
  * CPU: the oracle's restatement of tls1_enc reproduces every reference
    record body and opens it (pins oracle/aead.c's framing to the reference);
  * GPU: tlsgpu_open_wire (device ssl3_get_record) opens the reference's wire,
    tlsgpu_seal_wire (device do_ssl3_write) re-creates it byte for byte, and
    the batch path (tlsgpu_open_batch / tlsgpu_seal_batch with the in-kernel
    nonce/AAD) does the same per record — rows a1, a19, a20, f1 of SURVEY.md
    §8 pinned to reference output, not to a restatement.
"""
import base64
import json
import os
import sys

import numpy as np
import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle as po  # noqa: E402

FIXTURE = os.path.join(ROOT, "tests", "golden", "wire_ref.json")
SUITES = json.load(open(FIXTURE))["suites"]
CASES = [(c, d["dir"]) for c, s in SUITES.items() for d in s["directions"]]
APP_DATA = 23
MAX_FRAG = 16384


def splitmix_fill(n: int, key: int) -> bytes:
    """oracle/wire_capture.c fill(): SplitMix64 keyed by `key`, 8 bytes per step."""
    g = np.uint64(0x9E3779B97F4A7C15)
    steps = (n + 7) // 8
    with np.errstate(over="ignore"):
        x = np.uint64(key) * g + g * np.arange(1, steps + 1, dtype=np.uint64)
        z = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    return z.astype("<u8").tobytes()[:n]


def direction(cipher, dname):
    s = SUITES[cipher]
    d = next(x for x in s["directions"] if x["dir"] == dname)
    kind = getattr(po, s["aead"])
    wire = base64.b64decode(d["wire_b64"])
    return kind, d, wire


def parse_records(wire: bytes, off: int, length: int):
    """The 5-byte headers of a write's wire region -> (type, version, body_off, body_len)."""
    out, p = [], off
    while p < off + length:
        rtype, ver, ln = wire[p], (wire[p + 1] << 8) | wire[p + 2], (wire[p + 3] << 8) | wire[p + 4]
        out.append((rtype, ver, p + 5, ln))
        p += 5 + ln
    assert p == off + length
    return out


def explicit_len(kind):
    return 8 if kind in (po.AES_128_GCM, po.AES_256_GCM) else 0


@pytest.mark.parametrize("cipher,dname", CASES)
def test_reference_wire_shape(cipher, dname):
    """Header fields and fragmenting of the reference's bytes (s3_pkt.c:531-536,
    662-696): what the device framing has to reproduce."""
    kind, d, wire = direction(cipher, dname)
    assert len(wire) == d["wire_bytes"]
    assert d["version"] == 0x0303 and d["tag_len"] == 16
    assert bytes.fromhex(d["fixed_nonce"]) == bytes.fromhex(d["fixed_nonce"])[:po.FIXED_IV_LEN[kind]]
    assert len(bytes.fromhex(d["fixed_nonce"])) == po.FIXED_IV_LEN[kind]
    seq = int(d["start_seq"], 16)
    for w in d["writes"]:
        recs = parse_records(wire, w["wire_off"], w["wire_len"])
        assert len(recs) == -(-w["len"] // MAX_FRAG)
        for j, (rtype, ver, _, ln) in enumerate(recs):
            frag = min(MAX_FRAG, w["len"] - j * MAX_FRAG)
            assert rtype == APP_DATA and ver == 0x0303
            assert ln == explicit_len(kind) + frag + 16
        seq += len(recs)
    assert seq == int(d["end_seq"], 16)


@pytest.mark.parametrize("cipher,dname", CASES)
def test_oracle_reproduces_reference_records(oracle, cipher, dname):
    """The CPU restatement of tls1_enc (oracle/aead.c, t1_enc.c:832-975) seals
    every fragment to the reference's record body and opens the body back."""
    kind, d, wire = direction(cipher, dname)
    sess = oracle.tls_session(kind, bytes.fromhex(d["key"]), bytes.fromhex(d["fixed_nonce"]))
    seq = int(d["start_seq"], 16)
    for w in d["writes"]:
        data = splitmix_fill(w["len"], w["seed"])
        for j, (_, _, boff, ln) in enumerate(parse_records(wire, w["wire_off"], w["wire_len"])):
            frag = data[j * MAX_FRAG:(j + 1) * MAX_FRAG]
            body = wire[boff:boff + ln]
            assert oracle.tls_seal(sess, seq, APP_DATA, frag) == body, (w["len"], j)
            st, pt = oracle.tls_open(sess, seq, APP_DATA, body)
            assert st == 1 and pt == frag
            seq += 1


@pytest.mark.parametrize("cipher,dname", CASES)
def test_seal_wire_size_matches_reference(cipher, dname):
    """tlsgpu_seal_wire_size (host arithmetic) equals the bytes the reference emitted."""
    import talos_amd as ta
    kind, d, _ = direction(cipher, dname)
    for w in d["writes"]:
        assert ta.seal_wire_size(kind, w["len"]) == w["wire_len"]


# ---------------------------------------------------------------------------
# GPU: the device record layer on the reference's bytes


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


def install(ta, engine, kind, d):
    table = ta.SessionTable(engine, 1)
    table.install(0, [ta.SessionParams(kind, bytes.fromhex(d["key"]),
                                       bytes.fromhex(d["fixed_nonce"]), version=d["version"])])
    return table


@pytest.mark.gpu
@pytest.mark.parametrize("cipher,dname", CASES)
def test_open_wire_on_reference_bytes(ta, engine, cipher, dname):
    """tlsgpu_open_wire frames and opens the reference's whole wire of one
    direction as one connection's read-ahead buffer (ssl3_get_record,
    s3_pkt.c:279-495): every record delivered, every plaintext the writer's."""
    kind, d, wire = direction(cipher, dname)
    table = install(ta, engine, kind, d)
    nrec = sum(len(parse_records(wire, w["wire_off"], w["wire_len"])) for w in d["writes"])
    ws = np.array([(0, len(wire), 0, int(d["start_seq"], 16), d["version"], 0, 0)],
                  dtype=ta.WIRE_STREAM_DTYPE)
    bufs = [ta.DeviceBuffer(engine, x) for x in
            (len(wire) + 16, ws.nbytes, 32 * (nrec + 4), 4 * (nrec + 4),
             ta.WIRE_RESULT_DTYPE.itemsize, 4)]
    d_wire, d_ws, d_recs, d_status, d_res, d_total = bufs
    d_wire.upload(np.frombuffer(wire + bytes(16), np.uint8))
    d_ws.upload(ws.view(np.uint8))
    ta.open_wire(table, d_ws.ptr, 1, d_wire.ptr, nrec + 4, d_recs.ptr, d_status.ptr, d_res.ptr,
                 d_total.ptr)
    engine.sync()
    res = d_res.download().view(ta.WIRE_RESULT_DTYPE)[0]
    assert res["alert"] == 0 and res["records"] == nrec and res["delivered"] == nrec
    assert res["consumed"] == len(wire)
    plain = d_wire.download().tobytes()
    recs = d_recs.download().view(ta.RECORD_DTYPE)
    st = d_status.download().view(np.int32)
    got = b"".join(plain[int(recs[res["first"] + j]["out_off"]):
                         int(recs[res["first"] + j]["out_off"]) + int(st[res["first"] + j])]
                   for j in range(nrec))
    assert got == b"".join(splitmix_fill(w["len"], w["seed"]) for w in d["writes"])
    for b in bufs:
        b.free()
    table.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cipher,dname", CASES)
def test_seal_wire_reproduces_reference_bytes(ta, engine, cipher, dname):
    """tlsgpu_seal_wire (ssl3_write_bytes + do_ssl3_write on the device), given
    the same application writes and the reference's write sequence, emits the
    reference's wire byte for byte."""
    kind, d, wire = direction(cipher, dname)
    table = install(ta, engine, kind, d)
    data, streams, seq = bytearray(), [], int(d["start_seq"], 16)
    for w in d["writes"]:
        nrec = -(-w["len"] // MAX_FRAG)
        streams.append((len(data), w["wire_off"], seq, w["len"], 0, d["version"], APP_DATA, 0, 0))
        data += splitmix_fill(w["len"], w["seed"])
        seq += nrec
    desc = np.array(streams, dtype=ta.WRITE_STREAM_DTYPE)
    max_records = seq - int(d["start_seq"], 16) + 4
    bufs = [ta.DeviceBuffer(engine, x) for x in
            (len(data) + 16, len(wire) + 16, desc.nbytes, 32 * max_records, 4 * max_records,
             ta.WRITE_RESULT_DTYPE.itemsize * len(streams), 4)]
    d_data, d_wire, d_streams, d_recs, d_status, d_results, d_total = bufs
    d_data.upload(np.frombuffer(bytes(data) + bytes(16), np.uint8))
    d_wire.fill(0xA5)
    d_streams.upload(desc.view(np.uint8))
    ta.seal_wire(table, d_streams.ptr, len(streams), d_data.ptr, d_data.nbytes, d_wire.ptr,
                 len(wire) + 16, max_records, d_recs.ptr, d_status.ptr, d_results.ptr, d_total.ptr)
    engine.sync()
    got = d_wire.download().tobytes()
    res = d_results.download().view(ta.WRITE_RESULT_DTYPE)
    for i, w in enumerate(d["writes"]):
        assert int(res[i]["wire_len"]) == w["wire_len"]
    assert got[:len(wire)] == wire
    assert int(res[-1]["next_seq"]) == int(d["end_seq"], 16)
    for b in bufs:
        b.free()
    table.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cipher,dname", CASES)
def test_batch_path_on_reference_records(ta, engine, cipher, dname):
    """The batch ABI's in-kernel framing (nonce and 13-byte AAD from the
    descriptor's seq and type, t1_enc.c:841-948) on the reference's records:
    tlsgpu_open_batch opens each body, tlsgpu_seal_batch re-seals each
    fragment to the reference's body."""
    kind, d, wire = direction(cipher, dname)
    table = install(ta, engine, kind, d)
    ex = explicit_len(kind)
    seq = int(d["start_seq"], 16)
    open_desc, seal_desc, frags = [], [], bytearray()
    for w in d["writes"]:
        data = splitmix_fill(w["len"], w["seed"])
        for j, (_, _, boff, ln) in enumerate(parse_records(wire, w["wire_off"], w["wire_len"])):
            frag = data[j * MAX_FRAG:(j + 1) * MAX_FRAG]
            open_desc.append((boff, boff, seq, 0, ta.len_type(ln, APP_DATA)))
            seal_desc.append((len(frags), boff, seq, 0, ta.len_type(len(frag), APP_DATA)))
            frags += frag
            seq += 1
    n = len(open_desc)
    od = np.array(open_desc, dtype=ta.RECORD_DTYPE)
    sd = np.array(seal_desc, dtype=ta.RECORD_DTYPE)
    d_wire = ta.DeviceBuffer(engine, len(wire) + 16)
    d_plain = ta.DeviceBuffer(engine, len(wire) + 16)
    d_frags = ta.DeviceBuffer(engine, len(frags) + 16)
    d_sealed = ta.DeviceBuffer(engine, len(wire) + 16)
    d_od, d_sd = ta.DeviceBuffer(engine, od.nbytes), ta.DeviceBuffer(engine, sd.nbytes)
    d_st = ta.DeviceBuffer(engine, 4 * n)
    d_wire.upload(np.frombuffer(wire + bytes(16), np.uint8))
    d_frags.upload(np.frombuffer(bytes(frags) + bytes(16), np.uint8))
    d_od.upload(od.view(np.uint8))
    d_sd.upload(sd.view(np.uint8))
    d_sealed.fill(0)
    # open out of place: plaintext at the body offset of a second buffer
    ta.open_batch(table, d_od.ptr, n, d_wire.ptr, len(wire), d_plain.ptr, len(wire), d_st.ptr)
    engine.sync()
    st = d_st.download().view(np.int32).copy()
    plain = d_plain.download().tobytes()
    k = 0
    for r, (boff, _, _, _, lt) in enumerate(open_desc):
        ln = lt & 0xFFFFFF
        assert st[r] == ln - ex - 16, r
        assert plain[boff:boff + st[r]] == bytes(frags[k:k + st[r]]), r
        k += int(st[r])
    ta.seal_batch(table, d_sd.ptr, n, d_frags.ptr, len(frags), d_sealed.ptr, len(wire), d_st.ptr)
    engine.sync()
    st = d_st.download().view(np.int32)
    sealed = d_sealed.download().tobytes()
    for r, (boff, _, _, _, lt) in enumerate(open_desc):
        ln = lt & 0xFFFFFF
        assert st[r] == ln, r
        assert sealed[boff:boff + ln] == wire[boff:boff + ln], r
    for b in (d_wire, d_plain, d_frags, d_sealed, d_od, d_sd, d_st):
        b.free()
    table.close()
