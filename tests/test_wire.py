"""GPU parity of tlsgpu_open_wire against a model of
ssl3_get_record (ssl/s3_pkt.c:279-495) driving the oracle's tls1_enc(s, 0).

Each stream is one connection's read-ahead bytes.  The model below restates the
reference's per-record loop: header checks (version :319-329, major :331-335,
rbuf overflow :337-341), wait for a complete fragment (:346-354), encrypted
length limit (:376-380), enc() = 0 -> decryption_failed (:385-390), -1 ->
bad_record_mac (:450-462), plaintext > 16384 -> record_overflow (:465-469); the
first failure ends the connection.  Plaintexts, zero-fill on bad MAC, per
record statuses and per stream alerts must match exactly.
"""
import os
import random
import sys

import numpy as np
import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle as po  # noqa: E402

pytestmark = pytest.mark.gpu

RBUF_DEFAULT = 16384 + 320 + 5 + 3
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


def header(rtype, version, length):
    return bytes([rtype, version >> 8, version & 0xFF, length >> 8, length & 0xFF])


def model_stream(oracle, osess, kind, wire, version, first_packet, rbuf_len, seq0):
    """ssl3_get_record over one stream -> (records[(status, pt)], consumed, alert, alert_rec, delivered)."""
    rbuf = rbuf_len or RBUF_DEFAULT
    framed, pos, alert = [], 0, 0
    while pos + 5 <= len(wire):
        rtype, ver, ln = wire[pos], (wire[pos + 1] << 8) | wire[pos + 2], (wire[pos + 3] << 8) | wire[pos + 4]
        if not first_packet and ver != version:
            alert = 70
            break
        if ver >> 8 != 3:
            alert = -1
            break
        if ln > rbuf - 5:
            alert = 22
            break
        if pos + 5 + ln > len(wire):
            break
        if ln > 16704:
            alert = 22
            break
        framed.append((pos, rtype, ln))
        pos += 5 + ln
    consumed = pos
    out, dead, alert_rec, delivered = [], False, len(framed), len(framed)
    for i, (p, rtype, ln) in enumerate(framed):
        if dead:
            out.append((-3, None))
            continue
        frag = bytes(wire[p + 5:p + 5 + ln])
        if osess is None:
            est, pt = 0, b""
        else:
            est, pt = oracle.tls_open(osess, seq0 + i, rtype, frag)
        if est == -1:
            st, a = -1, 20
        elif est == 0:
            st, a = -2, 21
        elif len(pt) > 16384:
            st, a = -4, 22
        else:
            st, a = len(pt), 0
        out.append((st, pt if st >= 0 else None))
        if a:
            dead, alert, alert_rec, delivered = True, a, i, i
    return out, consumed, alert, alert_rec, delivered


def build_streams(oracle, ta, rnd, kind):
    """Good, tampered, malformed and truncated streams of one AEAD kind."""
    key = bytes(rnd.randrange(256) for _ in range(po.KEY_LEN[kind]))
    fiv = bytes(rnd.randrange(256) for _ in range(po.FIXED_IV_LEN[kind]))
    params = ta.SessionParams(kind, key, fiv)
    osess = oracle.tls_session(kind, key, fiv)

    def rec(seq, n, rtype=23, version=TLS12):
        pt = bytes(rnd.randrange(256) for _ in range(n))
        body = oracle.tls_seal(osess, seq, rtype, pt)
        return header(rtype, version, len(body)) + body

    def stream(parts, seq0, version=TLS12, first_packet=False, rbuf_len=0, session=0):
        return dict(wire=b"".join(parts), seq=seq0, version=version, first=first_packet,
                    rbuf=rbuf_len, session=session)

    S = []
    q = rnd.randrange(1 << 40)
    # good records of mixed lengths + 3 trailing bytes of the next header
    S.append(stream([rec(q, 0), rec(q + 1, 1), rec(q + 2, 1400), rec(q + 3, 16384), rec(q + 4, 7),
                     header(23, TLS12, 100)[:3]], q))
    # tampered 4th record: bad_record_mac, the rest skipped
    q = rnd.randrange(1 << 40)
    parts = [rec(q + i, rnd.randrange(1, 3000)) for i in range(6)]
    b = bytearray(parts[3])
    b[5 + rnd.randrange(len(b) - 5)] ^= 0x10
    parts[3] = bytes(b)
    S.append(stream(parts, q))
    # wrong version on the 3rd header -> protocol_version
    q = rnd.randrange(1 << 40)
    S.append(stream([rec(q, 50), rec(q + 1, 60), rec(q + 2, 70, version=0x0301)], q))
    # first packet: any version accepted
    q = rnd.randrange(1 << 40)
    S.append(stream([rec(q, 33, version=0x0301), rec(q + 1, 44, version=0x0302)], q,
                    first_packet=True))
    # major version 2 -> error without alert
    q = rnd.randrange(1 << 40)
    S.append(stream([rec(q, 20), header(23, 0x0203, 40) + bytes(40)], q))
    # length above rbuf: overflow at the header even without the fragment
    S.append(stream([header(23, TLS12, 16708) + bytes(10)], 0))
    # 16704 < length <= rbuf - 5, full fragment: overflow after the read
    S.append(stream([header(23, TLS12, 16705) + bytes(16705)], 0))
    # fragment shorter than explicit nonce + tag: decryption_failed
    S.append(stream([rec(9, 5), header(23, TLS12, 10) + bytes(10)], 9))
    # plaintext longer than 16384 (fragment within 16704): record_overflow
    q = rnd.randrange(1 << 40)
    S.append(stream([rec(q, 100), rec(q + 1, 16400), rec(q + 2, 10)], q))
    # the last record's fragment is incomplete: framed up to it
    q = rnd.randrange(1 << 40)
    last = rec(q + 2, 900)
    S.append(stream([rec(q, 10), rec(q + 1, 20), last[:400]], q))
    # small rbuf: overflow check uses it
    q = rnd.randrange(1 << 40)
    S.append(stream([rec(q, 100), rec(q + 1, 2000)], q, rbuf_len=1024))
    # unknown session: framed, publicly invalid -> decryption_failed
    S.append(stream([rec(5, 10)], 5, session=7))
    return params, osess, S


def run_wire(ta, engine, table, streams, max_records):
    wire = bytearray()
    descs = np.zeros(len(streams), dtype=ta.WIRE_STREAM_DTYPE)
    offs = []
    for i, s in enumerate(streams):
        wire += bytes((-len(wire) - 5) % 16)  # fragments 16-B aligned (any alignment works)
        offs.append(len(wire))
        descs[i] = (len(wire), len(s["wire"]), s["session"], s["seq"], s["version"],
                    ta.WIRE_FIRST_PACKET if s["first"] else 0, s["rbuf"])
        wire += s["wire"]
    d_wire = ta.DeviceBuffer(engine, len(wire) + 64)
    d_wire.upload(bytes(wire) + bytes(64))
    d_streams = ta.DeviceBuffer(engine, descs.nbytes)
    d_streams.upload(descs.view(np.uint8))
    d_recs = ta.DeviceBuffer(engine, 32 * max(max_records, 1))
    d_status = ta.DeviceBuffer(engine, 4 * max(max_records, 1))
    d_results = ta.DeviceBuffer(engine, 32 * len(streams))
    d_total = ta.DeviceBuffer(engine, 4)
    ta.open_wire(table, d_streams.ptr, len(streams), d_wire.ptr, max_records, d_recs.ptr,
                 d_status.ptr, d_results.ptr, d_total.ptr)
    engine.sync()
    out = dict(wire=d_wire.download()[:len(wire)].tobytes(), offs=offs,
               status=d_status.download().view(np.int32)[:max_records].copy(),
               results=d_results.download().view(ta.WIRE_RESULT_DTYPE).copy(),
               total=int(d_total.download().view(np.uint32)[0]),
               recs=d_recs.download().view(ta.RECORD_DTYPE)[:max_records].copy())
    for b in (d_wire, d_streams, d_recs, d_status, d_results, d_total):
        b.free()
    return out


@pytest.mark.parametrize("kind", [po.AES_128_GCM, po.AES_256_GCM, po.CHACHA20_POLY1305,
                                  po.CHACHA20_POLY1305_OLD])
def test_open_wire_matches_ssl3_get_record(ta, engine, oracle, kind):
    rnd = random.Random(100 + kind)
    params, osess, streams = build_streams(oracle, ta, rnd, kind)
    table = ta.SessionTable(engine, 1)
    table.install(0, [params])
    got = run_wire(ta, engine, table, streams, max_records=256)
    check_against_model(oracle, osess, kind, streams, got)
    table.close()


def check_against_model(oracle, osess, kind, streams, got):
    """Every stream's result, descriptors, statuses and opened bytes equal the
    ssl3_get_record model (model_stream)."""
    eiv = 8 if kind in (po.AES_128_GCM, po.AES_256_GCM) else 0
    total = 0
    for i, s in enumerate(streams):
        recs, consumed, alert, alert_rec, delivered = model_stream(
            oracle, osess if s["session"] == 0 else None, kind, s["wire"], s["version"], s["first"],
            s["rbuf"], s["seq"])
        r = got["results"][i]
        assert int(r["records"]) == len(recs), (i, r)
        assert int(r["consumed"]) == consumed, (i, r)
        assert int(r["alert"]) == alert, (i, r)
        assert int(r["delivered"]) == delivered, (i, r)
        assert int(r["alert_record"]) == alert_rec, (i, r)
        total += len(recs)
        pos = 0
        for k, (st, pt) in enumerate(recs):
            idx = int(r["first"]) + k
            assert int(got["status"][idx]) == st, (i, k, int(got["status"][idx]), st)
            d = got["recs"][idx]
            assert int(d["seq"]) == s["seq"] + k and int(d["session"]) == s["session"]
            ln = int(d["len_type"]) & 0xFFFFFF
            frag_off = got["offs"][i] + pos + 5
            assert int(d["in_off"]) == frag_off
            if st >= 0:
                assert got["wire"][frag_off + eiv:frag_off + eiv + st] == pt, (i, k)
            elif st == -1:
                n = ln - eiv - 16
                assert got["wire"][frag_off + eiv:frag_off + eiv + n] == bytes(n), (i, k)
            pos += 5 + ln
    assert got["total"] == total


def test_open_wire_long_runs(ta, engine, oracle):
    """Streams longer than the framing kernel's 16 KiB window and its 64
    speculative headers: equal-length runs accepted in bulk, runs broken by a
    different length, a failing header or a tampered record inside a run, and
    16 KiB records (the finish kernel's 64-record status chunks included)."""
    rnd = random.Random(77)
    kind = po.AES_128_GCM
    key = bytes(rnd.randrange(256) for _ in range(16))
    fiv = bytes(rnd.randrange(256) for _ in range(4))
    params = ta.SessionParams(kind, key, fiv)
    osess = oracle.tls_session(kind, key, fiv)

    def recs(seq0, lens, version=TLS12):
        out = []
        for i, n in enumerate(lens):
            body = oracle.tls_seal(osess, seq0 + i, 23, bytes(rnd.randrange(256) for _ in range(n)))
            out.append(header(23, version, len(body)) + body)
        return out

    def stream(parts, seq0):
        return dict(wire=b"".join(parts), seq=seq0, version=TLS12, first=False, rbuf=0, session=0)

    S = []
    lens = [100] * 150 + [7, 3000, 1] + [1400] * 70 + [0] * 5 + [rnd.randrange(0, 2000) for _ in range(40)]
    S.append(stream(recs(10, lens), 10))
    parts = recs(500, [300] * 140)  # wrong version at record 100, inside a run
    parts[100] = recs(600, [300], version=0x0301)[0]
    S.append(stream(parts, 500))
    parts = recs(1000, [64] * 200)  # tampered record 130: bad_record_mac, 131.. skipped
    b = bytearray(parts[130])
    b[20] ^= 1
    parts[130] = bytes(b)
    S.append(stream(parts, 1000))
    S.append(stream(recs(2000, [16384] * 20 + [16000]), 2000))
    parts = recs(3000, [200] * 90)  # record 70 claims more than rbuf: overflow at its header
    parts[70] = header(23, TLS12, 16708) + parts[70][5:]
    S.append(stream(parts, 3000))
    S.append(stream(recs(4000, [50] * 100) + [recs(4100, [900])[0][:300]], 4000))  # incomplete tail
    # more records than the framing kernel's per-stream list (kList = 1024): second walk
    long_lens = [rnd.randrange(0, 40) for _ in range(1100)]
    S.append(stream(recs(6000, long_lens), 6000))
    table = ta.SessionTable(engine, 1)
    table.install(0, [params])
    got = run_wire(ta, engine, table, S, max_records=4096)
    check_against_model(oracle, osess, kind, S, got)
    # capacity cut inside a bulk run: every stream is framed up to what fits
    got = run_wire(ta, engine, table, S[:1], max_records=90)
    r = got["results"][0]
    assert int(r["records"]) == 90 and int(r["alert"]) == 0 and got["total"] == len(lens)
    assert int(r["consumed"]) == sum(5 + 8 + n + 16 for n in lens[:90])
    assert all(int(x) >= 0 for x in got["status"][:90])
    # capacity cut in the second-walk path
    got = run_wire(ta, engine, table, S[-1:], max_records=1050)
    r = got["results"][0]
    assert int(r["records"]) == 1050 and int(r["alert"]) == 0 and got["total"] == len(long_lens)
    assert int(r["consumed"]) == sum(5 + 8 + n + 16 for n in long_lens[:1050])
    assert all(int(x) >= 0 for x in got["status"][:1050])
    table.close()


def test_open_wire_capacity_truncates_at_record_boundary(ta, engine, oracle):
    rnd = random.Random(5)
    kind = po.AES_128_GCM
    key, fiv = bytes(range(16)), bytes(4)
    params = ta.SessionParams(kind, key, fiv)
    osess = oracle.tls_session(kind, key, fiv)
    streams = []
    for s in range(4):
        parts = []
        for k in range(5):
            pt = bytes(rnd.randrange(256) for _ in range(rnd.randrange(1, 500)))
            body = oracle.tls_seal(osess, 1000 * s + k, 23, pt)
            parts.append(header(23, TLS12, len(body)) + body)
        streams.append(dict(wire=b"".join(parts), seq=1000 * s, version=TLS12, first=False, rbuf=0,
                            session=0))
    table = ta.SessionTable(engine, 1)
    table.install(0, [params])
    got = run_wire(ta, engine, table, streams, max_records=12)
    recs = got["results"]["records"]
    assert int(recs.sum()) == 12 and got["total"] == 20
    for i, s in enumerate(streams):
        r = got["results"][i]
        n = int(r["records"])
        assert int(r["alert"]) == 0 and int(r["delivered"]) == n
        # consumed covers exactly the n framed records
        pos = 0
        for _ in range(n):
            pos += 5 + ((s["wire"][pos + 3] << 8) | s["wire"][pos + 4])
        assert int(r["consumed"]) == pos
        for k in range(n):
            assert int(got["status"][int(r["first"]) + k]) >= 0
    table.close()
