"""Pin the CPU restatement (oracle/) to the reference's own known-answer data.

Vectors: tests/golden/aeadtests.txt (reference data file, 85 cases driven the
way tests/aeadtest.c:155-217 drives them), gcm128test.c's 20 NIST cases
(tests/gcm128test.c:855-913), chachatest.c and poly1305test.c vectors, and
record-level vectors sealed by the reference build (records.json).
"""
import hashlib
import json
import os

import pytest

import sys
from conftest import ROOT, load_aeadtests
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import pyoracle as po

GOLD = os.path.join(ROOT, "tests", "golden")


def test_aeadtests_count():
    assert len(load_aeadtests()) == 85


@pytest.mark.parametrize("case", load_aeadtests(), ids=lambda c: f"line{c['line']}-{c['AEAD']}")
def test_aeadtests_oracle(oracle, case):
    kind = po.KIND_BY_NAME[case["AEAD"]]
    tag = case.get("TAG", b"")
    ctx = oracle.aead(kind, case["KEY"], len(tag))
    assert ctx is not None
    ok, out = oracle.seal(ctx, case["NONCE"], case["IN"], case["AD"],
                          max_out=len(case["IN"]) + 16)
    assert ok == 1
    assert out == case["CT"] + tag
    ok, back = oracle.open(ctx, case["NONCE"], out, case["AD"], max_out=len(case["IN"]))
    assert ok == 1 and back == case["IN"]
    bad = bytes([out[0] ^ 0x80]) + out[1:]
    ok, zeros = oracle.open(ctx, case["NONCE"], bad, case["AD"], max_out=len(case["IN"]))
    assert ok == 0 and zeros == bytes(len(case["IN"]))


@pytest.mark.parametrize("tv", json.load(open(os.path.join(GOLD, "gcm128_vectors.json"))),
                         ids=lambda t: f"case{t['case']}")
def test_gcm128_nist(oracle, tv):
    K, IV, P, A, Cx, T = (bytes.fromhex(tv[k]) for k in ("K", "IV", "P", "A", "C", "T"))
    ct, tag = oracle.gcm(K, IV, A, P)
    assert tag == T
    assert ct == Cx
    pt, tag2 = oracle.gcm(K, IV, A, Cx, decrypt=True)
    assert tag2 == T and pt == P


@pytest.mark.parametrize("tv", json.load(open(os.path.join(GOLD, "chacha_vectors.json"))),
                         ids=lambda t: t["desc"][:4])
def test_chacha_keystream(oracle, tv):
    ks = oracle.chacha20(bytes.fromhex(tv["key"]), bytes.fromhex(tv["iv"]), bytes(tv["len"]))
    assert ks.hex() == tv["out"]


def test_poly1305_vectors(oracle):
    v = {k: bytes.fromhex(x) for k, x in
         json.load(open(os.path.join(GOLD, "poly1305_vectors.json"))).items()}
    msg = v["nacl_msg"]
    assert oracle.poly1305(v["nacl_key"], [msg]) == v["nacl_mac"]
    cuts = [0, 32, 96, 112, 120, 124, 126, 127, 128, 129, 130, 131]  # poly1305test.c:123-135
    assert oracle.poly1305(v["nacl_key"], [msg[a:b] for a, b in zip(cuts, cuts[1:])]) == v["nacl_mac"]
    assert oracle.poly1305(v["wrap_key"], [v["wrap_msg"]]) == v["wrap_mac"]
    macs = []
    for i in range(256):
        macs.append(oracle.poly1305(bytes([i]) * 32, [bytes([i]) * i]))
    assert oracle.poly1305(v["total_key"], macs) == v["total_mac"]


def _records():
    return json.load(open(os.path.join(GOLD, "records.json")))["records"]


@pytest.mark.parametrize("r", _records(), ids=lambda r: f"{r['aead']}-{r['pt_len']}")
def test_record_vectors_oracle(oracle, r):
    from make_golden import fill_bytes  # noqa
    kind = po.KIND_BY_NAME[r["aead"]]
    key, fiv = bytes.fromhex(r["key"]), bytes.fromhex(r["fixed_iv"])
    pt = fill_bytes(r["pt_seed"], 3, r["pt_len"])
    s = oracle.tls_session(kind, key, fiv, r["version"])
    body = oracle.tls_seal(s, r["seq"], r["type"], pt)
    assert len(body) == r["body_len"]
    assert hashlib.sha256(body).hexdigest() == r["body_sha256"]
    if "body" in r:
        assert body.hex() == r["body"]
    st, back = oracle.tls_open(s, r["seq"], r["type"], body)
    assert st == 1 and back == pt
    # wrong sequence number => bad_record_mac, zero-filled plaintext
    st, z = oracle.tls_open(s, r["seq"] ^ 1, r["type"], body)
    assert st == -1 and z == bytes(len(pt))
    # truncated below the explicit nonce / tag => publicly invalid
    st, _ = oracle.tls_open(s, r["seq"], r["type"], body[:7])
    assert st == 0


def test_fill_bytes_matches_c(oracle):
    import ctypes as C
    from make_golden import fill_bytes
    oracle.lib.oracle_fill_bytes.argtypes = [C.c_uint64, C.c_uint64, C.c_void_p, C.c_size_t]
    for seed, idx, n in [(1, 0, 5), (0x5EED0001, 77, 100), (2**63 + 5, 2**40, 4099)]:
        buf = (C.c_ubyte * n)()
        oracle.lib.oracle_fill_bytes(seed, idx, buf, n)
        assert bytes(buf) == fill_bytes(seed, idx, n)


def _batches():
    return json.load(open(os.path.join(GOLD, "batch_digests.json")))["batches"]


@pytest.mark.parametrize("name", [k for k in _batches() if k.endswith("_small")])
def test_batch_digests_oracle(oracle, name):
    """The CPU restatement re-derives the reference's small seeded batch digests
    (tests/golden/batch_digests.json, made by oracle/_ref/batch_digest over the
    reference libcrypto): same sessions / seqs / plaintexts as
    talos_amd.workload, sealed, tampered, opened, hashed in record order."""
    import ctypes as C
    import numpy as np
    from talos_amd.workload import session_plan, zipf_lengths
    d = _batches()[name]
    kind = po.KIND_BY_NAME[d["aead"]]
    n, S, seed, te = d["records"], d["sessions"], d["seed"], d["tamper_every"]
    lo, hi = d.get("range", (0, n))     # a shard of a split batch: global record indices
    lengths = (zipf_lengths(n, seed) if d["lengths"] == "zipf"
               else np.full(n, d["lengths"], dtype=np.int64))
    params, _, session, seq = session_plan(kind, n, S, seed, d.get("interleave", False))
    sess = [oracle.tls_session(kind, p.key, p.fixed_iv) for p in params]
    oracle.lib.oracle_fill_bytes.argtypes = [C.c_uint64, C.c_uint64, C.c_void_p, C.c_size_t]
    eiv = 8 if kind in (po.AES_128_GCM, po.AES_256_GCM) else 0
    hs, ho, bad = hashlib.sha256(), hashlib.sha256(), 0
    for r in range(lo, hi):
        ln = int(lengths[r])
        buf = (C.c_ubyte * max(ln, 1))()
        oracle.lib.oracle_fill_bytes(seed, r, buf, ln)
        pt = bytes(buf)[:ln]
        body = bytearray(oracle.tls_seal(sess[session[r]], int(seq[r]), 23, pt))
        hs.update(body)
        if te and r % te == te // 2:
            body[eiv + (r * 7919) % (ln + 16)] ^= 1 << (r % 8)
        st, out = oracle.tls_open(sess[session[r]], int(seq[r]), 23, bytes(body))
        bad += st == -1
        ho.update(out if st == 1 else bytes(ln))
    assert hs.hexdigest() == d["sealed_sha256"]
    assert ho.hexdigest() == d["opened_sha256"]
    assert bad == d["bad_record_mac"]
