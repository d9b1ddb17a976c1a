"""Full-size parity against the reference: the seeded
BASELINE batches B (64 Ki x 16 KiB AES-128-GCM), C (1 Mi x 1,400 B
ChaCha20-Poly1305), D (256 Ki Zipf AES-256-GCM) and the session-count variants
S = 1 and S = #records are built on the device (talos_amd.workload), sealed by
the HIP path, hashed, tampered 1 in 1,024, opened by the HIP path and hashed
again.  Both SHA-256 digests must equal the ones the reference LibreSSL
computed on the same batch in the build container
(tests/golden/batch_digests.json, oracle/batch_digest.c over the reference
libcrypto) — bit-exact bodies and plaintexts, zero-filled tamper set.

Also: every record of tests/golden/records.json (sealed by the reference
itself, 0 B - 16 KiB, all four AEADs) is sealed and opened by the HIP path.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu
GOLD = os.path.join(ROOT, "tests", "golden")


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


def _batches():
    return json.load(open(os.path.join(GOLD, "batch_digests.json")))["batches"]


@pytest.mark.parametrize("name", ["B", "C", "D", "B_S1", "B_Sn", "B_inter", "D_inter", "old_small",
                                  "D_small", "inter_small", "E_shard_small"] +
                         [f"E_shard{r}" for r in range(8)] + ["B:hinted", "D:hinted"])
def test_batch_digest_matches_reference(ta, engine, name):
    """E_shard<r>: config E is one 524,288-record batch split
    across 8 GPUs; each of its 8 shards is built here, on one GPU, exactly as
    GPU r builds it under bench.py --gpus 8, and must reproduce the reference's
    digest of that slice of the batch."""
    from talos_amd.workload import Workload, zipf_lengths
    # ":hinted": the batch-shape hints bench.py states (talos_amd.batch_hints),
    # so B and D run the fused queue kernel (engine.cpp run_batch `fused`)
    name, _, hinted = name.partition(":")
    d = _batches()[name]
    kind = ta.AEAD_NAMES[d["aead"]]
    n, S, seed, te = d["records"], d["sessions"], d["seed"], d["tamper_every"]
    lo, hi = d.get("range", (0, n))
    zipf = d["lengths"] == "zipf"
    wl = Workload(engine, kind, n, S, seed, lengths=zipf_lengths(n, seed)[lo:hi] if zipf else None,
                  record_len=0 if zipf else d["lengths"], interleave=d.get("interleave", False),
                  shard=(lo, hi))
    try:
        if hinted:
            wl.table.hint(ta.batch_hints(wl.lengths + ta.EXPLICIT_NONCE_LEN[kind] + ta.TAG_LEN,
                                         wl.session, seal=False))
        assert int(wl.lengths.sum()) == d["payload_bytes"]
        assert wl.sealed_digest() == d["sealed_sha256"], "sealed bodies differ from the reference"
        wl.apply_tamper(te)
        wl.open()
        engine.sync()
        st = wl.status()
        assert int((st == -1).sum()) == d["bad_record_mac"]
        assert np.array_equal(st, np.where(wl.tampered, -1, wl.lengths).astype(np.int32))
        assert wl.opened_digest() == d["opened_sha256"], "opened plaintexts differ"
    finally:
        wl.free()


def test_reference_record_vectors_on_gpu(ta, engine):
    """records.json: the reference's own sealed records, through the batch path."""
    import sys
    sys.path.insert(0, GOLD)
    from make_golden import fill_bytes
    from talos_amd.batch import RecordBatch
    recs = json.load(open(os.path.join(GOLD, "records.json")))["records"]
    table = ta.SessionTable(engine, len(recs))
    table.install(0, [ta.SessionParams(ta.AEAD_NAMES[r["aead"]], bytes.fromhex(r["key"]),
                                       bytes.fromhex(r["fixed_iv"]), 0, r["version"])
                      for r in recs])
    pts = [fill_bytes(r["pt_seed"], 3, r["pt_len"]) for r in recs]
    sb = RecordBatch(engine, [(i, r["seq"], r["type"], pt, ta.AEAD_NAMES[r["aead"]])
                              for i, (r, pt) in enumerate(zip(recs, pts))], "seal")
    sb.run(table)
    bodies = []
    for (st, body), r in zip(sb.results(), recs):
        assert st == r["body_len"] and hashlib.sha256(body).hexdigest() == r["body_sha256"]
        if "body" in r:
            assert body.hex() == r["body"]
            body = bytes.fromhex(r["body"])     # open the reference's own bytes
        bodies.append(body)
    ob = RecordBatch(engine, [(i, r["seq"], r["type"], b, ta.AEAD_NAMES[r["aead"]])
                              for i, (r, b) in enumerate(zip(recs, bodies))], "open")
    ob.run(table)
    for (st, pt), want in zip(ob.results(), pts):
        assert st == len(want) and pt == want
    table.close()
