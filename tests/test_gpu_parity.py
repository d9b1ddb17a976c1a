"""GPU parity: libtlsgpu.so (HIP, gfx950) against the oracle, bit-exact.

Mirrors the reference's own tests: tests/aeadtest.c (seal -> compare CT/TAG,
open -> compare PT, flip a bit -> open must fail) through the drop-in EVP ABI,
and record-level checks of tls1_enc's AEAD branch (ssl/t1_enc.c:832-975) for
the batch ABI: every byte of every ciphertext/tag/plaintext equal to the
oracle's, bad_record_mac with zero-filled plaintext on tampering, publicly
invalid short records, misaligned buffers, in-place decryption and
interleaved sessions.
"""
import os
import random
import sys

import numpy as np
import pytest

from conftest import ROOT, load_aeadtests

sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import pyoracle as po  # noqa: E402

pytestmark = pytest.mark.gpu

KINDS = {"aes-128-gcm": po.AES_128_GCM, "aes-256-gcm": po.AES_256_GCM,
         "chacha20-poly1305": po.CHACHA20_POLY1305,
         "chacha20-poly1305-old": po.CHACHA20_POLY1305_OLD}
LENGTHS = [0, 1, 2, 13, 15, 16, 17, 31, 32, 33, 63, 64, 65, 100, 255, 256, 511, 1000, 1023,
           1024, 1025, 1400, 2047, 4095, 4096, 8191, 16383, 16384, 16385, 20000]


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


# ---------------------------------------------------------------- EVP drop-in

@pytest.mark.parametrize("case", load_aeadtests(), ids=lambda c: f"line{c['line']}-{c['AEAD']}")
def test_evp_aeadtests(ta, case):
    """tests/aeadtest.c:155-217 through libtlsgpu.so's EVP_AEAD_* on the GPU."""
    kind = KINDS[case["AEAD"]]
    tag = case["TAG"]
    a = ta.EvpAead(kind, case["KEY"], len(tag))
    assert a.ok == 1
    ok, out, _ = a.seal(case["NONCE"], case["IN"], case["AD"], max_out=len(case["IN"]) + 16)
    assert ok == 1
    assert out == case["CT"] + tag
    ok, back, ol = a.open(case["NONCE"], out, case["AD"], max_out=len(case["IN"]))
    assert ok == 1 and back == case["IN"] and ol == len(case["IN"])
    bad = bytes([out[0] ^ 0x80]) + out[1:]
    ok, z, ol = a.open(case["NONCE"], bad, case["AD"], max_out=len(case["IN"]))
    assert ok == 0 and z == bytes(len(case["IN"])) and ol == 0
    a.cleanup()


def test_evp_error_semantics(ta):
    """evp_aead.c / e_aes.c argument checks: zero-fill + out_len 0 on failure."""
    a = ta.EvpAead(ta.AES_128_GCM, bytes(16))
    ok, out, ol = a.seal(bytes(12), b"x" * 32, b"", max_out=40)   # too small (< 32+16)
    assert ok == 0 and out == bytes(40) and ol == 0
    ok, out, ol = a.open(bytes(12), b"short", b"", max_out=8)     # in_len < tag_len
    assert ok == 0 and out == bytes(8) and ol == 0
    bad = ta.EvpAead(ta.AES_128_GCM, bytes(15))                    # wrong key size
    assert bad.ok == 0
    big_tag = ta.EvpAead(ta.AES_256_GCM, bytes(32), 17)
    assert big_tag.ok == 0
    c = ta.EvpAead(ta.CHACHA20_POLY1305, bytes(32))
    ok, out, ol = c.seal(bytes(8), b"abc", b"")                    # wrong nonce length
    assert ok == 0 and ol == 0
    # check_alias (evp_aead.c:79-87): out may alias in only at or before it
    import ctypes as C
    for fn, shift, want in ((a.lib.EVP_AEAD_CTX_seal, 1, 0), (a.lib.EVP_AEAD_CTX_seal, 0, 1),
                            (a.lib.EVP_AEAD_CTX_open, 3, 0)):
        buf = (C.c_ubyte * 256)(*([0x5A] * 256))
        base = C.addressof(buf)
        ol = C.c_size_t(99)
        ok = fn(C.byref(a.ctx), C.c_void_p(base + 16 + shift), C.byref(ol), 100,
                a._b(bytes(12)), 12, C.c_void_p(base + 16), 64, a._b(b""), 0)
        assert ok == want, (shift, ok)
        if not want:  # rejected before any cipher work: zero-filled, out_len 0
            assert bytes(buf)[16 + shift:16 + shift + 100] == bytes(100) and ol.value == 0
    a.cleanup()
    c.cleanup()


@pytest.mark.parametrize("name", ["aes-128-gcm", "aes-256-gcm"])
def test_evp_gcm_odd_ivs(ta, oracle, name):
    """Non-96-bit IVs take the GHASH(IV) path (gcm128.c:770-812)."""
    kind = KINDS[name]
    rnd = random.Random(7)
    for iv_len in (1, 8, 16, 60, 64, 77):
        key = bytes(rnd.randrange(256) for _ in range(po.KEY_LEN[kind]))
        iv = bytes(rnd.randrange(256) for _ in range(iv_len))
        pt = bytes(rnd.randrange(256) for _ in range(rnd.randrange(0, 300)))
        ad = bytes(rnd.randrange(256) for _ in range(rnd.randrange(0, 70)))
        octx = oracle.aead(kind, key)
        ok, exp = oracle.seal(octx, iv, pt, ad)
        g = ta.EvpAead(kind, key)
        ok2, got, _ = g.seal(iv, pt, ad)
        assert ok == ok2 == 1 and got == exp
        ok3, back, _ = g.open(iv, got, ad)
        assert ok3 == 1 and back == pt
        g.cleanup()


@pytest.mark.parametrize("name", ["aes-128-gcm", "aes-256-gcm"])
def test_evp_gcm_split_jobs(ta, oracle, name):
    """Raw EVP jobs run one per workgroup with the blocks split over its 16
    waves (gcm_raw_kernel): lengths around the 64-block step and the per-wave
    range boundaries, a partial last range, jobs far above a TLS record, short
    tags, odd IVs and long AAD; seal equals the oracle, open round-trips, and a
    flipped byte anywhere zero-fills the whole max_out."""
    kind = KINDS[name]
    rnd = random.Random(91)
    key = bytes(rnd.randrange(256) for _ in range(po.KEY_LEN[kind]))
    for n, iv_len, ad_len, tag_len in ((0, 12, 0, 16), (1, 12, 13, 16), (1023, 12, 13, 16),
                                       (1024, 12, 13, 16), (1025, 12, 13, 12),
                                       (2048, 1, 0, 16), (16384, 12, 13, 16),
                                       (16385, 60, 1000, 16), (65543, 12, 13, 14),
                                       (200000, 12, 17, 16), (16 * 64 * 16 * 2 + 5, 8, 300, 16)):
        iv = bytes(rnd.randrange(256) for _ in range(iv_len))
        ad = bytes(rnd.randrange(256) for _ in range(ad_len))
        pt = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes()
        octx = oracle.aead(kind, key, tag_len)
        ok, exp = oracle.seal(octx, iv, pt, ad)
        g = ta.EvpAead(kind, key, tag_len)
        ok2, got, _ = g.seal(iv, pt, ad)
        assert ok == ok2 == 1 and got == exp, (n, iv_len, ad_len, tag_len)
        ok3, back, ol = g.open(iv, got, ad)
        assert ok3 == 1 and back == pt and ol == n, n
        if n:
            bad = bytearray(got)
            bad[rnd.randrange(len(bad))] ^= 0x04
            ok4, z, ol = g.open(iv, bytes(bad), ad, max_out=n + 5)
            assert ok4 == 0 and z == bytes(n + 5) and ol == 0, n
        g.cleanup()


@pytest.mark.parametrize("name", ["chacha20-poly1305", "chacha20-poly1305-old"])
def test_evp_chacha_wave_jobs(ta, oracle, name):
    """Raw ChaCha20-Poly1305 jobs run one per wave (chacha_wave.h for the RFC
    7539 AEAD: 64 keystream blocks per pass, Poly1305 split over the lanes by
    block index mod 64 and recombined with r^1..r^64; the draft AEAD on lane
    0).  Lengths around the pass boundary (63 data blocks in pass 0, 64 after),
    AD longer than 64 Poly1305 blocks, short tags; seal equals the oracle, open
    round-trips, a flipped byte anywhere zero-fills the whole max_out."""
    kind = KINDS[name]
    rnd = random.Random(93)
    key = bytes(rnd.randrange(256) for _ in range(32))
    nlen = 12 if kind == po.CHACHA20_POLY1305 else 8
    for n, ad_len, tag_len in ((0, 0, 16), (0, 13, 16), (1, 0, 16), (15, 13, 16),
                               (1400, 13, 16), (4031, 13, 16), (4032, 13, 16), (4033, 13, 12),
                               (4096, 0, 16), (8128, 17, 16), (8129, 1024, 16),
                               (16384, 13, 16), (16400, 2049, 13), (70001, 13, 16)):
        nonce = bytes(rnd.randrange(256) for _ in range(nlen))
        ad = bytes(rnd.randrange(256) for _ in range(ad_len))
        pt = np.random.default_rng(n + 7).integers(0, 256, n, dtype=np.uint8).tobytes()
        octx = oracle.aead(kind, key, tag_len)
        ok, exp = oracle.seal(octx, nonce, pt, ad)
        g = ta.EvpAead(kind, key, tag_len)
        ok2, got, _ = g.seal(nonce, pt, ad)
        assert ok == ok2 == 1 and got == exp, (n, ad_len, tag_len)
        ok3, back, ol = g.open(nonce, got, ad)
        assert ok3 == 1 and back == pt and ol == n, n
        bad = bytearray(got)
        bad[rnd.randrange(len(bad))] ^= 0x10
        ok4, z, ol = g.open(nonce, bytes(bad), ad, max_out=n + 5)
        assert ok4 == 0 and z == bytes(n + 5) and ol == 0, n
        g.cleanup()


# ------------------------------------------------------------- batch records

def _mk_sessions(ta, rnd, kinds_per_sid):
    params = []
    for kind in kinds_per_sid:
        key = bytes(rnd.randrange(256) for _ in range(po.KEY_LEN[kind]))
        fiv = bytes(rnd.randrange(256) for _ in range(po.FIXED_IV_LEN[kind]))
        params.append(ta.SessionParams(kind, key, fiv))
    return params


def _oracle_sessions(oracle, params):
    return [oracle.tls_session(p.aead, p.key, p.fixed_iv, p.version) for p in params]


def _records(rnd, nsess, lengths, kinds, grouped=True):
    recs = []
    order = []
    for sid in range(nsess):
        for ln in lengths:
            order.append((sid, ln))
    if not grouped:
        rnd.shuffle(order)
    for sid, ln in order:
        seq = rnd.choice([0, 1, 0xFF, 0xFFFFFFFF, rnd.getrandbits(64)])
        rtype = rnd.choice([20, 21, 22, 23])
        pt = bytes(rnd.getrandbits(8) for _ in range(ln))
        recs.append((sid, seq, rtype, pt, kinds[sid]))
    return recs


def _run_seal_open(ta, engine, oracle, kinds, lengths, grouped=True, in_shift=0, out_shift=0,
                   seed=1, in_place=False, hints=0):
    """in_shift: one shift for every record's input, or a function of the record index."""
    from talos_amd.batch import RecordBatch
    rnd = random.Random(seed)
    params = _mk_sessions(ta, rnd, kinds)
    table = ta.SessionTable(engine, len(params))
    table.install(0, params)
    table.hint(hints)
    osess = _oracle_sessions(oracle, params)
    recs = _records(rnd, len(params), lengths, kinds, grouped)

    # seal on the GPU, compare with the oracle's tls1_enc(s, 1)
    if callable(in_shift):
        in_shift = [in_shift(i) for i in range(len(recs))]
    sb = RecordBatch(engine, recs, "seal", in_shift=in_shift, out_shift=out_shift)
    sb.run(table)
    bodies = []
    for (st, body), (sid, seq, rtype, pt, kind) in zip(sb.results(), recs):
        exp = oracle.tls_seal(osess[sid], seq, rtype, pt)
        assert st == len(exp), (kind, len(pt), st)
        assert body == exp, (kind, len(pt))
        bodies.append(exp)

    # open the oracle's records on the GPU; tamper every 5th
    open_recs, tampered = [], []
    for i, ((sid, seq, rtype, pt, kind), body) in enumerate(zip(recs, bodies)):
        b = bytearray(body)
        t = (i % 5 == 3) and len(b) > 0
        if t:
            pos = rnd.randrange(len(b))
            b[pos] ^= 1 << rnd.randrange(8)
        open_recs.append((sid, seq, rtype, bytes(b), kind))
        tampered.append(t)
    ob = RecordBatch(engine, open_recs, "open", in_shift=in_shift, out_shift=out_shift,
                     in_place=in_place)
    ob.run(table)
    for (st, got), (sid, seq, rtype, body, kind), t, (_, _, _, pt, _) in zip(
            ob.results(), open_recs, tampered, recs):
        est, exp = oracle.tls_open(osess[sid], seq, rtype, body)
        assert st == (len(exp) if est == 1 else (-1 if est == -1 else -2)), (kind, len(pt), st)
        if est == 1:
            assert not t or got == pt
            assert got == pt
        elif est == -1:
            assert got == bytes(len(got))
    table.close()


@pytest.mark.parametrize("name", list(KINDS))
def test_batch_seal_open_all_lengths(ta, engine, oracle, name):
    _run_seal_open(ta, engine, oracle, [KINDS[name]] * 3, LENGTHS, seed=11)


EXPERIMENTAL_IMPLS = ("hybrid", "bitslice", "fused")


@pytest.fixture
def gcm_impl(ta):
    """Run a test under one GCM kernel and restore the default afterwards.  The
    slower variants exist only in a `make EXPERIMENTAL=1` build."""
    prev = ta.get_gcm_impl()

    def use(impl):
        try:
            ta.set_gcm_impl(impl)
        except ta.TlsGpuError:
            if impl in EXPERIMENTAL_IMPLS:
                pytest.skip(f"gcm impl {impl} not built (make EXPERIMENTAL=1)")
            raise
    yield use
    ta.set_gcm_impl(prev)


@pytest.mark.parametrize("impl", ["auto", "split", "queue", "ttable", "hybrid", "bitslice", "fused"])
@pytest.mark.parametrize("name", ["aes-128-gcm", "aes-256-gcm"])
def test_batch_gcm_impls_all_lengths(ta, engine, oracle, gcm_impl, impl, name):
    gcm_impl(impl)
    _run_seal_open(ta, engine, oracle, [KINDS[name]] * 2, LENGTHS, seed=21)


@pytest.mark.parametrize("name", ["chacha20-poly1305", "aes-128-gcm"])
def test_batch_mixed_alignment_waves(ta, engine, oracle, name):
    """Waves of 64 records whose inputs are all 16-B aligned next to waves with
    one misaligned record and all-misaligned waves (ChaCha: the sector-ring and
    line kernels take complementary waves of one batch)."""
    lengths = [1400, 1, 15, 16, 17, 63, 64, 65, 127, 128, 129, 1000, 0, 4096, 333] * 30
    shift = lambda i: 0 if (i // 64) % 3 == 0 else (i % 7 if (i // 64) % 3 == 2 else
                                                   (5 if i % 64 == 17 else 0))
    _run_seal_open(ta, engine, oracle, [KINDS[name]] * 2, lengths, seed=41, in_shift=shift)


@pytest.mark.parametrize("hints", [1, 2, 3])
def test_batch_wrong_hints_still_exact(ta, engine, oracle, gcm_impl, hints):
    """tlsgpu_sessions_hint is performance only: short records under
    NO_SHORT_RECORDS take the long-record path, interleaved sessions under
    SESSION_RUNS the run-at-a-time queue; results stay the oracle's."""
    gcm_impl("queue")
    kinds = [KINDS["aes-128-gcm"], KINDS["aes-256-gcm"]] * 3
    _run_seal_open(ta, engine, oracle, kinds, LENGTHS, grouped=False, seed=31, hints=hints)


# Long records: pairs of >= 16 KiB aligned records take the bitsliced passes
# (1024 blocks each); remainders and unpaired / misaligned records the T-tables.
BS_LENGTHS = [16384, 16384, 32768, 40000, 16384, 16400, 50000, 16384, 16384, 100, 16384,
              16384, 65536 + 17, 16384, 16384]


@pytest.mark.parametrize("impl", ["hybrid", "bitslice", "queue", "fused"])
@pytest.mark.parametrize("shift", [0, 3])
@pytest.mark.parametrize("name", ["aes-128-gcm", "aes-256-gcm"])
def test_batch_bitsliced_long_records(ta, engine, oracle, gcm_impl, name, shift, impl):
    gcm_impl(impl)
    _run_seal_open(ta, engine, oracle, [KINDS[name]] * 2, BS_LENGTHS, seed=22,
                   in_shift=shift, out_shift=shift)


@pytest.mark.parametrize("name", ["aes-128-gcm", "aes-256-gcm"])
def test_bitsliced_aes_core_ecb(ta, engine, oracle, gcm_impl, name):
    """The bitsliced AES core against the oracle's AES (aes_core.c) on random
    blocks, plus the FIPS-197 C.1 / C.3 known answers (EXPERIMENTAL build)."""
    gcm_impl("bitslice")   # skips when the experimental kernels are not built
    rnd = random.Random(31)
    kind = KINDS[name]
    klen = po.KEY_LEN[kind]
    fips_key = bytes(range(klen))
    fips_pt = bytes.fromhex("00112233445566778899aabbccddeeff")
    fips_ct = {16: "69c4e0d86a7b0430d8cdb78070b4c55a",
               32: "8ea2b7ca516745bfeafc49904b496089"}[klen]
    keys = [fips_key] + [bytes(rnd.getrandbits(8) for _ in range(klen)) for _ in range(2)]
    table = ta.SessionTable(engine, len(keys))
    table.install(0, [ta.SessionParams(kind, k, bytes(4)) for k in keys])
    nblocks = 2048 + 37   # a partial lane group at the end
    for sid, key in enumerate(keys):
        blocks = bytearray(rnd.getrandbits(8) for _ in range(16 * nblocks))
        blocks[:16] = fips_pt
        d_in = ta.DeviceBuffer(engine, len(blocks))
        d_out = ta.DeviceBuffer(engine, len(blocks))
        d_in.upload(bytes(blocks))
        ta.aes_ecb_bitsliced(table, sid, d_in.ptr, d_out.ptr, nblocks)
        engine.sync()
        got = d_out.download().tobytes()
        if sid == 0:
            assert got[:16].hex() == fips_ct
        for b in range(0, nblocks, 97):
            assert got[16 * b:16 * b + 16] == oracle.aes_encrypt(key, bytes(blocks[16 * b:16 * b + 16])), b
        d_in.free()
        d_out.free()
    table.close()


@pytest.mark.parametrize("name", ["aes-128-gcm", "chacha20-poly1305"])
def test_batch_misaligned(ta, engine, oracle, name):
    _run_seal_open(ta, engine, oracle, [KINDS[name]] * 2, [0, 5, 16, 33, 1400, 4099],
                   in_shift=3, out_shift=5, seed=12)


def test_batch_chacha_interleaved_sessions(ta, engine, oracle):
    """RFC 7539 sessions only (the fused staged kernel) with the records of 5
    sessions interleaved: most waves hold several sessions and read their keys
    from LDS, the grouped cases above take the one-session s_load keys (UKEY)."""
    _run_seal_open(ta, engine, oracle, [po.CHACHA20_POLY1305] * 5,
                   [0, 1, 15, 16, 17, 64, 65, 1400, 1401, 4096, 16384], grouped=False, seed=15)


def test_batch_interleaved_sessions_mixed_kinds(ta, engine, oracle):
    kinds = [po.AES_128_GCM, po.AES_256_GCM, po.CHACHA20_POLY1305, po.AES_128_GCM,
             po.CHACHA20_POLY1305_OLD, po.AES_256_GCM]
    _run_seal_open(ta, engine, oracle, kinds, [1, 17, 300, 1400, 5000], grouped=False, seed=13)


@pytest.mark.parametrize("name", ["aes-128-gcm", "chacha20-poly1305"])
def test_batch_open_in_place(ta, engine, oracle, name):
    _run_seal_open(ta, engine, oracle, [KINDS[name]] * 2, [0, 16, 1000, 16384], in_place=True,
                   seed=14)


def test_batch_publicly_invalid(ta, engine, oracle):
    """Fragments shorter than explicit nonce / tag: tls1_enc returns 0."""
    from talos_amd.batch import RecordBatch
    rnd = random.Random(5)
    params = _mk_sessions(ta, rnd, [po.AES_128_GCM, po.CHACHA20_POLY1305])
    table = ta.SessionTable(engine, 2)
    table.install(0, params)
    recs = [(0, 1, 23, bytes(n), po.AES_128_GCM) for n in (0, 7, 8, 23)] + \
           [(1, 1, 23, bytes(n), po.CHACHA20_POLY1305) for n in (0, 15)]
    ob = RecordBatch(engine, recs, "open")
    ob.run(table)
    assert [s for s, _ in ob.results()] == [-2] * len(recs)
    table.close()


def test_batch_repeated_fresh_batches(ta, engine, oracle, gcm_impl):
    """Back-to-back fresh batches on one stream (new tables and buffers each
    time): the queue kernels' per-record constants must never come from an
    earlier batch.  A stream-ordered-pool scratch failed this on MI355X in about
    one iteration of five; the per-stream scratch passes."""
    gcm_impl("queue")
    for it in range(24):
        name = ["aes-128-gcm", "aes-256-gcm"][it % 2]
        _run_seal_open(ta, engine, oracle, [KINDS[name]] * 2, LENGTHS[::3], seed=300 + it)


# Short-record packs (gcm_pack): runs of records with
# nb + 2 <= 64 GHASH elements share one wave.  Lengths cross the pack limit
# (992 B = 62 blocks is the longest packed plaintext), packs of up to 32 empty
# records, odd tails; every 5th record tampered (zero-fill inside a pack).
PACK_LENGTHS = [0, 0, 1, 15, 16, 17, 31, 100, 255, 991, 992, 993, 1008, 0, 3, 47, 500, 64,
                0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                0, 0, 0, 0, 2000, 12, 13, 14, 700, 800, 900, 15, 16, 16, 16, 16]


@pytest.mark.parametrize("shift,in_place", [(0, False), (3, False), (0, True)])
@pytest.mark.parametrize("name", ["aes-128-gcm", "aes-256-gcm"])
def test_batch_short_record_packs(ta, engine, oracle, gcm_impl, name, shift, in_place):
    gcm_impl("queue")
    _run_seal_open(ta, engine, oracle, [KINDS[name]] * 3, PACK_LENGTHS, seed=41,
                   in_shift=shift, out_shift=shift, in_place=in_place)


def test_batch_short_record_packs_zipf(ta, engine, oracle, gcm_impl):
    """The config-D length mix (Zipf 64 B - 16 KiB) on a few sessions."""
    from talos_amd.workload import zipf_lengths
    gcm_impl("queue")
    lengths = [int(x) for x in zipf_lengths(400, 0x5EED0003)]
    _run_seal_open(ta, engine, oracle, [KINDS["aes-256-gcm"]] * 2, lengths, seed=42)


def test_batch_packs_long_runs(ta, engine, oracle, gcm_impl):
    """One session over 600 K mostly-short records: every workgroup's range is
    longer than the LDS pack plan (kPlanCap = 2,048 records), so runs are split.
    Device seal -> tamper 1/97 -> device open; statuses exact, sampled
    plaintexts equal, tampered records zero-filled (Workload.verify_open);
    sampled sealed bodies equal the oracle's (a symmetric seal/open error in
    the shared pack GHASH code would cancel out in the round trip alone)."""
    import numpy as np
    from talos_amd.workload import Workload
    gcm_impl("queue")
    n = 600_000
    rng = np.random.default_rng(7)
    lengths = rng.integers(0, 200, n)
    lengths[rng.random(n) < 0.05] = 3000   # long records between the packs
    for kind in (po.AES_128_GCM, po.AES_256_GCM):
        wl = Workload(engine, kind, n, 1, 0x5EED0041, lengths=lengths, record_len=0,
                      tamper_every=97)
        p = wl.params[0]
        osess = oracle.tls_session(kind, p.key, p.fixed_iv)
        for i in np.random.default_rng(kind).choice(n, 64, replace=False).tolist() + [0, n - 1]:
            if wl.tampered[i]:
                continue
            ln = int(wl.lengths[i])
            pt = wl.d_pt.download(ln, int(wl.pt_off[i])).tobytes()
            body = wl.d_body.download(ln + 24, int(wl.body_off[i])).tobytes()
            assert body == oracle.tls_seal(osess, int(wl.seq[i]), 23, pt), i
        wl.open()
        engine.sync()
        wl.verify_open(sample=512)
        wl.free()


# Records of 63+ blocks only: the prep pass leaves the pack flag clear, so the
# no-pack queue-kernel variant runs (the one config B uses); AES-128 and
# AES-256 in one batch check the per-key-size flag words.
LONG_ONLY = [ln for ln in LENGTHS + BS_LENGTHS if ln > 992]


@pytest.mark.parametrize("shift,in_place", [(0, False), (3, False), (0, True)])
@pytest.mark.parametrize("name", ["aes-128-gcm", "aes-256-gcm"])
def test_batch_queue_no_pack_variant(ta, engine, oracle, gcm_impl, name, shift, in_place):
    gcm_impl("queue")
    _run_seal_open(ta, engine, oracle, [KINDS[name]] * 2, LONG_ONLY, seed=43, in_shift=shift,
                   in_place=in_place)


# Session runs of config-B records with a ragged tail: the run's last claims
# (the tail-priority window) over long, ragged and misaligned
# records, every 5th tampered.
RUN_TAIL = [16384] * 40 + [16383, 4096, 4097, 8191, 5000, 12345, 16385, 20000, 4095, 1000,
                           16384, 6000, 7000, 9000, 10000, 16384]


@pytest.mark.parametrize("shift", [0, lambda i: 5 if i % 7 == 3 else 0])
@pytest.mark.parametrize("name", ["aes-128-gcm", "aes-256-gcm"])
def test_batch_queue_run_tails(ta, engine, oracle, gcm_impl, name, shift):
    gcm_impl("queue")
    _run_seal_open(ta, engine, oracle, [KINDS[name]] * 3, RUN_TAIL, seed=47, in_shift=shift)


def test_batch_queue_mixed_key_sizes_pack_flags(ta, engine, oracle, gcm_impl):
    """Short AES-128 records beside long-only AES-256 records in one batch."""
    gcm_impl("queue")
    kinds = [po.AES_128_GCM, po.AES_256_GCM]
    from talos_amd.batch import RecordBatch
    rnd = random.Random(44)
    params = _mk_sessions(ta, rnd, kinds)
    table = ta.SessionTable(engine, 2)
    table.install(0, params)
    osess = _oracle_sessions(oracle, params)
    recs = [(0, i, 23, bytes(rnd.getrandbits(8) for _ in range(ln)), kinds[0])
            for i, ln in enumerate([0, 5, 100, 700])]
    recs += [(1, i, 23, bytes(rnd.getrandbits(8) for _ in range(ln)), kinds[1])
             for i, ln in enumerate([2000, 16384, 5000])]
    sb = RecordBatch(engine, recs, "seal")
    sb.run(table)
    for (st, body), (sid, seq, rtype, pt, _) in zip(sb.results(), recs):
        assert body == oracle.tls_seal(osess[sid], seq, rtype, pt)
    table.close()


def test_batch_packs_disabled_env(ta):
    """TLSGPU_PACK=0 (read at library load): the short-record mix runs through
    the no-pack variant, in a child process with the variable set."""
    import subprocess
    code = ("import sys; sys.path[:0] = [%r, %r]\n"
            "import test_gpu_parity as t, pyoracle as po, talos_amd as ta\n"
            "ta.load_library(); e = ta.Engine(0); o = po.Oracle()\n"
            "for k in (po.AES_128_GCM, po.AES_256_GCM):\n"
            "    t._run_seal_open(ta, e, o, [k] * 2, t.PACK_LENGTHS, seed=45)\n"
            "e.close(); print('ok')\n") % (os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"))
    env = dict(os.environ, TLSGPU_PACK="0", TLSGPU_GCM_IMPL="queue")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=100,
                       env=env, cwd=ROOT)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-2000:]


@pytest.mark.parametrize("mode", ["seal", "open"])
def test_batch_bounds(ta, engine, oracle, mode):
    """tlsgpu_open/seal_batch take the buffer sizes: a record whose input or
    output span leaves its buffer gets REC_OUT_OF_BOUNDS and nothing of it is
    written; the other records of the batch are unaffected."""
    import numpy as np
    from talos_amd.batch import RecordBatch
    rnd = random.Random(77)
    kinds = [po.AES_128_GCM, po.CHACHA20_POLY1305]
    params = _mk_sessions(ta, rnd, kinds)
    table = ta.SessionTable(engine, 2)
    table.install(0, params)
    osess = _oracle_sessions(oracle, params)
    pts = [bytes(rnd.getrandbits(8) for _ in range(n)) for n in (100, 2000, 16384, 77)]
    recs = [(i % 2, 5 + i, 23, pt, kinds[i % 2]) for i, pt in enumerate(pts)]
    if mode == "open":
        recs = [(sid, seq, rt, oracle.tls_seal(osess[sid], seq, rt, pt), k)
                for sid, seq, rt, pt, k in recs]
    b = RecordBatch(engine, recs, mode)
    descs = b.d_recs.download().view(ta.RECORD_DTYPE).copy()
    descs[1]["in_off"] = b.d_in.nbytes - 10             # input runs past d_in
    descs[2]["out_off"] = b.d_out.nbytes - 100          # output runs past d_out
    descs[3]["in_off"] = (1 << 63) + 5                  # offset overflow
    b.d_recs.upload(descs.view(np.uint8))
    b.run(table)
    res = b.results()
    assert [s for s, _ in res[1:]] == [ta.REC_OUT_OF_BOUNDS] * 3
    sid, seq, rt, payload, _ = recs[0]
    want = (oracle.tls_seal(osess[sid], seq, rt, payload) if mode == "seal" else pts[0])
    assert res[0] == (len(want), want)
    out = b.d_out.download()
    for i in (1, 2, 3):   # untouched output regions keep the 0xA5 fill
        o = int(descs[i]["out_off"]) if i != 2 else None
        if o is not None and o < len(out):
            assert (out[o:o + 32] == 0xA5).all()
    assert (out[-100:] == 0xA5).all()
    table.close()


@pytest.mark.parametrize("mode", ["open", "seal"])
@pytest.mark.parametrize("hints", [2, 3])
@pytest.mark.parametrize("name", ["aes-128-gcm", "aes-256-gcm"])
def test_batch_fused_prologue(ta, engine, oracle, gcm_impl, mode, hints, name):
    gcm_impl("queue")
    _fused_case(ta, engine, oracle, mode, hints, name)


@pytest.mark.parametrize("mode", ["open", "seal"])
def test_batch_fused_chacha(ta, engine, oracle, mode):
    """The fused ChaCha batch (round 5, engine.cpp run_batch `fused_cc`): a
    table of RFC 7539 ChaCha20-Poly1305 sessions only, so the staged ChaCha
    kernel is the batch's only launch and checks bounds and writes the statuses
    of the records it does not run itself (no check_record_bounds, no
    descriptor copy) — the same cases as the fused GCM prologue."""
    _fused_case(ta, engine, oracle, mode, 0, "chacha20-poly1305")


def _fused_case(ta, engine, oracle, mode, hints, name, lengths=None):
    """The fused queue kernel (round 5, engine.cpp run_batch `fused`): one AES
    key size installed and SESSION_RUNS stated, so the queue kernel is the
    batch's only launch and checks bounds, writes the initial statuses and
    derives each record's constants in its own prologue (no
    check_record_bounds, no gcm_prep_kernel, no descriptor copy).  hints = 3
    (NO_SHORT_RECORDS too) runs the no-pack variant, 2 the pack variant.  Every
    record equals the oracle's tls1_enc, tampered records are zero-filled,
    out-of-bounds records (input past d_in, output past d_out, offset
    overflow; short records, which the pack plan must leave out, among them)
    get REC_OUT_OF_BOUNDS and leave their output untouched."""
    import numpy as np
    from talos_amd.batch import RecordBatch
    rnd = random.Random(90 + hints)
    kind = KINDS[name]
    params = _mk_sessions(ta, rnd, [kind] * 4)
    table = ta.SessionTable(engine, 4)
    table.install(0, params)
    table.hint(hints)
    osess = _oracle_sessions(oracle, params)
    lengths = lengths or [0, 1, 15, 16, 17, 100, 1000, 16384, 5000, 64, 992, 993, 2000]
    recs = []
    for sid in range(4):                           # session runs of 80 records
        for i in range(80):
            n = lengths[(i + sid) % len(lengths)]
            recs.append((sid, 1000 * sid + i, 23, bytes(rnd.getrandbits(8) for _ in range(n)), kind))
    if mode == "open":
        tamper = {i for i in range(len(recs)) if i % 7 == 3 and recs[i][3]}
        bodies = []
        for i, (sid, seq, rt, pt, k) in enumerate(recs):
            b = bytearray(oracle.tls_seal(osess[sid], seq, rt, pt))
            if i in tamper:
                b[rnd.randrange(len(b))] ^= 4
            bodies.append((sid, seq, rt, bytes(b), k))
        batch = RecordBatch(engine, bodies, "open")
    else:
        batch = RecordBatch(engine, recs, "seal")
    descs = batch.d_recs.download().view(ta.RECORD_DTYPE).copy()
    oob = {5: ("in_off", batch.d_in.nbytes - 3), 81: ("out_off", batch.d_out.nbytes - 8),
           162: ("in_off", (1 << 63) + 5), 252: ("out_off", batch.d_out.nbytes - 8)}
    for i, (f, v) in oob.items():
        descs[i][f] = v
    batch.d_recs.upload(descs.view(np.uint8))
    batch.run(table)
    res = batch.results()
    out = batch.d_out.download()
    for i, ((st, got), (sid, seq, rt, pt, k)) in enumerate(zip(res, recs)):
        if i in oob:
            assert st == ta.REC_OUT_OF_BOUNDS, (i, st)
            continue
        if mode == "seal":
            exp = oracle.tls_seal(osess[sid], seq, rt, pt)
            assert st == len(exp) and got == exp, (i, len(pt), st)
        else:
            est, exp = oracle.tls_open(osess[sid], seq, rt, bodies[i][3])
            if i in tamper:
                assert est == -1 and st == ta.REC_BAD_MAC and got == bytes(len(got)), i
            else:
                assert st == len(pt) and got == pt, (i, len(pt), st)
    o = int(descs[252]["out_off"])
    assert (out[o:] == 0xA5).all()                 # nothing written past d_out
    table.close()


# 16 KiB records every 40th, the rest 0..17 bytes: a 16 KiB record outweighs
# a workgroup's share of the work, so some work-balanced ranges are empty
# (the out-of-bounds records of _fused_case get >= 9 bytes)
SKEWED_LENGTHS = [16384] + [17, 16, 15, 12, 9] * 7 + [3, 5, 1, 0]


@pytest.mark.parametrize("balance,snap,pieces", [("1", "0", "0"), ("2", "0", "0"), ("2", "300", "0"),
                                                 ("0", "0", "2")])
def test_batch_fused_balanced_ranges(ta, balance, snap, pieces):
    """Work-balanced ranges (round 5, engine.cpp run_batch `balance`,
    gcm_hybrid.h work_cut): the fused kernel's workgroups take the records
    between cuts at equal work (payload bytes + 256 per record) instead of
    equal counts (opt-in, measured no faster on config D).  TLSGPU_BALANCE=1
    cuts the pack variant's batches, 2 the no-pack variant's too;
    TLSGPU_BALANCE_SNAP moves cuts near a session-run boundary onto it.
    TLSGPU_PIECES=2: whole pieces (a session run inside a count range)
    sorted by work and dealt to the workgroups in snake order.
    The fused prologue cases — bounds, statuses, tamper, both variants — and a
    skewed batch whose cuts leave ranges empty, all against the oracle, in a
    child process with the variable set."""
    import subprocess
    code = ("import sys; sys.path[:0] = [%r, %r]\n"
            "import test_gpu_parity as t, pyoracle as po, talos_amd as ta\n"
            "ta.load_library(); e = ta.Engine(0); o = po.Oracle()\n"
            "for name in ('aes-128-gcm', 'aes-256-gcm'):\n"
            "    for mode in ('seal', 'open'):\n"
            "        for hints in (2, 3):\n"
            "            t._fused_case(ta, e, o, mode, hints, name)\n"
            "            t._fused_case(ta, e, o, mode, hints, name, lengths=t.SKEWED_LENGTHS)\n"
            "e.close(); print('ok')\n") % (os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"))
    env = dict(os.environ, TLSGPU_BALANCE=balance, TLSGPU_BALANCE_SNAP=snap, TLSGPU_PIECES=pieces,
               TLSGPU_GCM_IMPL="queue")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=110,
                       env=env, cwd=ROOT)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-2000:]


def test_batch_per_wave_session_kernel_forced(ta):
    """TLSGPU_PWS=1: every queue-impl GCM batch runs on the per-wave-session
    kernel (gcm_pw.hip: per-wave nibble GHASH tables, Shoup weights from HBM,
    no session runs) — the full length matrix, misaligned and in-place
    buffers, short records, interleaved sessions of mixed kinds and tamper
    zero-fill, against the oracle, in a child process with the variable set."""
    import subprocess
    code = ("import sys; sys.path[:0] = [%r, %r]\n"
            "import test_gpu_parity as t, pyoracle as po, talos_amd as ta\n"
            "ta.load_library(); e = ta.Engine(0); o = po.Oracle()\n"
            "for k in (po.AES_128_GCM, po.AES_256_GCM):\n"
            "    t._run_seal_open(ta, e, o, [k] * 3, t.LENGTHS, seed=51)\n"
            "    t._run_seal_open(ta, e, o, [k] * 2, t.BS_LENGTHS, seed=52, in_shift=3, out_shift=5)\n"
            "    t._run_seal_open(ta, e, o, [k] * 2, t.PACK_LENGTHS, seed=53, in_place=True)\n"
            "    t._run_seal_open(ta, e, o, [k] * 7, [1, 17, 300, 1400, 5000, 16384], grouped=False, seed=54)\n"
            "t._run_seal_open(ta, e, o, [po.AES_128_GCM, po.AES_256_GCM, po.CHACHA20_POLY1305,\n"
            "                 po.AES_256_GCM, po.AES_128_GCM], [0, 33, 999, 16384], grouped=False, seed=55)\n"
            "e.close(); print('ok')\n") % (os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"))
    env = dict(os.environ, TLSGPU_PWS="1", TLSGPU_GCM_IMPL="queue")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=110,
                       env=env, cwd=ROOT)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-2000:]


# Randomized differential sweep (round 5): each seed draws a batch shape the
# fixed cases above do not combine — a random mix of the four AEADs over up to
# 9 sessions, lengths weighted toward the block / pack / step edges (0..20000),
# per-record input shifts, grouped or interleaved order, any hint word — and
# the whole seal + open round trip (every 5th record tampered) must equal the
# oracle's tls1_enc byte for byte.
EDGE_LENGTHS = [0, 1, 15, 16, 17, 63, 64, 65, 991, 992, 993, 1023, 1024, 1025, 1400, 4095,
                4096, 4097, 16383, 16384, 16385]


# TLSGPU_FUZZ_SEEDS=<n> widens the sweep for a soak run (default 12 seeds)
@pytest.mark.parametrize("seed", range(int(os.environ.get("TLSGPU_FUZZ_SEEDS", "12"))))
def test_batch_random_differential(ta, engine, oracle, seed):
    rnd = random.Random(9000 + seed)
    kinds = [rnd.choice(list(KINDS.values())) for _ in range(rnd.randint(1, 9))]
    lengths = [rnd.choice(EDGE_LENGTHS) if rnd.random() < 0.5 else rnd.randrange(0, 20001)
               for _ in range(rnd.randint(4, 24))]
    shifts = [rnd.choice([0, 0, 0, 1, 3, 8, 13]) for _ in range(len(kinds) * len(lengths))]
    _run_seal_open(ta, engine, oracle, kinds, lengths, grouped=rnd.random() < 0.5,
                   in_shift=shifts, out_shift=rnd.choice([0, 0, 5]), seed=seed,
                   in_place=False, hints=rnd.choice([0, 0, 1, 2, 3]))
