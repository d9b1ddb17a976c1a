"""Synthetic TLS record workloads of BASELINE.json / SURVEY.md §8d, built on the GPU.

Each workload is generated deterministically from its seed with the counter
SplitMix64 stream (tlsgpu_fill_synthetic == oracle_fill_bytes), so any shard or
test can regenerate any record independently:

* sessions s = 0..S-1: key = fill(seed ^ KEY_TAG, s), fixed IV = fill(seed ^ IV_TAG, s),
  start sequence number = fill(seed ^ SEQ_TAG, s) (8 bytes, little endian);
* record r belongs to session r // (R / S) (records grouped by connection, as a
  server's read-ahead batches are), seq = start_seq + r % (R / S);
* plaintext of record r = fill(seed, r, length_r).

A batch split across GPUs (config E) is ONE such batch: the
GPU of shard [lo, hi) builds records lo..hi-1 with their global index (session,
sequence number, plaintext and tamper rule all keyed by it) and installs only
the sessions those records use, so a shard's outputs equal that slice of the
whole batch's — oracle/batch_digest range=LO:HI pins each slice.

Ciphertexts for the decrypt configurations are produced on the device by the
validated sealer (tlsgpu_seal_batch), as SURVEY.md §8d prescribes.
"""
from __future__ import annotations

import numpy as np

from . import (EXPLICIT_NONCE_LEN, FIXED_IV_LEN, KEY_LEN, RECORD_DTYPE, TAG_LEN, DeviceBuffer,
               SessionParams, SessionTable, len_type, open_batch, seal_batch)

KEY_TAG = 0x4B45590000000000
IV_TAG = 0x4956000000000000
SEQ_TAG = 0x5345510000000000
M64 = (1 << 64) - 1


def fill_bytes(seed: int, index: int, n: int) -> bytes:
    """Host twin of tlsgpu_fill_synthetic for small spans (keys, IVs, seqs)."""
    st = (seed ^ (index * 0xD1B54A32D192ED03)) & M64
    out = bytearray()
    w = 0
    while len(out) < n:
        w += 1
        z = (st + w * 0x9E3779B97F4A7C15) & M64
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        z ^= z >> 31
        out += z.to_bytes(8, "little")
    return bytes(out[:n])


def zipf_lengths(n: int, seed: int, lo: int = 64, hi: int = 16384, alpha: float = 1.0):
    """P(l) ∝ (l - lo + 1)^-alpha for integer l in [lo, hi]."""
    ls = np.arange(lo, hi + 1)
    p = (ls - lo + 1.0) ** (-alpha)
    p /= p.sum()
    rng = np.random.default_rng(seed)
    return rng.choice(ls, size=n, p=p).astype(np.int64)


def session_plan(kind: int, n_records: int, n_sessions: int, seed: int,
                 interleave: bool = False):
    """(session params, start seqs, per-record session, per-record seq) of a
    workload; oracle/batch_digest.c restates the same rule in C.  Records are
    grouped by session (record r -> session r // (R / S)), or with
    `interleave` dealt round-robin (r -> r % S, the k-th record of a session
    has seq start + k) as a many-connection server batch would arrive."""
    params, start_seq = [], []
    for s in range(n_sessions):
        key = fill_bytes(seed ^ KEY_TAG, s, KEY_LEN[kind])
        fiv = fill_bytes(seed ^ IV_TAG, s, FIXED_IV_LEN[kind])
        params.append(SessionParams(kind, key, fiv))
        sq = int.from_bytes(fill_bytes(seed ^ SEQ_TAG, s, 8), "little")
        # some sessions sit just below a byte / 32-bit carry
        if s % 7 == 1:
            sq = (sq | 0xFF) - 3
        elif s % 7 == 2:
            sq = (sq | 0xFFFFFFFF) - 5
        start_seq.append(sq & M64)
    r = np.arange(n_records, dtype=np.int64)
    if interleave:
        session = (r % n_sessions).astype(np.uint32)
        k = r // n_sessions
    else:
        per = max(1, n_records // n_sessions)
        session = np.minimum(r // per, n_sessions - 1).astype(np.uint32)
        k = r % per
    seq = np.array(start_seq, dtype=np.uint64)[session] + k.astype(np.uint64)
    return params, start_seq, session, seq


class Workload:
    """R records over S sessions of one AEAD kind, resident in HBM.

    Buffers: ``pt`` (plaintexts, 16-B aligned), ``body`` (record fragments,
    ciphertext 16-B aligned), ``out`` (decrypted plaintexts).  ``open_descs``
    decrypt body -> out, ``seal_descs`` encrypt pt -> body.
    """

    def __init__(self, engine, kind: int, n_records: int, n_sessions: int, seed: int,
                 lengths=None, record_len: int = 16384, tamper_every: int = 0,
                 interleave: bool = False, shard: tuple[int, int] | None = None,
                 slot_align: int = 16):
        """n_records / n_sessions describe the whole batch; `shard` = (lo, hi)
        keeps records [lo, hi) of it on this engine (default: all).  `lengths`
        are the kept records' lengths.  `slot_align` (a multiple of 16): the
        alignment of every plaintext and ciphertext slot (16 by default; 128
        puts every record on its own cache lines — a measurement option)."""
        if slot_align < 16 or slot_align % 16:
            raise ValueError("slot_align must be a multiple of 16")
        lo, hi = shard if shard is not None else (0, n_records)
        if not 0 <= lo <= hi <= n_records:
            raise ValueError(f"shard {lo}:{hi} outside the {n_records}-record batch")
        self.engine = engine
        self.kind = kind
        self.lo = lo
        self.n = hi - lo
        self.seed = seed
        self.lengths = (np.full(self.n, record_len, dtype=np.int64) if lengths is None
                        else np.asarray(lengths, dtype=np.int64))
        if len(self.lengths) != self.n:
            raise ValueError("lengths must cover the shard's records")
        total = n_records
        n_records = hi - lo   # from here on: this shard's records
        eiv = EXPLICIT_NONCE_LEN[kind]
        A = slot_align
        shift = (A - eiv) % A   # the ciphertext (after the explicit nonce) A-B aligned
        pt_slot = (self.lengths + A - 1) // A * A
        if A == 16:   # the default layout (golden digests depend on it)
            body_slot = (self.lengths + eiv + TAG_LEN + 15 + 16) // 16 * 16
        else:
            body_slot = (self.lengths + shift + eiv + TAG_LEN + A - 1) // A * A
        self.pt_off = np.concatenate([[0], np.cumsum(pt_slot)[:-1]]).astype(np.uint64)
        body_base = np.concatenate([[0], np.cumsum(body_slot)[:-1]]).astype(np.uint64)
        self.body_off = body_base + np.uint64(shift)
        self.pt_bytes = int(pt_slot.sum())
        self.body_bytes = int(body_slot.sum()) + 16

        # sessions, record -> session map and sequence numbers of the whole
        # batch, then this shard's slice; the device table holds the sessions
        # [s0, s0 + S) the slice uses (local id = global id - s0)
        params, start_seq, session, seq = session_plan(kind, total, n_sessions, seed, interleave)
        session, self.seq = session[lo:hi], seq[lo:hi]
        self.s0 = int(session.min()) if self.n else 0
        s1 = int(session.max()) + 1 if self.n else 1
        self.S = s1 - self.s0
        self.params, self.start_seq = params[self.s0:s1], start_seq[self.s0:s1]
        self.session = (session - self.s0).astype(np.uint32)
        self.table = SessionTable(engine, self.S)
        self.table.install(0, self.params)
        self.rtype = np.full(n_records, 23, dtype=np.uint32)

        # device buffers
        self.d_pt = DeviceBuffer(engine, self.pt_bytes)
        self.d_body = DeviceBuffer(engine, self.body_bytes)
        self.d_out = DeviceBuffer(engine, self.pt_bytes)
        self.d_status = DeviceBuffer(engine, 4 * n_records)
        if lengths is None:  # record i's plaintext = fill(seed, lo + i) at pt_off[i]
            engine.fill_synthetic(self.d_pt.ptr, (record_len + 15) // 16 * 16, record_len,
                                  n_records, seed, lo)
        else:  # variable spans: one launch over (offset, length) arrays
            d_offs = DeviceBuffer(engine, 8 * n_records)
            d_lens = DeviceBuffer(engine, 4 * n_records)
            d_offs.upload(self.pt_off.astype(np.uint64).view(np.uint8))
            d_lens.upload(self.lengths.astype(np.uint32).view(np.uint8))
            engine.fill_synthetic_spans(self.d_pt.ptr, d_offs.ptr, d_lens.ptr, n_records, seed,
                                        lo)
            engine.sync()
            d_offs.free()
            d_lens.free()
        seal = np.zeros(n_records, dtype=RECORD_DTYPE)
        seal["in_off"] = self.pt_off
        seal["out_off"] = self.body_off
        seal["seq"] = self.seq
        seal["session"] = self.session
        seal["len_type"] = (self.rtype << 24) | self.lengths.astype(np.uint32)
        opn = np.zeros(n_records, dtype=RECORD_DTYPE)
        opn["in_off"] = self.body_off
        opn["out_off"] = self.pt_off
        opn["seq"] = self.seq
        opn["session"] = self.session
        opn["len_type"] = (self.rtype << 24) | (self.lengths + eiv + TAG_LEN).astype(np.uint32)
        self.d_seal = DeviceBuffer(engine, seal.nbytes)
        self.d_seal.upload(seal.view(np.uint8))
        self.d_open = DeviceBuffer(engine, opn.nbytes)
        self.d_open.upload(opn.view(np.uint8))

        # ciphertexts by the validated sealer
        self.seal()
        engine.sync()
        st = self.status()
        body_len = self.lengths + eiv + TAG_LEN
        if not np.array_equal(st, body_len.astype(np.int32)):
            raise RuntimeError("workload seal failed for %d records" % int((st != body_len).sum()))
        self.tampered = np.zeros(n_records, dtype=bool)
        if tamper_every:
            self.apply_tamper(tamper_every)

    def apply_tamper(self, every: int) -> None:
        """Flip one ciphertext/tag bit of records every//2, every//2 + every, ...
        of the whole batch (SURVEY.md §8d tamper subset): bit g%8 of body byte
        eiv + (g*7919) % (len + 16) for global record index g.
        oracle/batch_digest.c applies the same rule."""
        eiv = EXPLICIT_NONCE_LEN[self.kind]
        first = (every // 2 - self.lo) % every
        idx = np.arange(first, self.n, every)
        for i in idx:
            g = self.lo + int(i)
            pos = int(self.body_off[i]) + eiv + int((g * 7919) % (self.lengths[i] + TAG_LEN))
            b = self.d_body.download(1, pos)
            b[0] ^= 1 << (g % 8)
            self.d_body.upload(b, pos)
        self.tampered[idx] = True

    def sealed_digest(self) -> str:
        """SHA-256 over the record bodies (explicit nonce || ct || tag) in record
        order, as tests/golden/batch_digests.json pins them."""
        import hashlib
        eiv = EXPLICIT_NONCE_LEN[self.kind]
        body = self.d_body.download()
        h = hashlib.sha256()
        mv = memoryview(body)
        for off, ln in zip(self.body_off.tolist(), (self.lengths + eiv + TAG_LEN).tolist()):
            h.update(mv[off:off + ln])
        return h.hexdigest()

    def opened_digest(self) -> str:
        """SHA-256 over the opened plaintexts (tampered records zero-filled) in
        record order."""
        import hashlib
        out = self.d_out.download()
        h = hashlib.sha256()
        mv = memoryview(out)
        for off, ln in zip(self.pt_off.tolist(), self.lengths.tolist()):
            h.update(mv[off:off + ln])
        return h.hexdigest()

    def seal(self, stream=None):
        seal_batch(self.table, self.d_seal.ptr, self.n, self.d_pt.ptr, self.d_pt.nbytes,
                   self.d_body.ptr, self.d_body.nbytes, self.d_status.ptr, stream)

    def open(self, stream=None):
        open_batch(self.table, self.d_open.ptr, self.n, self.d_body.ptr, self.d_body.nbytes,
                   self.d_out.ptr, self.d_out.nbytes, self.d_status.ptr, stream)

    def status(self) -> np.ndarray:
        return self.d_status.download().view(np.int32)[:self.n]

    def verify_open(self, sample: int = 64) -> None:
        """After open(): statuses exact, sampled plaintexts == originals, tampered zeroed."""
        st = self.status()
        want = np.where(self.tampered, -1, self.lengths).astype(np.int32)
        bad = np.nonzero(st != want)[0]
        if len(bad):
            raise RuntimeError(f"open status mismatch on {len(bad)} records (first {bad[:5]})")
        rng = np.random.default_rng(self.seed)
        idx = set(rng.choice(self.n, size=min(sample, self.n), replace=False).tolist())
        idx.update(np.nonzero(self.tampered)[0][:4].tolist())
        for i in sorted(idx):
            off, ln = int(self.pt_off[i]), int(self.lengths[i])
            got = self.d_out.download(ln, off)
            if self.tampered[i]:
                if got.any():
                    raise RuntimeError(f"tampered record {i} not zero-filled")
            elif not np.array_equal(got, self.d_pt.download(ln, off)):
                raise RuntimeError(f"record {i} plaintext mismatch")

    def free(self):
        for b in (self.d_pt, self.d_body, self.d_out, self.d_status, self.d_seal, self.d_open):
            b.free()
        self.table.close()
