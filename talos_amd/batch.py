"""Device-resident record batches for the engine (host packing helpers).

A :class:`RecordBatch` packs records into one device input buffer and one
device output buffer plus a ``tlsgpu_record`` descriptor array, the layout the
batch kernels consume.  Offsets are chosen so that GCM ciphertext (record body
+ 8) and plaintext start on 16-byte boundaries, which lets the kernels use
dwordx4 loads/stores; any other alignment is also handled (byte path).

Device memory comes from the engine itself (tlsgpu_malloc / tlsgpu_memcpy), so
no second GPU runtime is loaded next to libtlsgpu.so.
"""
from __future__ import annotations

import numpy as np

from . import (EXPLICIT_NONCE_LEN, RECORD_DTYPE, TAG_LEN, DeviceBuffer, SessionTable, len_type,
               open_batch, seal_batch)


def _align(v: int, a: int, rem: int = 0) -> int:
    v += (rem - v) % a
    return v


class RecordBatch:
    """Records of one direction, ready for tlsgpu_open_batch / _seal_batch.

    entries: list of (session_id, seq, content_type, payload_bytes, kind).
    For ``mode='seal'`` payload is plaintext; for ``mode='open'`` it is the
    record fragment (explicit nonce || ct || tag for GCM).
    """

    def __init__(self, engine, entries, mode: str, in_shift: int = 0, out_shift: int = 0,
                 in_place: bool = False):
        assert mode in ("seal", "open")
        self.mode = mode
        n = len(entries)
        descs = np.zeros(n, dtype=RECORD_DTYPE)
        in_offs, out_offs, out_lens = [], [], []
        ip = op = 0
        for i, (sid, seq, rtype, payload, kind) in enumerate(entries):
            eiv = EXPLICIT_NONCE_LEN[kind]
            ish = in_shift[i] if isinstance(in_shift, (list, tuple)) else in_shift
            if mode == "seal":
                ip = _align(ip, 16) + ish
                olen = len(payload) + eiv + TAG_LEN
                op = _align(op, 16, (16 - eiv) % 16) + out_shift
            else:
                ip = _align(ip, 16, (16 - eiv) % 16) + ish
                olen = max(len(payload) - eiv - TAG_LEN, 0)
                op = _align(op, 16) + out_shift
            in_offs.append(ip)
            out_offs.append(op)
            out_lens.append(olen)
            descs[i] = (ip, op, seq, sid, len_type(len(payload), rtype))
            ip += len(payload)
            op += max(olen, 1)
        self.n = n
        self.in_size = max(ip, 1) + 64
        self.out_size = max(op, 1) + 64
        host_in = np.zeros(self.in_size, dtype=np.uint8)
        for (sid, seq, rtype, payload, kind), off in zip(entries, in_offs):
            host_in[off:off + len(payload)] = np.frombuffer(payload, dtype=np.uint8)
        self.engine = engine
        self.d_in = DeviceBuffer(engine, self.in_size)
        self.d_in.upload(host_in)
        if in_place:
            # open in place: plaintext lands at fragment + explicit nonce length
            self.d_out = self.d_in
            for i, (sid, seq, rtype, payload, kind) in enumerate(entries):
                descs[i]["out_off"] = in_offs[i] + (EXPLICIT_NONCE_LEN[kind] if mode == "open" else 0)
                out_offs[i] = int(descs[i]["out_off"])
        else:
            self.d_out = DeviceBuffer(engine, self.out_size)
            self.d_out.fill(0xA5)
        self.d_recs = DeviceBuffer(engine, max(descs.nbytes, 32))
        self.d_recs.upload(descs.view(np.uint8))
        self.d_status = DeviceBuffer(engine, 4 * max(n, 1))
        self.out_offs = out_offs
        self.out_lens = out_lens
        self.entries = entries

    def run(self, table: SessionTable, stream: int | None = None) -> None:
        fn = seal_batch if self.mode == "seal" else open_batch
        fn(table, self.d_recs.ptr, self.n, self.d_in.ptr, self.d_in.nbytes, self.d_out.ptr,
           self.d_out.nbytes, self.d_status.ptr, stream)

    def results(self):
        """[(status, output_bytes)] — output length = status when >= 0, else the
        region the kernel zero-fills (plaintext length) or b''."""
        self.engine.sync()
        out = self.d_out.download()
        st = self.d_status.download().view(np.int32)[:self.n]
        res = []
        for i in range(self.n):
            s = int(st[i])
            ln = s if s >= 0 else (self.out_lens[i] if s == -1 else 0)
            res.append((s, out[self.out_offs[i]:self.out_offs[i] + ln].tobytes()))
        return res

    def free(self) -> None:
        for b in {id(x): x for x in (self.d_in, self.d_out, self.d_recs, self.d_status)}.values():
            b.free()
