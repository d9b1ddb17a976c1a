"""talos_amd — MI355X-native TLS 1.2 record bulk-cipher engine (Python host side).

The engine itself is ``libtlsgpu.so`` (HIP kernels for gfx950 behind a C ABI,
``include/tlsgpu.h`` + the drop-in EVP_AEAD ABI ``include/tlsgpu_evp.h``).
This module binds that ABI with ctypes and mirrors the reference's record-layer
interface for the batch path:

* :class:`Engine` / :class:`SessionTable` — device + device session table, the
  state ``tls1_change_cipher_state_aead`` installs (ssl/t1_enc.c:444-495);
* :func:`open_batch` / :func:`seal_batch` — ``tls1_enc(s, 0/1)``'s AEAD branch
  (ssl/t1_enc.c:832-975) over a device-resident array of records;
* :class:`EvpAead` — the per-call ``EVP_AEAD_CTX_*`` functions of
  crypto/evp/evp_aead.c as exported by libtlsgpu.so.

There is no CPU fallback: if the shared library is missing or no GPU is
present the calls raise :class:`TlsGpuError`.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIBPATH = os.environ.get("TLSGPU_LIBRARY") or os.path.join(HERE, "libtlsgpu.so")  # override: experiments only
INCLUDE = os.path.join(ROOT, "include")

AES_128_GCM, AES_256_GCM, CHACHA20_POLY1305, CHACHA20_POLY1305_OLD = 1, 2, 3, 4
AEAD_NAMES = {"aes-128-gcm": AES_128_GCM, "aes-256-gcm": AES_256_GCM,
              "chacha20-poly1305": CHACHA20_POLY1305,
              "chacha20-poly1305-old": CHACHA20_POLY1305_OLD}
KEY_LEN = {AES_128_GCM: 16, AES_256_GCM: 32, CHACHA20_POLY1305: 32, CHACHA20_POLY1305_OLD: 32}
FIXED_IV_LEN = {AES_128_GCM: 4, AES_256_GCM: 4, CHACHA20_POLY1305: 12, CHACHA20_POLY1305_OLD: 0}
EXPLICIT_NONCE_LEN = {AES_128_GCM: 8, AES_256_GCM: 8, CHACHA20_POLY1305: 0,
                      CHACHA20_POLY1305_OLD: 0}
TAG_LEN = 16

REC_BAD_MAC = -1          # tls1_enc returns -1 (bad_record_mac)
REC_PUBLIC_INVALID = -2   # tls1_enc returns 0
MAX_RECORD = 65534 * 16

# tlsgpu_record (include/tlsgpu.h), 32 bytes
# tlsgpu_wire_stream / tlsgpu_wire_result (include/tlsgpu.h)
WIRE_STREAM_DTYPE = np.dtype([("wire_off", "<u8"), ("wire_len", "<u4"), ("session", "<u4"),
                              ("seq", "<u8"), ("version", "<u2"), ("flags", "<u2"),
                              ("rbuf_len", "<u4")])
WIRE_RESULT_DTYPE = np.dtype([("first", "<u4"), ("records", "<u4"), ("delivered", "<u4"),
                              ("consumed", "<u4"), ("alert", "<i4"), ("alert_record", "<u4"),
                              ("reserved", "<u4", (2,))])
assert WIRE_STREAM_DTYPE.itemsize == 32 and WIRE_RESULT_DTYPE.itemsize == 32
WIRE_FIRST_PACKET = 1
# tlsgpu_write_stream / tlsgpu_write_result (include/tlsgpu.h)
WRITE_STREAM_DTYPE = np.dtype([("data_off", "<u8"), ("wire_off", "<u8"), ("seq", "<u8"),
                               ("data_len", "<u4"), ("session", "<u4"), ("version", "<u2"),
                               ("type", "u1"), ("reserved", "u1"), ("max_fragment", "<u4")])
WRITE_RESULT_DTYPE = np.dtype([("first", "<u4"), ("records", "<u4"), ("wire_len", "<u8"),
                               ("next_seq", "<u8"), ("reserved", "<u8")])
assert WRITE_STREAM_DTYPE.itemsize == 40 and WRITE_RESULT_DTYPE.itemsize == 32
REC_BAD_MAC, REC_PUBLIC_INVALID, REC_SKIPPED, REC_OVERFLOW, REC_OUT_OF_BOUNDS = -1, -2, -3, -4, -5

RECORD_DTYPE = np.dtype([("in_off", "<u8"), ("out_off", "<u8"), ("seq", "<u8"),
                         ("session", "<u4"), ("len_type", "<u4")])
assert RECORD_DTYPE.itemsize == 32


class TlsGpuError(RuntimeError):
    pass


class _SessionParams(C.Structure):
    _fields_ = [("aead", C.c_int32), ("key_len", C.c_uint32), ("key", C.c_uint8 * 32),
                ("fixed_iv_len", C.c_uint32), ("fixed_iv", C.c_uint8 * 12),
                ("tag_len", C.c_uint32), ("version", C.c_uint16), ("reserved", C.c_uint16)]


@dataclass
class SessionParams:
    aead: int
    key: bytes
    fixed_iv: bytes = b""
    tag_len: int = 0
    version: int = 0x0303

    def to_c(self) -> _SessionParams:
        p = _SessionParams()
        p.aead = self.aead
        p.key_len = len(self.key)
        C.memmove(p.key, self.key, len(self.key))
        p.fixed_iv_len = len(self.fixed_iv)
        if self.fixed_iv:
            C.memmove(p.fixed_iv, self.fixed_iv, len(self.fixed_iv))
        p.tag_len = self.tag_len
        p.version = self.version
        return p


def build(quiet: bool = True) -> None:
    """Compile libtlsgpu.so for gfx950 in-tree (hipcc)."""
    subprocess.run(["make", "-C", HERE, "-j8"], check=True,
                   stdout=subprocess.DEVNULL if quiet else None)


_LIB = None


def load_library(path: str = LIBPATH) -> C.CDLL:
    """Load libtlsgpu.so; raise loudly when it is missing (no fallback)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(path):
        raise TlsGpuError(f"{path} not built: run `make -C talos_amd` (or __graft_entry__.build())")
    lib = C.CDLL(path, mode=os.RTLD_LOCAL | os.RTLD_NOW)
    vp, u32, u64, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int
    sigs = {
        "tlsgpu_device_count": (i32, [C.POINTER(i32)]),
        "tlsgpu_engine_create": (i32, [i32, C.POINTER(vp)]),
        "tlsgpu_engine_destroy": (None, [vp]),
        "tlsgpu_engine_stream": (vp, [vp]),
        "tlsgpu_engine_sync": (i32, [vp]),
        "tlsgpu_engine_num_cus": (i32, [vp]),
        "tlsgpu_sessions_create": (i32, [vp, u32, C.POINTER(vp)]),
        "tlsgpu_sessions_destroy": (None, [vp]),
        "tlsgpu_sessions_install": (i32, [vp, u32, u32, vp]),
        "tlsgpu_sessions_hint": (i32, [vp, u32]),
        "tlsgpu_open_batch": (i32, [vp, vp, u32, vp, C.c_size_t, vp, C.c_size_t, vp, vp]),
        "tlsgpu_seal_batch": (i32, [vp, vp, u32, vp, C.c_size_t, vp, C.c_size_t, vp, vp]),
        "tlsgpu_fill_synthetic": (i32, [vp, vp, u64, u32, u32, u64, u64, vp]),
        "tlsgpu_fill_synthetic_spans": (i32, [vp, vp, vp, vp, u32, u64, u64, vp]),
        "tlsgpu_last_error": (C.c_char_p, []),
        "tlsgpu_set_gcm_impl": (i32, [i32]),
        "tlsgpu_get_gcm_impl": (i32, []),
        "tlsgpu_aes_ecb_bitsliced": (i32, [vp, u32, vp, vp, u32, vp]),
        "tlsgpu_debug_phase_stats": (i32, [vp, C.POINTER(C.c_ulonglong), i32]),
        "tlsgpu_debug_wg_times": (i32, [vp, C.POINTER(C.c_ulonglong), C.c_uint]),
        "tlsgpu_open_wire": (i32, [vp, vp, u32, vp, u32, vp, vp, vp, vp, vp]),
        "tlsgpu_open_host": (i32, [vp, vp, u32, vp, C.c_size_t, vp, C.c_size_t, vp]),
        "tlsgpu_seal_wire": (i32, [vp, vp, u32, vp, C.c_size_t, vp, C.c_size_t, u32, vp, vp, vp,
                                   vp, vp]),
        "tlsgpu_seal_wire_size": (u64, [i32, u32, u32, u32]),
        "tlsgpu_host_pipeline": (i32, [vp, C.c_uint, C.c_size_t]),
        "tlsgpu_seal_host": (i32, [vp, vp, u32, vp, C.c_size_t, vp, C.c_size_t, vp]),
        "tlsgpu_sessions_set_owner": (i32, [vp, u32, u32, vp]),
        "tlsgpu_deliver_host": (i32, [vp, vp, vp, u32, vp, C.c_size_t, vp, vp, vp]),
        "tlsgpu_hook_write_streams": (i32, [vp, vp, u32, vp, C.c_size_t]),
        "tlsgpu_talos_hook_stats": (i32, [C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
        "tls_processing_register_ssl_read_processing_cb": (None, [vp]),
        "tls_processing_register_ssl_write_processing_cb": (None, [vp]),
        "tls_processing_register_new_connection_cb": (None, [vp]),
        "tls_processing_register_free_connection_cb": (None, [vp]),
        "tlsgpu_evp_cipher_stats": (i32, [C.POINTER(C.c_uint64)]),
        "tlsgpu_evp_set_batching": (i32, [C.c_uint, C.c_uint, C.c_uint]),
        "tlsgpu_evp_batch_stats": (i32, [C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
        "tlsgpu_evp_call_stats": (i32, [C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
        "tlsgpu_evp_context_slot": (i32, [vp, C.POINTER(C.c_void_p), C.POINTER(C.c_uint32)]),
        "tlsgpu_evp_set_doorbell": (i32, [C.c_uint, C.c_uint]),
        "tlsgpu_evp_doorbell_stats": (i32, [C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
        "tlsgpu_evp_doorbell_scrub_stats": (i32, [C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
        "tlsgpu_evp_doorbell_warm": (i32, []),
        "tlsgpu_evp_shutdown": (i32, []),
        "tlsgpu_sessions_debug_read": (i32, [vp, u32, vp, C.c_size_t]),
        "tlsgpu_evp_device_count": (u32, []),
        "tlsgpu_evp_device_stats": (i32, [u32, C.POINTER(i32), C.POINTER(C.c_uint64),
                                          C.POINTER(C.c_uint64)]),
        "tlsgpu_malloc": (i32, [vp, C.c_size_t, C.POINTER(vp)]),
        "tlsgpu_free": (i32, [vp, vp]),
        "tlsgpu_host_alloc": (i32, [vp, C.c_size_t, C.POINTER(vp)]),
        "tlsgpu_host_free": (i32, [vp, vp]),
        "tlsgpu_memcpy": (i32, [vp, vp, vp, C.c_size_t, vp]),
        "tlsgpu_memset": (i32, [vp, vp, i32, C.c_size_t, vp]),
        "tlsgpu_stream_create": (i32, [vp, C.POINTER(vp)]),
        "tlsgpu_stream_destroy": (i32, [vp, vp]),
        "tlsgpu_stream_sync": (i32, [vp, vp]),
        "tlsgpu_event_create": (i32, [vp, C.POINTER(vp)]),
        "tlsgpu_event_destroy": (i32, [vp, vp]),
        "tlsgpu_event_record": (i32, [vp, vp, vp]),
        "tlsgpu_event_elapsed_ms": (i32, [vp, vp, vp, C.POINTER(C.c_float)]),
        "tlsgpu_group_create": (i32, [C.POINTER(i32), u32, C.POINTER(vp)]),
        "tlsgpu_group_destroy": (None, [vp]),
        "tlsgpu_group_size": (u32, [vp]),
        "tlsgpu_group_engine": (vp, [vp, u32]),
        "tlsgpu_group_sessions_create": (i32, [vp, u32, C.POINTER(vp)]),
        "tlsgpu_group_sessions_destroy": (None, [vp]),
        "tlsgpu_group_sessions_member": (vp, [vp, u32]),
        "tlsgpu_group_sessions_install": (i32, [vp, u32, u32, vp]),
        "tlsgpu_split_by_bytes": (i32, [vp, u32, u32, C.POINTER(u32)]),
        "tlsgpu_group_open_host": (i32, [vp, vp, u32, vp, C.c_size_t, vp, C.c_size_t, vp]),
        "tlsgpu_group_seal_host": (i32, [vp, vp, u32, vp, C.c_size_t, vp, C.c_size_t, vp]),
        "tlsgpu_group_open_batch": (i32, [vp, vp]),
        "tlsgpu_group_seal_batch": (i32, [vp, vp]),
        "tlsgpu_group_sync": (i32, [vp]),
        "EVP_aead_aes_128_gcm": (vp, []),
        "EVP_aead_aes_256_gcm": (vp, []),
        "EVP_aead_chacha20_poly1305": (vp, []),
        "EVP_aead_chacha20_poly1305_old": (vp, []),
        "EVP_AEAD_key_length": (C.c_size_t, [vp]),
        "EVP_AEAD_nonce_length": (C.c_size_t, [vp]),
        "EVP_AEAD_max_overhead": (C.c_size_t, [vp]),
        "EVP_AEAD_max_tag_len": (C.c_size_t, [vp]),
        "EVP_AEAD_CTX_init": (i32, [vp, vp, vp, C.c_size_t, C.c_size_t, vp]),
        "EVP_AEAD_CTX_cleanup": (None, [vp]),
        "EVP_AEAD_CTX_seal": (i32, [vp, vp, C.POINTER(C.c_size_t), C.c_size_t, vp, C.c_size_t,
                                    vp, C.c_size_t, vp, C.c_size_t]),
        "EVP_AEAD_CTX_open": (i32, [vp, vp, C.POINTER(C.c_size_t), C.c_size_t, vp, C.c_size_t,
                                    vp, C.c_size_t, vp, C.c_size_t]),
    }
    for name, (res, args) in sigs.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = lib
    return lib


def _check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load_library().tlsgpu_last_error()
        raise TlsGpuError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


def device_count() -> int:
    n = C.c_int(0)
    rc = load_library().tlsgpu_device_count(C.byref(n))
    return n.value if rc == 0 else 0


class Engine:
    """One GPU + HIP stream (tlsgpu_engine_create)."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        h = C.c_void_p()
        _check(self.lib.tlsgpu_engine_create(device, C.byref(h)), "tlsgpu_engine_create")
        self.handle = h
        self.device = device
        self._owned = True

    @classmethod
    def member(cls, group: "Group", k: int) -> "Engine":
        """Member k's engine of a Group (tlsgpu_group_engine).  The group owns
        it: close() leaves it alone, tlsgpu_group_destroy frees it."""
        h = group.lib.tlsgpu_group_engine(group.handle, k)
        if not h:
            raise TlsGpuError(f"group has no member {k}")
        e = cls.__new__(cls)
        e.lib, e.handle, e.device, e._owned = group.lib, C.c_void_p(h), -1, False
        return e

    @property
    def stream(self) -> int:
        return self.lib.tlsgpu_engine_stream(self.handle)

    @property
    def num_cus(self) -> int:
        return self.lib.tlsgpu_engine_num_cus(self.handle)

    def sync(self) -> None:
        _check(self.lib.tlsgpu_engine_sync(self.handle), "tlsgpu_engine_sync")

    def sync_stream(self, stream: int | None = None) -> None:
        _check(self.lib.tlsgpu_stream_sync(self.handle, stream), "tlsgpu_stream_sync")

    def new_stream(self) -> int:
        h = C.c_void_p()
        _check(self.lib.tlsgpu_stream_create(self.handle, C.byref(h)), "tlsgpu_stream_create")
        return h.value

    def fill_synthetic(self, d_out: int, stride: int, span_len: int, n: int, seed: int,
                       index0: int = 0, stream: int | None = None) -> None:
        _check(self.lib.tlsgpu_fill_synthetic(self.handle, d_out, stride, span_len, n, seed,
                                              index0, stream), "tlsgpu_fill_synthetic")

    def fill_synthetic_spans(self, d_out: int, d_offsets: int, d_lengths: int, n: int, seed: int,
                             index0: int = 0, stream: int | None = None) -> None:
        _check(self.lib.tlsgpu_fill_synthetic_spans(self.handle, d_out, d_offsets, d_lengths, n,
                                                    seed, index0, stream),
               "tlsgpu_fill_synthetic_spans")

    def close(self) -> None:
        if self.handle and getattr(self, "_owned", True):
            self.lib.tlsgpu_engine_destroy(self.handle)
        self.handle = None


class DeviceBuffer:
    """HBM buffer owned through the engine (tlsgpu_malloc); numpy on the host side."""

    def __init__(self, engine: Engine, nbytes: int):
        self.engine = engine
        self.lib = engine.lib
        self.nbytes = int(nbytes)
        p = C.c_void_p()
        _check(self.lib.tlsgpu_malloc(engine.handle, max(self.nbytes, 1), C.byref(p)),
               "tlsgpu_malloc")
        self.ptr = p.value

    def upload(self, data, offset: int = 0, stream: int | None = None, sync: bool = True):
        arr = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8)
                                   if isinstance(data, (bytes, bytearray)) else data)
        assert offset + arr.nbytes <= self.nbytes
        _check(self.lib.tlsgpu_memcpy(self.engine.handle, self.ptr + offset,
                                      arr.ctypes.data, arr.nbytes, stream), "tlsgpu_memcpy")
        if sync:
            self.engine.sync_stream(stream)

    def download(self, nbytes: int | None = None, offset: int = 0,
                 stream: int | None = None) -> np.ndarray:
        nbytes = self.nbytes - offset if nbytes is None else nbytes
        out = np.empty(nbytes, dtype=np.uint8)
        _check(self.lib.tlsgpu_memcpy(self.engine.handle, out.ctypes.data, self.ptr + offset,
                                      nbytes, stream), "tlsgpu_memcpy")
        self.engine.sync_stream(stream)
        return out

    def copy_from(self, src: "DeviceBuffer", nbytes: int | None = None,
                  stream: int | None = None) -> None:
        """Device-to-device copy, stream-ordered (no host sync)."""
        n = min(self.nbytes, src.nbytes) if nbytes is None else nbytes
        _check(self.lib.tlsgpu_memcpy(self.engine.handle, self.ptr, src.ptr, n, stream),
               "tlsgpu_memcpy")

    def fill(self, value: int, stream: int | None = None, sync: bool = True) -> None:
        _check(self.lib.tlsgpu_memset(self.engine.handle, self.ptr, value, self.nbytes, stream),
               "tlsgpu_memset")
        if sync:
            self.engine.sync_stream(stream)

    def free(self) -> None:
        if self.ptr and self.engine.handle:
            self.lib.tlsgpu_free(self.engine.handle, self.ptr)
        self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Event:
    def __init__(self, engine: Engine):
        self.engine = engine
        h = C.c_void_p()
        _check(engine.lib.tlsgpu_event_create(engine.handle, C.byref(h)), "tlsgpu_event_create")
        self.handle = h.value

    def record(self, stream: int | None = None) -> None:
        _check(self.engine.lib.tlsgpu_event_record(self.engine.handle, self.handle, stream),
               "tlsgpu_event_record")

    def elapsed_ms(self, end: "Event") -> float:
        ms = C.c_float()
        _check(self.engine.lib.tlsgpu_event_elapsed_ms(self.engine.handle, self.handle,
                                                       end.handle, C.byref(ms)),
               "tlsgpu_event_elapsed_ms")
        return ms.value

    def close(self) -> None:
        if self.handle:
            self.engine.lib.tlsgpu_event_destroy(self.engine.handle, self.handle)
            self.handle = None


class SessionTable:
    """Device session table (tlsgpu_sessions_create / _install)."""

    def __init__(self, engine: Engine, capacity: int):
        self.engine = engine
        self.lib = engine.lib
        h = C.c_void_p()
        _check(self.lib.tlsgpu_sessions_create(engine.handle, capacity, C.byref(h)),
               "tlsgpu_sessions_create")
        self.handle = h
        self.capacity = capacity

    def install(self, first: int, params: list[SessionParams]) -> None:
        arr = (_SessionParams * len(params))(*[p.to_c() for p in params])
        _check(self.lib.tlsgpu_sessions_install(self.handle, first, len(params), arr),
               "tlsgpu_sessions_install")

    def hint(self, hints: int) -> None:
        """Batch-shape hints (tlsgpu_sessions_hint): HINT_NO_SHORT_RECORDS,
        HINT_SESSION_RUNS; performance only."""
        _check(self.lib.tlsgpu_sessions_hint(self.handle, hints), "tlsgpu_sessions_hint")

    def close(self) -> None:
        if self.handle:
            self.lib.tlsgpu_sessions_destroy(self.handle)
            self.handle = None


HINT_NO_SHORT_RECORDS, HINT_SESSION_RUNS = 1, 2


def batch_hints(lengths, sessions, seal: bool) -> int:
    """The hints a caller that built the batch can state (tlsgpu.h): no GCM
    record short enough for a pack, session runs of >= 12 records on average.
    `lengths` are the descriptors' length fields, as the engine's host_hints
    reads them: fragment lengths (explicit nonce + ciphertext + tag) for an
    open, plaintext lengths for a seal."""
    lengths = np.asarray(lengths)
    sessions = np.asarray(sessions)
    short_max = 992 if seal else 992 + 8 + 16
    h = 0
    if len(lengths) and int(lengths.min()) > short_max:
        h |= HINT_NO_SHORT_RECORDS
    runs = 1 + int(np.count_nonzero(sessions[1:] != sessions[:-1])) if len(sessions) else 0
    if runs * 12 <= len(sessions):
        h |= HINT_SESSION_RUNS
    return h


GCM_BITSLICE, GCM_TTABLE, GCM_HYBRID, GCM_QUEUE, GCM_FUSED, GCM_SPLIT, GCM_AUTO = 0, 1, 2, 3, 4, 5, 6
_GCM_IMPLS = {"bitslice": GCM_BITSLICE, "ttable": GCM_TTABLE, "hybrid": GCM_HYBRID,
              "queue": GCM_QUEUE, "fused": GCM_FUSED, "split": GCM_SPLIT, "auto": GCM_AUTO}


def set_gcm_impl(impl: int | str) -> None:
    """Select the GCM TLS batch kernel (tlsgpu_set_gcm_impl):
    auto|split|queue|ttable|hybrid|bitslice|fused."""
    if isinstance(impl, str):
        impl = _GCM_IMPLS[impl]
    _check(load_library().tlsgpu_set_gcm_impl(impl), "tlsgpu_set_gcm_impl")


def get_gcm_impl() -> str:
    v = load_library().tlsgpu_get_gcm_impl()
    return {i: n for n, i in _GCM_IMPLS.items()}[v]


def debug_phase_stats(engine: "Engine", reset: bool = True) -> list[int]:
    """Diagnostic (TLSGPU_PHASE_STATS=1): 16 x (cycles, events) of the hybrid kernel's phases."""
    out = (C.c_ulonglong * 32)()
    _check(engine.lib.tlsgpu_debug_phase_stats(engine.handle, out, int(reset)),
           "tlsgpu_debug_phase_stats")
    return list(out)


def debug_wg_times(engine: "Engine", groups: int) -> list[tuple[int, int, int, int]]:
    """Diagnostic (TLSGPU_WG_TIMES=1): {start, end (100 MHz ticks), records, work}
    per workgroup of the last queue-kernel launch."""
    out = (C.c_ulonglong * (4 * groups))()
    _check(engine.lib.tlsgpu_debug_wg_times(engine.handle, out, groups), "tlsgpu_debug_wg_times")
    return [tuple(out[4 * g:4 * g + 4]) for g in range(groups)]


def aes_ecb_bitsliced(table: "SessionTable", session: int, d_in: int, d_out: int, nblocks: int,
                      stream: int | None = None) -> None:
    """Diagnostic: bitsliced AES-ECB of nblocks device blocks under a GCM session's key."""
    _check(table.lib.tlsgpu_aes_ecb_bitsliced(table.handle, session, d_in, d_out, nblocks, stream),
           "tlsgpu_aes_ecb_bitsliced")


def len_type(length: int, rtype: int) -> int:
    return ((rtype & 0xFF) << 24) | (length & 0xFFFFFF)


def open_wire(table: "SessionTable", d_streams: int, n_streams: int, d_wire: int,
              max_records: int, d_recs: int, d_status: int, d_results: int, d_total: int,
              stream: int | None = None) -> None:
    """Frame and open raw TLS wire records in place (tlsgpu_open_wire, ssl3_get_record)."""
    _check(table.lib.tlsgpu_open_wire(table.handle, d_streams, n_streams, d_wire, max_records,
                                      d_recs, d_status, d_results, d_total, stream),
           "tlsgpu_open_wire")


def open_batch(table: SessionTable, d_recs: int, n: int, d_in: int, in_bytes: int, d_out: int,
               out_bytes: int, d_status: int, stream: int | None = None) -> None:
    """Decrypt n device-resident records (tls1_enc(s, 0) per record); d_in /
    d_out hold in_bytes / out_bytes (records outside get REC_OUT_OF_BOUNDS)."""
    _check(table.lib.tlsgpu_open_batch(table.handle, d_recs, n, d_in, in_bytes, d_out, out_bytes,
                                       d_status, stream), "tlsgpu_open_batch")


def seal_wire(table: SessionTable, d_streams: int, n_streams: int, d_data: int, data_bytes: int,
              d_wire: int, wire_bytes: int, max_records: int, d_recs: int, d_status: int,
              d_results: int, d_total: int, stream: int | None = None) -> None:
    """Fragment, frame and seal application data of many connections
    (tlsgpu_seal_wire: ssl3_write_bytes + do_ssl3_write for AEAD suites)."""
    _check(table.lib.tlsgpu_seal_wire(table.handle, d_streams, n_streams, d_data, data_bytes,
                                      d_wire, wire_bytes, max_records, d_recs, d_status,
                                      d_results, d_total, stream), "tlsgpu_seal_wire")


def seal_wire_size(aead: int, data_len: int, max_fragment: int = 0, tag_len: int = 0) -> int:
    return int(load_library().tlsgpu_seal_wire_size(aead, data_len, max_fragment, tag_len))


def open_host(table: SessionTable, h_recs: int, n: int, h_in: int, in_bytes: int, h_out: int,
              out_bytes: int, h_status: int) -> None:
    """Host-resident batch open (tlsgpu_open_host): host descriptors, fragments,
    plaintext and statuses; synchronous, pipelined over several HIP streams."""
    _check(table.lib.tlsgpu_open_host(table.handle, h_recs, n, h_in, in_bytes, h_out, out_bytes,
                                      h_status), "tlsgpu_open_host")


def seal_host(table: SessionTable, h_recs: int, n: int, h_in: int, in_bytes: int, h_out: int,
              out_bytes: int, h_status: int) -> None:
    """Host-resident batch seal (tlsgpu_seal_host)."""
    _check(table.lib.tlsgpu_seal_host(table.handle, h_recs, n, h_in, in_bytes, h_out, out_bytes,
                                      h_status), "tlsgpu_seal_host")


# TaLoS module callbacks: void (*)(const SSL*, char*, unsigned int*)
TALOS_RW_CB = C.CFUNCTYPE(None, C.c_void_p, C.POINTER(C.c_uint8), C.POINTER(C.c_uint))


def talos_register(on_read=None, on_write=None) -> tuple:
    """Register TaLoS read / write processing callbacks through the reference
    interface libtlsgpu.so exports (tls_processing_register_ssl_*_processing_cb,
    include/tlsgpu_talos.h).  Python callables f(ssl, data_ptr, len_ptr); None
    clears.  Returns the ctypes callbacks, which the caller keeps alive."""
    lib = load_library()
    cbs = tuple(TALOS_RW_CB(f) if f else None for f in (on_read, on_write))
    lib.tls_processing_register_ssl_read_processing_cb(C.cast(cbs[0], C.c_void_p) if cbs[0] else None)
    lib.tls_processing_register_ssl_write_processing_cb(C.cast(cbs[1], C.c_void_p) if cbs[1] else None)
    return cbs


def set_session_owners(table: "SessionTable", first: int, owners: list[int]) -> None:
    """Associate an SSL* (any pointer-sized value) with sessions first.. for the
    TaLoS hooks (tlsgpu_sessions_set_owner)."""
    arr = (C.c_void_p * len(owners))(*owners)
    _check(table.lib.tlsgpu_sessions_set_owner(table.handle, first, len(owners), arr),
           "tlsgpu_sessions_set_owner")


def talos_hook_stats() -> tuple[int, int]:
    r, w = C.c_uint64(0), C.c_uint64(0)
    _check(load_library().tlsgpu_talos_hook_stats(C.byref(r), C.byref(w)), "tlsgpu_talos_hook_stats")
    return r.value, w.value


def deliver_host(table: "SessionTable", d_recs: int, d_status: int, n: int, d_out: int,
                 out_bytes: int, h_out: int, h_status: int, stream: int | None = None) -> None:
    """Host delivery of a device-resident open, read hooks included (tlsgpu_deliver_host)."""
    _check(table.lib.tlsgpu_deliver_host(table.handle, d_recs, d_status, n, d_out, out_bytes,
                                         h_out, h_status, stream), "tlsgpu_deliver_host")


def hook_write_streams(table: "SessionTable", h_streams: int, n: int, h_data: int,
                       data_bytes: int) -> None:
    """Write hooks over host application data of tlsgpu_seal_wire streams."""
    _check(table.lib.tlsgpu_hook_write_streams(table.handle, h_streams, n, h_data, data_bytes),
           "tlsgpu_hook_write_streams")


def host_pipeline(engine: "Engine", streams: int = 0, chunk_bytes: int = 0) -> None:
    """Shape of the tlsgpu_open_host pipeline (0 = keep)."""
    _check(engine.lib.tlsgpu_host_pipeline(engine.handle, streams, chunk_bytes),
           "tlsgpu_host_pipeline")


def seal_batch(table: SessionTable, d_recs: int, n: int, d_in: int, in_bytes: int, d_out: int,
               out_bytes: int, d_status: int, stream: int | None = None) -> None:
    """Encrypt n device-resident records (tls1_enc(s, 1) per record)."""
    _check(table.lib.tlsgpu_seal_batch(table.handle, d_recs, n, d_in, in_bytes, d_out, out_bytes,
                                       d_status, stream), "tlsgpu_seal_batch")


# ---------------------------------------------------------------------------
# Multi-GPU batch split (include/tlsgpu.h tlsgpu_group_*)

SHARD_DTYPE = np.dtype([("d_recs", "<u8"), ("n", "<u4"), ("reserved", "<u4"), ("d_in", "<u8"),
                        ("in_bytes", "<u8"), ("d_out", "<u8"), ("out_bytes", "<u8"),
                        ("d_status", "<u8")])
assert SHARD_DTYPE.itemsize == 56


def split_by_bytes(recs: np.ndarray, parts: int) -> list[int]:
    """Byte-balanced contiguous cuts of a RECORD_DTYPE array (tlsgpu_split_by_bytes,
    host only)."""
    recs = np.ascontiguousarray(recs, dtype=RECORD_DTYPE)
    cuts = (C.c_uint32 * (parts + 1))()
    _check(load_library().tlsgpu_split_by_bytes(recs.ctypes.data if len(recs) else None,
                                                 len(recs), parts, cuts),
           "tlsgpu_split_by_bytes")
    return list(cuts)


class Group:
    """One engine per listed device, one worker thread per engine
    (tlsgpu_group_create; devices=None: every visible GPU)."""

    def __init__(self, devices: list[int] | None = None):
        self.lib = load_library()
        h = C.c_void_p()
        arr = (C.c_int * len(devices))(*devices) if devices else None
        _check(self.lib.tlsgpu_group_create(arr, len(devices) if devices else 0, C.byref(h)),
               "tlsgpu_group_create")
        self.handle = h

    @property
    def size(self) -> int:
        return int(self.lib.tlsgpu_group_size(self.handle))

    def sync(self) -> None:
        _check(self.lib.tlsgpu_group_sync(self.handle), "tlsgpu_group_sync")

    def close(self) -> None:
        if self.handle:
            self.lib.tlsgpu_group_destroy(self.handle)
            self.handle = None


class GroupSessionTable:
    """Session table replicated on every group member (tlsgpu_group_sessions_*)."""

    def __init__(self, group: Group, capacity: int):
        self.group = group
        self.lib = group.lib
        h = C.c_void_p()
        _check(self.lib.tlsgpu_group_sessions_create(group.handle, capacity, C.byref(h)),
               "tlsgpu_group_sessions_create")
        self.handle = h

    def install(self, first: int, params: list[SessionParams]) -> None:
        arr = (_SessionParams * len(params))(*[p.to_c() for p in params])
        _check(self.lib.tlsgpu_group_sessions_install(self.handle, first, len(params), arr),
               "tlsgpu_group_sessions_install")

    def open_host(self, h_recs: int, n: int, h_in: int, in_bytes: int, h_out: int,
                  out_bytes: int, h_status: int) -> None:
        _check(self.lib.tlsgpu_group_open_host(self.handle, h_recs, n, h_in, in_bytes, h_out,
                                               out_bytes, h_status), "tlsgpu_group_open_host")

    def seal_host(self, h_recs: int, n: int, h_in: int, in_bytes: int, h_out: int,
                  out_bytes: int, h_status: int) -> None:
        _check(self.lib.tlsgpu_group_seal_host(self.handle, h_recs, n, h_in, in_bytes, h_out,
                                               out_bytes, h_status), "tlsgpu_group_seal_host")

    def batch(self, shards: np.ndarray, seal: bool) -> None:
        """shards: SHARD_DTYPE, one per member (device pointers on that member)."""
        shards = np.ascontiguousarray(shards, dtype=SHARD_DTYPE)
        fn = self.lib.tlsgpu_group_seal_batch if seal else self.lib.tlsgpu_group_open_batch
        _check(fn(self.handle, shards.ctypes.data), "tlsgpu_group_batch")

    def close(self) -> None:
        if self.handle:
            self.lib.tlsgpu_group_sessions_destroy(self.handle)
            self.handle = None


class _EvpCtx(C.Structure):
    _fields_ = [("aead", C.c_void_p), ("aead_state", C.c_void_p)]


class EvpAead:
    """EVP_AEAD_CTX over libtlsgpu.so's drop-in ABI (evp.h:1211-1315)."""

    GETTERS = {AES_128_GCM: "EVP_aead_aes_128_gcm", AES_256_GCM: "EVP_aead_aes_256_gcm",
               CHACHA20_POLY1305: "EVP_aead_chacha20_poly1305",
               CHACHA20_POLY1305_OLD: "EVP_aead_chacha20_poly1305_old"}

    def __init__(self, kind: int, key: bytes, tag_len: int = 0):
        self.lib = load_library()
        self.aead = getattr(self.lib, self.GETTERS[kind])()
        self.ctx = _EvpCtx()
        kb = (C.c_ubyte * max(len(key), 1)).from_buffer_copy(key or b"\0")
        self.ok = self.lib.EVP_AEAD_CTX_init(C.byref(self.ctx), self.aead, kb, len(key),
                                             tag_len, None)

    @staticmethod
    def _b(b: bytes):
        return (C.c_ubyte * max(len(b), 1)).from_buffer_copy(b or b"\0") if b is not None else None

    def _call(self, fn, nonce, data, ad, max_out):
        out = (C.c_ubyte * max(max_out, 1))()
        ol = C.c_size_t(12345)
        ok = fn(C.byref(self.ctx), out, C.byref(ol), max_out, self._b(nonce), len(nonce),
                self._b(data), len(data), self._b(ad), len(ad))
        return ok, bytes(out)[:ol.value] if ok else bytes(out)[:max_out], ol.value

    def seal(self, nonce: bytes, pt: bytes, ad: bytes, max_out: int | None = None):
        max_out = len(pt) + 16 if max_out is None else max_out
        return self._call(self.lib.EVP_AEAD_CTX_seal, nonce, pt, ad, max_out)

    def open(self, nonce: bytes, ct: bytes, ad: bytes, max_out: int | None = None):
        max_out = len(ct) if max_out is None else max_out
        return self._call(self.lib.EVP_AEAD_CTX_open, nonce, ct, ad, max_out)

    def cleanup(self) -> None:
        self.lib.EVP_AEAD_CTX_cleanup(C.byref(self.ctx))


def evp_set_batching(window_us: int, max_jobs: int = 0, pool_sessions: int = 0) -> None:
    """Turn on / retune the EVP coalescing queue (tlsgpu_evp_set_batching)."""
    _check(load_library().tlsgpu_evp_set_batching(window_us, max_jobs, pool_sessions),
           "tlsgpu_evp_set_batching")


def evp_device_stats() -> list[tuple[int, int, int]]:
    """(device ordinal, contexts, calls) of each GPU the EVP surface uses."""
    lib = load_library()
    out = []
    for k in range(lib.tlsgpu_evp_device_count()):
        d, c, n = C.c_int(0), C.c_uint64(0), C.c_uint64(0)
        _check(lib.tlsgpu_evp_device_stats(k, C.byref(d), C.byref(c), C.byref(n)),
               "tlsgpu_evp_device_stats")
        out.append((d.value, c.value, n.value))
    return out


def evp_set_doorbell(groups: int, lifetime_ms: int = 0) -> None:
    """Per-call AES-GCM and RFC 7539 ChaCha20-Poly1305 EVP jobs through
    resident server workgroups (tlsgpu_evp_set_doorbell; a short GCM job's
    input is staged into LDS by the server's idle waves); before the first
    EVP call."""
    _check(load_library().tlsgpu_evp_set_doorbell(groups, lifetime_ms), "tlsgpu_evp_set_doorbell")


def evp_doorbell_warm() -> None:
    """Launch a server instance now where the next call would (tlsgpu_evp_doorbell_warm)."""
    _check(load_library().tlsgpu_evp_doorbell_warm(), "tlsgpu_evp_doorbell_warm")


def evp_shutdown() -> None:
    """The doorbell's shutdown contract (tlsgpu_evp_shutdown): stop every
    server and wait until every launched instance has left; later EVP calls
    take the launched path."""
    _check(load_library().tlsgpu_evp_shutdown(), "tlsgpu_evp_shutdown")


def evp_doorbell_stats() -> tuple[int, int]:
    j, l = C.c_uint64(), C.c_uint64()
    _check(load_library().tlsgpu_evp_doorbell_stats(C.byref(j), C.byref(l)),
           "tlsgpu_evp_doorbell_stats")
    return j.value, l.value


def evp_doorbell_scrub_stats() -> tuple[int, int]:
    """(scrub jobs served, LDS flushes by the other server workgroups)."""
    n, f = C.c_uint64(), C.c_uint64()
    _check(load_library().tlsgpu_evp_doorbell_scrub_stats(C.byref(n), C.byref(f)),
           "tlsgpu_evp_doorbell_scrub_stats")
    return n.value, f.value


def evp_batch_stats() -> tuple[int, int]:
    """(batches run, jobs served) by the EVP coalescing queue."""
    b, j = C.c_uint64(0), C.c_uint64(0)
    _check(load_library().tlsgpu_evp_batch_stats(C.byref(b), C.byref(j)), "tlsgpu_evp_batch_stats")
    return b.value, j.value


def header_symbols() -> list[str]:
    """Function names declared in include/*.h (the exported ABI)."""
    import re
    names = []
    for h in ("tlsgpu.h", "tlsgpu_evp.h", "tlsgpu_talos.h"):
        src = open(os.path.join(INCLUDE, h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names += re.findall(r"\b((?:tlsgpu|EVP|tls_processing|ecall_tls_processing)_\w+)\s*\(",
                            src)
    return sorted(set(n for n in names if not n.startswith("TLSGPU")))
