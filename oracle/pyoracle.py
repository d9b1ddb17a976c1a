"""ctypes bindings for the oracle — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module.  It wraps

* ``oracle/liboracle.so``   — our CPU restatement of the LibreSSL 2.4.1 record
  cipher path (see oracle/oracle.h for the reference file:line map), and
* ``oracle/_ref/libref.so`` — the reference itself compiled from
  /root/reference sources by oracle/Makefile (EVP_AEAD ABI of
  include/openssl/evp.h:1211-1315), when it has been built.

The TLS record framing helpers restate ssl/t1_enc.c:832-975 on top of either
library's AEAD so that record-level vectors can be produced by the reference
and checked against the restatement.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIBORACLE = os.path.join(HERE, "liboracle.so")
LIBREF = os.path.join(HERE, "_ref", "libref.so")
CPUBENCH = os.path.join(HERE, "_ref", "cpubench")

AES_128_GCM, AES_256_GCM, CHACHA20_POLY1305, CHACHA20_POLY1305_OLD = 1, 2, 3, 4
KIND_BY_NAME = {
    "aes-128-gcm": AES_128_GCM,
    "aes-256-gcm": AES_256_GCM,
    "chacha20-poly1305": CHACHA20_POLY1305,
    "chacha20-poly1305-old": CHACHA20_POLY1305_OLD,
}
KEY_LEN = {AES_128_GCM: 16, AES_256_GCM: 32, CHACHA20_POLY1305: 32, CHACHA20_POLY1305_OLD: 32}
FIXED_IV_LEN = {AES_128_GCM: 4, AES_256_GCM: 4, CHACHA20_POLY1305: 12, CHACHA20_POLY1305_OLD: 0}


def build(quiet: bool = True) -> None:
    """Compile liboracle.so (and _ref/* when the reference tree exists)."""
    subprocess.run(["make", "-C", HERE, "-s"], check=True,
                   stdout=subprocess.DEVNULL if quiet else None)


def _buf(b: bytes | None):
    if b is None or len(b) == 0:
        return None
    return (C.c_ubyte * len(b)).from_buffer_copy(b)


class _AeadCtx(C.Structure):
    # oracle_aead_ctx is opaque here; reserve generously (see oracle.h)
    _fields_ = [("raw", C.c_ubyte * 4096)]


class Oracle:
    """CPU restatement (liboracle.so)."""

    def __init__(self, path: str = LIBORACLE):
        if not os.path.exists(path):
            build()
        self.lib = C.CDLL(path)
        L = self.lib
        L.oracle_aead_init.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t, C.c_size_t]
        for fn in (L.oracle_aead_seal, L.oracle_aead_open):
            fn.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_size_t), C.c_size_t,
                           C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
        L.oracle_tls_session_init.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t,
                                              C.c_void_p, C.c_size_t, C.c_uint16]
        L.oracle_tls_open.argtypes = [C.c_void_p, C.c_uint64, C.c_uint8, C.c_void_p, C.c_size_t,
                                      C.c_void_p, C.POINTER(C.c_size_t)]
        L.oracle_tls_seal.argtypes = [C.c_void_p, C.c_uint64, C.c_uint8, C.c_void_p, C.c_size_t,
                                      C.c_void_p, C.POINTER(C.c_size_t)]
        L.oracle_gcm_init.argtypes = [C.c_void_p, C.c_void_p]
        L.oracle_gcm_setiv.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.oracle_gcm_aad.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.oracle_gcm_encrypt.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]
        L.oracle_gcm_decrypt.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]
        L.oracle_gcm_tag.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.oracle_aes_set_encrypt_key.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        L.oracle_aes_encrypt.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_gf128_mul.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_chacha20.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p,
                                      C.c_uint64]
        L.oracle_poly1305_init.argtypes = [C.c_void_p, C.c_void_p]
        L.oracle_poly1305_update.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.oracle_poly1305_finish.argtypes = [C.c_void_p, C.c_void_p]

    # -- AEAD ------------------------------------------------------------
    def aead(self, kind: int, key: bytes, tag_len: int = 0):
        ctx = _AeadCtx()
        ok = self.lib.oracle_aead_init(C.byref(ctx), kind, _buf(key), len(key), tag_len)
        return ctx if ok else None

    def seal(self, ctx, nonce: bytes, pt: bytes, ad: bytes, max_out: int | None = None):
        max_out = len(pt) + 16 if max_out is None else max_out
        out = (C.c_ubyte * max(max_out, 1))()
        ol = C.c_size_t(0)
        ok = self.lib.oracle_aead_seal(C.byref(ctx), out, C.byref(ol), max_out, _buf(nonce),
                                       len(nonce), _buf(pt), len(pt), _buf(ad), len(ad))
        return ok, bytes(out)[:ol.value] if ok else bytes(out)[:max_out]

    def open(self, ctx, nonce: bytes, ct: bytes, ad: bytes, max_out: int | None = None):
        max_out = len(ct) if max_out is None else max_out
        out = (C.c_ubyte * max(max_out, 1))()
        ol = C.c_size_t(0)
        ok = self.lib.oracle_aead_open(C.byref(ctx), out, C.byref(ol), max_out, _buf(nonce),
                                       len(nonce), _buf(ct), len(ct), _buf(ad), len(ad))
        return ok, bytes(out)[:ol.value] if ok else bytes(out)[:max_out]

    # -- TLS records -------------------------------------------------------
    def tls_session(self, kind: int, key: bytes, fixed_iv: bytes, version: int = 0x0303):
        s = _AeadCtx()
        ok = self.lib.oracle_tls_session_init(C.byref(s), kind, _buf(key), len(key),
                                              _buf(fixed_iv), len(fixed_iv), version)
        if not ok:
            raise ValueError("oracle_tls_session_init failed")
        return s

    def tls_seal(self, sess, seq: int, rtype: int, pt: bytes) -> bytes:
        out = (C.c_ubyte * (len(pt) + 8 + 16))()
        bl = C.c_size_t(0)
        r = self.lib.oracle_tls_seal(C.byref(sess), seq, rtype, _buf(pt), len(pt), out,
                                     C.byref(bl))
        if r != 1:
            raise RuntimeError("oracle_tls_seal failed")
        return bytes(out)[:bl.value]

    def tls_open(self, sess, seq: int, rtype: int, body: bytes):
        """Returns (status, plaintext_or_zeros) with tls1_enc's 1 / 0 / -1."""
        out = (C.c_ubyte * max(len(body), 1))()
        pl = C.c_size_t(0)
        r = self.lib.oracle_tls_open(C.byref(sess), seq, rtype, _buf(body), len(body), out,
                                     C.byref(pl))
        return r, bytes(out)[:pl.value] if r != 0 else b""

    # -- primitives --------------------------------------------------------
    def aes_encrypt(self, key: bytes, block: bytes) -> bytes:
        ks = (C.c_ubyte * 256)()
        self.lib.oracle_aes_set_encrypt_key(_buf(key), len(key) * 8, ks)
        out = (C.c_ubyte * 16)()
        self.lib.oracle_aes_encrypt(_buf(block), out, ks)
        return bytes(out)

    def gf128_mul(self, a: bytes, b: bytes) -> bytes:
        out = (C.c_ubyte * 16)()
        self.lib.oracle_gf128_mul(_buf(a), _buf(b), out)
        return bytes(out)

    def gcm(self, key: bytes, iv: bytes, aad: bytes, data: bytes, decrypt: bool = False):
        """Raw CRYPTO_gcm128_* sequence as tests/gcm128test.c:855-913 drives it."""
        ks = (C.c_ubyte * 256)()
        self.lib.oracle_aes_set_encrypt_key(_buf(key), len(key) * 8, ks)
        g = (C.c_ubyte * 2048)()
        self.lib.oracle_gcm_init(g, ks)
        self.lib.oracle_gcm_setiv(g, _buf(iv), len(iv))
        if aad:
            self.lib.oracle_gcm_aad(g, _buf(aad), len(aad))
        out = (C.c_ubyte * max(len(data), 1))()
        if data:
            fn = self.lib.oracle_gcm_decrypt if decrypt else self.lib.oracle_gcm_encrypt
            fn(g, _buf(data), out, len(data))
        tag = (C.c_ubyte * 16)()
        self.lib.oracle_gcm_tag(g, tag, 16)
        return bytes(out)[:len(data)], bytes(tag)

    def chacha20(self, key: bytes, iv: bytes, data: bytes, counter: int = 0) -> bytes:
        out = (C.c_ubyte * max(len(data), 1))()
        self.lib.oracle_chacha20(out, _buf(data), len(data), _buf(key), _buf(iv), counter)
        return bytes(out)[:len(data)]

    def poly1305(self, key: bytes, chunks) -> bytes:
        st = (C.c_ubyte * 256)()
        self.lib.oracle_poly1305_init(st, _buf(key))
        for ch in chunks:
            self.lib.oracle_poly1305_update(st, _buf(ch), len(ch))
        mac = (C.c_ubyte * 16)()
        self.lib.oracle_poly1305_finish(st, mac)
        return bytes(mac)


class _EvpCtx(C.Structure):
    _fields_ = [("aead", C.c_void_p), ("aead_state", C.c_void_p)]


class Reference:
    """The reference LibreSSL EVP_AEAD (oracle/_ref/libref.so)."""

    NAMES = {AES_128_GCM: "EVP_aead_aes_128_gcm", AES_256_GCM: "EVP_aead_aes_256_gcm",
             CHACHA20_POLY1305: "EVP_aead_chacha20_poly1305",
             CHACHA20_POLY1305_OLD: "EVP_aead_chacha20_poly1305_old"}

    def __init__(self, path: str = LIBREF):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        self.lib = C.CDLL(path, mode=os.RTLD_LOCAL | os.RTLD_NOW)
        L = self.lib
        for n in self.NAMES.values():
            getattr(L, n).restype = C.c_void_p
        L.EVP_AEAD_CTX_init.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t,
                                        C.c_size_t, C.c_void_p]
        for fn in (L.EVP_AEAD_CTX_seal, L.EVP_AEAD_CTX_open):
            fn.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_size_t), C.c_size_t,
                           C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
        L.EVP_AEAD_CTX_cleanup.argtypes = [C.c_void_p]

    def aead(self, kind: int, key: bytes, tag_len: int = 0):
        ctx = _EvpCtx()
        a = getattr(self.lib, self.NAMES[kind])()
        ok = self.lib.EVP_AEAD_CTX_init(C.byref(ctx), a, _buf(key), len(key), tag_len, None)
        return ctx if ok else None

    def seal(self, ctx, nonce, pt, ad, max_out=None):
        max_out = len(pt) + 16 if max_out is None else max_out
        out = (C.c_ubyte * max(max_out, 1))()
        ol = C.c_size_t(0)
        ok = self.lib.EVP_AEAD_CTX_seal(C.byref(ctx), out, C.byref(ol), max_out, _buf(nonce),
                                        len(nonce), _buf(pt), len(pt), _buf(ad), len(ad))
        return ok, bytes(out)[:ol.value] if ok else bytes(out)[:max_out]

    def open(self, ctx, nonce, ct, ad, max_out=None):
        max_out = len(ct) if max_out is None else max_out
        out = (C.c_ubyte * max(max_out, 1))()
        ol = C.c_size_t(0)
        ok = self.lib.EVP_AEAD_CTX_open(C.byref(ctx), out, C.byref(ol), max_out, _buf(nonce),
                                        len(nonce), _buf(ct), len(ct), _buf(ad), len(ad))
        return ok, bytes(out)[:ol.value] if ok else bytes(out)[:max_out]


# -- TLS framing over any AEAD object (ssl/t1_enc.c:832-975) -------------------

def tls_nonce(kind: int, fixed_iv: bytes, seq: int, explicit: bytes | None = None) -> bytes:
    seq8 = seq.to_bytes(8, "big")
    if kind == CHACHA20_POLY1305:          # xor_fixed_nonce (t1_enc.c:870-881, 928-939)
        padded = bytes(len(fixed_iv) - 8) + seq8
        return bytes(a ^ b for a, b in zip(padded, fixed_iv))
    if kind == CHACHA20_POLY1305_OLD:      # fixed 0 bytes || seq
        return fixed_iv + seq8
    return fixed_iv + (seq8 if explicit is None else explicit)   # GCM (:887-892, :941-948)


def tls_ad(seq: int, rtype: int, version: int, length: int) -> bytes:
    return seq.to_bytes(8, "big") + bytes([rtype, version >> 8, version & 0xFF,
                                           (length >> 8) & 0xFF, length & 0xFF])


def tls_seal_record(impl, ctx, kind, fixed_iv, seq, rtype, pt, version=0x0303) -> bytes:
    """Record body produced by tls1_enc(s, 1) with `impl` (Oracle or Reference)."""
    nonce = tls_nonce(kind, fixed_iv, seq)
    ok, out = impl.seal(ctx, nonce, pt, tls_ad(seq, rtype, version, len(pt)))
    if not ok:
        raise RuntimeError("seal failed")
    if kind in (AES_128_GCM, AES_256_GCM):
        return seq.to_bytes(8, "big") + out
    return out


def tls_open_record(impl, ctx, kind, fixed_iv, seq, rtype, body, version=0x0303, tag_len=16):
    """(status, plaintext-or-zeros) of tls1_enc(s, 0) with `impl`."""
    gcm = kind in (AES_128_GCM, AES_256_GCM)
    if len(body) < 8:
        return 0, b""
    nonce = tls_nonce(kind, fixed_iv, seq, body[:8] if gcm else None)
    ct = body[8:] if gcm else body
    if len(ct) < tag_len:
        return 0, b""
    n = len(ct) - tag_len
    ok, out = impl.open(ctx, nonce, ct, tls_ad(seq, rtype, version, n), max_out=n)
    return (1, out) if ok else (-1, out)


def run_cpubench(aead: str, op: str, rec_len: int, nrec: int, threads: int, seconds: float,
                 lib: str = LIBREF) -> dict:
    import json
    r = subprocess.run([CPUBENCH, lib, aead, op, str(rec_len), str(nrec), str(threads),
                        str(seconds)], check=True, capture_output=True, text=True)
    return json.loads(r.stdout)
