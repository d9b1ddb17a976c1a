#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ (run in the build container).

Inputs (read-only, never copied as source):
  * /root/reference/src/libressl-2.4.1/tests/aeadtests.txt — the reference's
    EVP_AEAD KAT data file, copied verbatim as a data fixture;
  * the vector tables inside the reference's tests/gcm128test.c:78-851,
    tests/chachatest.c:36-221 and tests/poly1305test.c (NaCl / wrap / total
    vectors) — only the numbers are extracted, re-encoded as JSON;
  * oracle/_ref/libref.so — the reference compiled from its own sources
    (oracle/Makefile); it seals TLS records with the t1_enc.c:832-975 framing
    to give record-level vectors at sizes no reference test covers
    (nothing pins 16 KiB / 1400 B / record level).

  * oracle/_ref/batch_digest (our generator over oracle/_ref/libssl_ref.so,
    the whole reference libcrypto compiled from its own sources) — SHA-256
    digests of the full-size seeded batches of SURVEY.md §8d (configs B, C, D,
    plus session-count variants), sealed and opened by the reference with the
    t1_enc framing and the workload rules of talos_amd/workload.py.

  * oracle/_ref/wire_capture (our harness over oracle/_ref/libssl_ref.so, the
    reference's unmodified libssl) — the raw wire bytes the reference's record
    layer (do_ssl3_write -> tls1_enc, s3_pkt.c:560-762, t1_enc.c:832-975)
    emitted for a list of application writes after a real handshake, with the
    record state it used (SSL_AEAD_CTX fields, ssl_locl.h:527-543; the key
    handed to EVP_AEAD_CTX_init; s3->write_sequence), for the four AEAD suites.

Outputs: aeadtests.txt, gcm128_vectors.json, chacha_vectors.json,
poly1305_vectors.json, records.json, batch_digests.json, wire_ref.json.
"""
from __future__ import annotations

import hashlib
import json
import os
import re
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle as po  # noqa: E402

REFT = "/root/reference/src/libressl-2.4.1/tests"


def c_byte_list(text: str) -> bytes:
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)   # drop C comments
    vals = re.findall(r"0x([0-9a-fA-F]{1,2})|\b(\d+)\b", text)
    return bytes(int(h, 16) if h else int(d) for h, d in vals)


def parse_gcm128(path: str):
    src = open(path).read()
    body = src[src.index("gcm128_tests[] = {"):src.index("#define N_TESTS")]
    cases = re.split(r"/\*\s*Test Case (\d+)\.\s*\*/", body)
    out = []
    for i in range(1, len(cases), 2):
        num, txt = int(cases[i]), cases[i + 1]
        f = {}
        for name in ("K", "IV", "P", "A", "C", "T"):
            m = re.search(r"\.%s\s*=\s*\{(.*?)\}" % name, txt, re.S)
            f[name] = c_byte_list(m.group(1)) if m else b""
        lens = {n: int(v) for n, v in re.findall(r"\.(\w+)_len\s*=\s*(\d+)", txt)}
        rec = {"case": num}
        for name in ("K", "IV", "P", "A", "C"):
            n = lens.get(name, 0)
            b = f[name][:n]
            rec[name] = (b + bytes(n - len(b))).hex()   # `{0}` => zero-filled
        rec["T"] = (f["T"] + bytes(16 - len(f["T"]))).hex()
        out.append(rec)
    return out


def parse_chacha(path: str):
    src = open(path).read()
    body = src[src.index("chacha_test_vectors[] = {"):src.index("#define N_VECTORS")]
    out = []
    for m in re.finditer(r'\{\s*"([^"]*)",\s*\{(.*?)\},\s*\{(.*?)\},\s*(\d+),\s*\{(.*?)\},\s*\}',
                         body, re.S):
        desc, key, iv, n, ks = m.groups()
        ks_b = c_byte_list(ks)
        out.append({"desc": desc, "key": c_byte_list(key).hex(), "iv": c_byte_list(iv).hex(),
                    "len": int(n), "out": (ks_b + bytes(int(n) - len(ks_b))).hex()})
    return out


def parse_poly1305(path: str):
    src = open(path).read()
    arrs = {}
    for m in re.finditer(r"static const unsigned char (\w+)\[(\d*)\]\s*=\s*\{(.*?)\};", src, re.S):
        b = c_byte_list(m.group(3))
        n = int(m.group(2)) if m.group(2) else len(b)
        arrs[m.group(1)] = (b + bytes(n - len(b))).hex()   # C zero-fills the rest
    return arrs


def fill_bytes(seed: int, index: int, n: int) -> bytes:
    """Counter-based SplitMix64 stream, identical to oracle_fill_bytes()."""
    M = (1 << 64) - 1
    st = (seed ^ (index * 0xD1B54A32D192ED03)) & M
    out = bytearray()
    w = 0
    while len(out) < n:
        w += 1
        z = (st + w * 0x9E3779B97F4A7C15) & M
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        z ^= z >> 31
        out += z.to_bytes(8, "little")
    return bytes(out[:n])


RECORD_SIZES = [0, 1, 13, 15, 16, 17, 31, 32, 63, 64, 65, 100, 255, 256, 1023, 1024,
                1400, 4095, 4096, 16383, 16384]
SEQS = [0, 1, 0xFF, 0x1FF, 0xFFFFFFFF, 0x0123456789ABCDEF, 0xFFFFFFFFFFFFFFFE]
HEX_LIMIT = 300


def make_records(ref: po.Reference):
    recs = []
    for kind_name, kind in po.KIND_BY_NAME.items():
        for i, n in enumerate(RECORD_SIZES):
            seed = 0x5EED1000 + 97 * kind + i
            key = fill_bytes(seed, 1, po.KEY_LEN[kind])
            fiv = fill_bytes(seed, 2, po.FIXED_IV_LEN[kind])
            seq = SEQS[i % len(SEQS)]
            rtype = 23 if i % 5 else 22
            pt = fill_bytes(seed, 3, n)
            ctx = ref.aead(kind, key)
            body = po.tls_seal_record(ref, ctx, kind, fiv, seq, rtype, pt)
            st, back = po.tls_open_record(ref, ctx, kind, fiv, seq, rtype, body)
            assert st == 1 and back == pt
            rec = {"aead": kind_name, "key": key.hex(), "fixed_iv": fiv.hex(), "seq": seq,
                   "type": rtype, "version": 0x0303, "pt_seed": seed, "pt_len": n,
                   "body_len": len(body), "body_sha256": hashlib.sha256(body).hexdigest()}
            if len(body) <= HEX_LIMIT:
                rec["body"] = body.hex()
            recs.append(rec)
    return recs


# name: (aead, records, sessions, seed, tamper_every, length or "zipf")
BATCHES = {
    # full-size BASELINE configs (checked on the GPU)
    "B": ("aes-128-gcm", 65536, 1024, 0x5EED0001, 1024, 16384),
    "C": ("chacha20-poly1305", 1 << 20, 4096, 0x5EED0002, 1024, 1400),
    "D": ("aes-256-gcm", 1 << 18, 1024, 0x5EED0003, 1024, "zipf"),
    # session-count sensitivity: one session, one record per session
    "B_S1": ("aes-128-gcm", 65536, 1, 0x5EED0001, 1024, 16384),
    "B_Sn": ("aes-128-gcm", 65536, 65536, 0x5EED0001, 1024, 16384),
    # records of 1,024 connections interleaved (a many-connection server batch)
    "B_inter": ("aes-128-gcm", 65536, 1024, 0x5EED0001, 1024, 16384, "interleave"),
    "D_inter": ("aes-256-gcm", 1 << 18, 8192, 0x5EED0003, 1024, "zipf", "interleave"),
    # small batches the CPU restatement re-derives in seconds (tests/test_oracle_kat.py)
    "B_small": ("aes-128-gcm", 96, 8, 0x5EED0001, 16, 16384),
    "C_small": ("chacha20-poly1305", 512, 32, 0x5EED0002, 64, 1400),
    "D_small": ("aes-256-gcm", 256, 16, 0x5EED0003, 32, "zipf"),
    "old_small": ("chacha20-poly1305-old", 128, 8, 0x5EED0005, 16, 1000),
    "inter_small": ("aes-256-gcm", 200, 7, 0x5EED0006, 16, "zipf", "interleave"),
    # a shard of a split batch at CPU-restatement size (config E's rules)
    "E_shard_small": ("aes-128-gcm", 512, 64, 0x5EED0004, 16, 1024, "range=256:384"),
}
# config E: ONE batch of 524,288 x 16 KiB records, 8,192 sessions
# of 64 records, split across 8 GPUs; shard r = records [65536 r, 65536 (r + 1))
E_RECORDS, E_SESSIONS, E_SHARDS = 524288, 8192, 8
for _r in range(E_SHARDS):
    _lo = _r * (E_RECORDS // E_SHARDS)
    BATCHES[f"E_shard{_r}"] = ("aes-128-gcm", E_RECORDS, E_SESSIONS, 0x5EED0004, 1024, 16384,
                               f"range={_lo}:{_lo + E_RECORDS // E_SHARDS}")


def make_batch_digests(only=None):
    import subprocess
    import tempfile

    import numpy as np
    sys.path.insert(0, ROOT)
    from talos_amd.workload import zipf_lengths
    exe = os.path.join(ROOT, "oracle", "_ref", "batch_digest")
    out = {}
    for name, (aead, n, S, seed, tamper, ln, *order) in BATCHES.items():
        if only and name not in only:
            continue
        with tempfile.NamedTemporaryFile(suffix=".u32") as f:
            if ln == "zipf":
                f.write(zipf_lengths(n, seed).astype(np.uint32).tobytes())
                f.flush()
                arg = "@" + f.name
            else:
                arg = str(ln)
            r = subprocess.run([exe, aead, str(n), str(S), hex(seed), str(tamper), arg] + order,
                               check=True, capture_output=True, text=True)
        d = json.loads(r.stdout)
        d["lengths"] = ln
        out[name] = d
        print(name, d["sealed_sha256"][:16], d["opened_sha256"][:16], flush=True)
    return out


WIRE_SUITES = {  # cipher string -> pyoracle AEAD kind
    "ECDHE-RSA-AES128-GCM-SHA256": "AES_128_GCM",
    "ECDHE-RSA-AES256-GCM-SHA384": "AES_256_GCM",
    "ECDHE-RSA-CHACHA20-POLY1305": "CHACHA20_POLY1305",
    "ECDHE-RSA-CHACHA20-POLY1305-OLD": "CHACHA20_POLY1305_OLD",
}


def make_wire_ref():
    """Run oracle/_ref/wire_capture per suite; keep its metadata and the wire
    bytes of both directions (base64)."""
    import base64
    import subprocess
    import tempfile
    exe = os.path.join(ROOT, "oracle", "_ref", "wire_capture")
    pem = os.path.join(HERE, "server.pem")
    suites = {}
    with tempfile.TemporaryDirectory() as td:
        for cipher, kind in WIRE_SUITES.items():
            prefix = os.path.join(td, "w")
            r = subprocess.run([exe, "-p", pem, "-c", cipher, "-o", prefix], check=True,
                               capture_output=True, text=True)
            d = json.loads(r.stdout)
            assert d["cipher"] == cipher, (d["cipher"], cipher)
            for dr in d["directions"]:
                wire = open(f"{prefix}.{dr['dir']}.bin", "rb").read()
                assert len(wire) == dr["wire_bytes"]
                dr["wire_b64"] = base64.b64encode(wire).decode()
            d["aead"] = kind
            suites[cipher] = d
            print(cipher, [dr["wire_bytes"] for dr in d["directions"]], flush=True)
    return {"generator": "tests/golden/make_golden.py via oracle/_ref/wire_capture "
                         "(reference libssl + libcrypto, oracle/_ref/libssl_ref.so)",
            "payload": "write k of direction dir (c2s = 1, s2c = 2) is SplitMix64 fill "
                       "keyed (dir << 32) | k, oracle/wire_capture.c fill()",
            "suites": suites}


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--wire":
        json.dump(make_wire_ref(), open(os.path.join(HERE, "wire_ref.json"), "w"))
        return
    if len(sys.argv) > 2 and sys.argv[1] == "--digests":
        # recompute only the named batch digests and merge them into the fixture
        path = os.path.join(HERE, "batch_digests.json")
        d = json.load(open(path))
        d["batches"].update(make_batch_digests(set(sys.argv[2:])))
        json.dump(d, open(path, "w"), indent=1)
        return
    os.makedirs(HERE, exist_ok=True)
    shutil.copyfile(os.path.join(REFT, "aeadtests.txt"), os.path.join(HERE, "aeadtests.txt"))
    json.dump(parse_gcm128(os.path.join(REFT, "gcm128test.c")),
              open(os.path.join(HERE, "gcm128_vectors.json"), "w"), indent=1)
    json.dump(parse_chacha(os.path.join(REFT, "chachatest.c")),
              open(os.path.join(HERE, "chacha_vectors.json"), "w"), indent=1)
    json.dump(parse_poly1305(os.path.join(REFT, "poly1305test.c")),
              open(os.path.join(HERE, "poly1305_vectors.json"), "w"), indent=1)
    po.build()
    ref = po.Reference()
    json.dump({"generator": "tests/golden/make_golden.py via oracle/_ref/libref.so",
               "records": make_records(ref)},
              open(os.path.join(HERE, "records.json"), "w"), indent=1)
    json.dump({"generator": "tests/golden/make_golden.py via oracle/_ref/batch_digest "
                            "(reference libcrypto, oracle/_ref/libssl_ref.so)",
               "batches": make_batch_digests()},
              open(os.path.join(HERE, "batch_digests.json"), "w"), indent=1)
    json.dump(make_wire_ref(), open(os.path.join(HERE, "wire_ref.json"), "w"))
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
