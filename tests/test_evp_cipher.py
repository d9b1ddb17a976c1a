"""The legacy EVP_CIPHER GCM surface (EVP_aes_{128,256}_gcm, crypto/evp/
e_aes.c:715-1059) of libtlsgpu.so against the reference
itself: oracle/_ref/evp_cipher_check drives LibreSSL 2.4.1's own generic EVP
code (evp_enc.c in oracle/_ref/libssl_ref.so) over every GCM feature — IV
lengths 1..64, AAD and data in random pieces, tag get/set and truncation,
a failing tag, EVP_CIPHER_CTX_copy mid-stream, the TLS record mode — and prints
a transcript of all outputs and return values.  With libtlsgpu.so
LD_PRELOADed the EVP_aes_*_gcm objects (and so all cipher work) are the GPU
engine's; the transcript must be byte-identical to the reference's own run.
"""
import json
import os
import subprocess

import pytest

from conftest import ROOT

CHECK = os.path.join(ROOT, "oracle", "_ref", "evp_cipher_check")
LIB = os.path.join(ROOT, "talos_amd", "libtlsgpu.so")


def _run(preload):
    if not os.path.exists(CHECK):
        pytest.skip("oracle/_ref/evp_cipher_check not built (reference tree absent at build time)")
    env = dict(os.environ)
    env.pop("LD_PRELOAD", None)
    if preload:
        env["LD_PRELOAD"] = LIB
    r = subprocess.run([CHECK], capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout, json.loads(r.stderr.strip().splitlines()[-1])


def test_evp_cipher_reference_transcript():
    """The reference's own run: tags verify, the flipped tag fails, TLS records round-trip."""
    out, info = _run(False)
    assert not info["tlsgpu_interposed"]
    assert out.count("open final 1 0 equal 1") == 2 * 9
    assert out.count("open final 0 0") == 2 * 9
    assert "open 100 pad 16 r -1 equal 0" in out


@pytest.mark.gpu
def test_evp_cipher_gpu_matches_reference():
    ref, _ = _run(False)
    gpu, info = _run(True)
    assert info["tlsgpu_interposed"] and info["gpu_programs"] > 100
    for n, (a, b) in enumerate(zip(ref.splitlines(), gpu.splitlines())):
        assert a == b, f"transcript line {n + 1}: reference {a[:120]!r} != gpu {b[:120]!r}"
    assert len(ref.splitlines()) == len(gpu.splitlines())
