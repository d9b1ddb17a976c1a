"""Drop-in proof (BASELINE configs[0]): the reference's own,
unmodified LibreSSL 2.4.1 libssl + libcrypto (oracle/_ref/libssl_ref.so,
compiled from /root/reference by oracle/Makefile) runs a TLS 1.2 memory-BIO
loopback (oracle/ssl_loopback.c, the shape of tests/ssltest.c:1324 doit) with
libtlsgpu.so LD_PRELOADed: tls1_enc's EVP_AEAD_CTX_seal/open PLT calls
(ssl/t1_enc.c:911,964) bind to the GPU engine, the handshake stays on the CPU.

Checked: every payload byte round-trips through SSL_write/SSL_read both ways,
and libtlsgpu's own call counters equal the number of records the exchange
must seal and open (both Finished messages + ceil(len/16384) records per write,
s3_pkt.c:531-536), i.e. every record cipher call ran on the GPU.  The CPU-only
run of the same program (no preload) is the configs[0] plumbing baseline.
"""
import json
import os
import subprocess

import pytest

from conftest import ROOT

LOOPBACK = os.path.join(ROOT, "oracle", "_ref", "ssl_loopback")
PEM = os.path.join(ROOT, "tests", "golden", "server.pem")
LIB = os.path.join(ROOT, "talos_amd", "libtlsgpu.so")
CIPHERS = ["ECDHE-RSA-AES128-GCM-SHA256", "ECDHE-RSA-AES256-GCM-SHA384",
           "ECDHE-RSA-CHACHA20-POLY1305", "ECDHE-RSA-CHACHA20-POLY1305-OLD"]


def _run(args, preload=False, env_extra=None, timeout=100):
    if not os.path.exists(LOOPBACK):
        pytest.skip("oracle/_ref/ssl_loopback not built (reference tree absent at build time)")
    env = dict(os.environ)
    env.pop("LD_PRELOAD", None)
    if preload:
        env["LD_PRELOAD"] = LIB
    env.update(env_extra or {})
    r = subprocess.run([LOOPBACK, "-p", PEM] + [str(a) for a in args], capture_output=True,
                       text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("cipher", CIPHERS)
def test_loopback_reference_cpu(cipher):
    """configs[0] as the reference runs it: CPU only, no interposition."""
    d = _run(["-c", cipher, "-n", 500])
    assert d["ok"] and d["cipher"] == cipher and not d["tlsgpu_interposed"]


@pytest.mark.gpu
@pytest.mark.parametrize("cipher,records", [(CIPHERS[0], 32768)] + [(c, 2000) for c in CIPHERS[1:]])
def test_loopback_libtlsgpu_preloaded(cipher, records):
    """Unmodified libssl + LD_PRELOAD=libtlsgpu.so: 1 KiB records, every record
    sealed and opened by the GPU (AES-128-GCM: 64 MiB through the loopback)."""
    d = _run(["-c", cipher, "-n", records], preload=True, timeout=110)
    assert d["ok"] and d["cipher"] == cipher and d["tlsgpu_interposed"]
    assert d["tlsgpu_seal_calls"] == d["records_sealed_expected"] == 2 * (1 + records)
    assert d["tlsgpu_open_calls"] == d["records_opened_expected"]


@pytest.mark.gpu
def test_loopback_libtlsgpu_fragmenting_writes():
    """40,000-B SSL_writes: do_ssl3_write splits at max_send_fragment into
    16384 + 16384 + 7232-B records (s3_pkt.c:531-536); all of them on the GPU."""
    d = _run(["-c", CIPHERS[0], "-r", 40000, "-n", 64, "-t", 2], preload=True)
    assert d["ok"] and d["tlsgpu_seal_calls"] == d["records_sealed_expected"] == 2 * 2 * (1 + 64 * 3)
    assert d["tlsgpu_open_calls"] == d["records_opened_expected"]


@pytest.mark.gpu
@pytest.mark.parametrize("cipher", [CIPHERS[0], CIPHERS[2]])
def test_loopback_libtlsgpu_batching_queue(cipher):
    """16 connections on 16 threads with the coalescing queue on
    (TLSGPU_EVP_BATCH_US): same bytes, same record counts."""
    d = _run(["-c", cipher, "-n", 400, "-t", 16], preload=True,
             env_extra={"TLSGPU_EVP_BATCH_US": "100"})
    assert d["ok"] and d["tlsgpu_seal_calls"] == d["records_sealed_expected"] == 16 * 2 * 401
    assert d["tlsgpu_open_calls"] == d["records_opened_expected"]
