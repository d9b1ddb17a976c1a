"""The draft ("old") ChaCha20-Poly1305 AEAD per call on one wave (round 5,
chacha_wave.h cc_wave_job_old): e_chacha20poly1305.c:124-286 with the 8-byte
nonce — ChaCha20 with a 64-bit block counter, and Poly1305 over the unpadded
byte stream AD || le64(|AD|) || CT || le64(|CT|) (:160-170), split over the
wave's lanes by stream block.  The stream's block boundaries fall wherever
|AD| + 8 puts them, so the cases sweep AD lengths 0..33 against ciphertext
lengths around 16-byte and 64-byte boundaries and the 4,032-byte first pass,
through the doorbell server (op 21) and through the launched one-wave kernel
(TLSGPU_EVP_DOORBELL=0), every output against the oracle; tampered records
return 0 with the output zero-filled.
"""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

_CHILD = r"""
import faulthandler; faulthandler.enable()
import os, random, sys
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, os.path.join(sys.argv[1], "oracle"))
import talos_amd as ta, pyoracle as po
ta.load_library()
orc = po.Oracle()
kind = po.CHACHA20_POLY1305_OLD
rnd = random.Random(int(sys.argv[2]))
cases = 0
for tag_len in (16, 10):
    key = bytes(rnd.randrange(256) for _ in range(32))
    ctx, octx = ta.EvpAead(kind, key, tag_len), orc.aead(kind, key, tag_len)
    assert ctx.ok == 1
    for ad_len in list(range(0, 18)) + [24, 31, 32, 33, 100]:
        for n in (0, 1, 7, 8, 15, 16, 17, 63, 64, 65, 100, 1400, 4031, 4032, 4033, 4100, 9000):
            if ad_len > 17 and n not in (0, 17, 1400, 4033):
                continue
            nonce = bytes(rnd.randrange(256) for _ in range(8))
            pt = bytes(rnd.randrange(256) for _ in range(n))
            ad = bytes(rnd.randrange(256) for _ in range(ad_len))
            ok, exp = orc.seal(octx, nonce, pt, ad)
            ok2, got, ol = ctx.seal(nonce, pt, ad)
            assert ok == ok2 == 1 and got == exp and ol == len(exp), (ad_len, n, tag_len)
            ok3, back, _ = ctx.open(nonce, got, ad)
            assert ok3 == 1 and back == pt, (ad_len, n, tag_len, "open")
            bad = bytearray(got); bad[rnd.randrange(len(bad))] ^= 1 << rnd.randrange(8)
            ok4, z, _ = ctx.open(nonce, bytes(bad), ad)
            assert ok4 == 0 and not any(z), (ad_len, n, "tampered record accepted or not zero-filled")
            cases += 1
    ctx.cleanup()
jobs, _ = ta.evp_doorbell_stats()
print("OK", cases, jobs)
"""


@pytest.mark.parametrize("doorbell", ["4", "0"])
def test_evp_chacha_old_wave_matches_oracle(doorbell):
    env = dict(os.environ, TLSGPU_EVP_DOORBELL=doorbell, TLSGPU_CRASH_TRACE="1")
    env.pop("TLSGPU_EVP_BATCH_US", None)
    r = subprocess.run([sys.executable, "-c", _CHILD, ROOT, "61"], env=env,
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
    _, cases, jobs = r.stdout.split()[-3:]
    assert int(cases) > 300
    if doorbell != "0":   # every call went through the server (op 21)
        assert int(jobs) >= 3 * int(cases), r.stdout
    else:
        assert int(jobs) == 0, r.stdout
