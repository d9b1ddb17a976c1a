"""EVP coalescing queue: many threads calling the drop-in
EVP_AEAD_CTX_seal/open concurrently are served in shared device batches, with
results bit-exact against the oracle and the reference's error semantics
(bad tag -> 0, zero-filled output) kept per call."""
import os
import random
import sys
import threading

import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle as po  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ta():
    import talos_amd
    talos_amd.load_library()
    talos_amd.evp_set_batching(300, 0, 64)
    yield talos_amd
    talos_amd.evp_set_batching(0)  # keep pooling, no waiting window for later tests


def test_evp_queue_concurrent_calls_match_oracle(ta, oracle):
    kinds = [po.AES_128_GCM, po.AES_256_GCM, po.CHACHA20_POLY1305, po.CHACHA20_POLY1305_OLD]
    nthreads, per_thread = 12, 12
    b0, j0 = ta.evp_batch_stats()
    errors = []

    def worker(t):
        rnd = random.Random(1000 + t)
        kind = kinds[t % len(kinds)]
        key = bytes(rnd.randrange(256) for _ in range(po.KEY_LEN[kind]))
        ctx = ta.EvpAead(kind, key)
        octx = oracle.aead(kind, key)
        nlen = 8 if kind == po.CHACHA20_POLY1305_OLD else 12
        try:
            assert ctx.ok == 1
            for i in range(per_thread):
                nonce = bytes(rnd.randrange(256) for _ in range(nlen))
                pt = bytes(rnd.randrange(256) for _ in range(rnd.choice([0, 1, 15, 16, 100, 1400, 5000])))
                ad = bytes(rnd.randrange(256) for _ in range(rnd.choice([0, 5, 13, 40])))
                ok, exp = oracle.seal(octx, nonce, pt, ad)
                ok2, got, ol = ctx.seal(nonce, pt, ad)
                assert ok == ok2 == 1 and got == exp and ol == len(exp), (t, i)
                ok3, back, ol3 = ctx.open(nonce, got, ad)
                assert ok3 == 1 and back == pt and ol3 == len(pt), (t, i)
                if got:
                    bad = bytearray(got)
                    bad[rnd.randrange(len(bad))] ^= 4
                    ok4, z, ol4 = ctx.open(nonce, bytes(bad), ad)
                    assert ok4 == 0 and z == bytes(len(bad)) and ol4 == 0, (t, i)
        except Exception as exc:  # surfaced below
            errors.append(repr(exc))
        finally:
            ctx.cleanup()

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(nthreads)]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    assert not errors, errors[:3]
    b1, j1 = ta.evp_batch_stats()
    jobs, batches = j1 - j0, b1 - b0
    assert jobs >= nthreads * per_thread * 2
    assert batches < jobs  # calls from different threads shared launches
