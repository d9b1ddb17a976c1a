"""Shared pytest configuration.

Markers:
  gpu — needs a real MI355X (runs on the GPU box via `pytest -m gpu`).
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs an MI355X GPU")


def pytest_collection_modifyitems(session, config, items):
    """The EVP coalescing-queue test turns batching on for the rest of the
    process (EVP contexts then live in the shared pool); run it last so every
    other EVP test exercises the per-call path."""
    items.sort(key=lambda it: "test_evp_queue" in it.nodeid)


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    pyoracle.build()
    return pyoracle.Oracle()


@pytest.fixture(scope="session")
def reference():
    import pyoracle
    if not os.path.exists(pyoracle.LIBREF):
        pytest.skip("oracle/_ref/libref.so not built (reference tree absent)")
    return pyoracle.Reference()


def load_aeadtests(path=None):
    """Parse the reference's aeadtests.txt data file (tests/aeadtest.c:60-75 format)."""
    path = path or os.path.join(ROOT, "tests", "golden", "aeadtests.txt")
    cases, cur, line_no, last_aead = [], {}, 0, None
    for line in open(path):
        line_no += 1
        line = line.strip()
        if line.startswith("#"):
            continue
        if not line:
            if cur:
                # the AEAD name buffer persists across cases (aeadtest.c:269)
                last_aead = cur.setdefault("AEAD", last_aead)
                for k in ("KEY", "NONCE", "IN", "AD", "CT", "TAG"):
                    cur.setdefault(k, b"")
                cases.append(cur)
                cur = {}
            continue
        k, _, v = line.partition(":")
        v = v.strip()
        cur[k.strip()] = v if k.strip() == "AEAD" else bytes.fromhex(v)
        cur.setdefault("line", line_no)
    if cur:
        cur.setdefault("AEAD", last_aead)
        for k in ("KEY", "NONCE", "IN", "AD", "CT", "TAG"):
            cur.setdefault(k, b"")
        cases.append(cur)
    return cases
