"""Batch-shape hints (tlsgpu_sessions_hint, include/tlsgpu.h): the rule a caller
applies to a batch it built (talos_amd.batch_hints) matches the engine's own
host-side rule for host-resident batches (engine.cpp host_hints) and the
device's kernel selection (pack: nb + 2 <= 64; per-wave sessions: runs x 12 >
records).  CPU only."""
import numpy as np

import talos_amd as ta


def test_uniform_long_grouped_batch_gets_both_hints():
    lengths = np.full(65536 // 16, 16384)
    sessions = np.repeat(np.arange(64), 64)
    assert ta.batch_hints(lengths, sessions, seal=False) == \
        ta.HINT_NO_SHORT_RECORDS | ta.HINT_SESSION_RUNS


def test_short_record_limit_open_and_seal():
    # open: 8-B explicit nonce + 16-B tag around a 992-B (62-block) plaintext
    s = np.zeros(64, dtype=np.int64)
    assert ta.batch_hints(np.full(64, 1016), s, seal=False) & ta.HINT_NO_SHORT_RECORDS == 0
    assert ta.batch_hints(np.full(64, 1017), s, seal=False) & ta.HINT_NO_SHORT_RECORDS
    assert ta.batch_hints(np.full(64, 992), s, seal=True) & ta.HINT_NO_SHORT_RECORDS == 0
    assert ta.batch_hints(np.full(64, 993), s, seal=True) & ta.HINT_NO_SHORT_RECORDS


def test_session_run_rule():
    lengths = np.full(120, 16384)
    assert ta.batch_hints(lengths, np.repeat(np.arange(10), 12), False) & ta.HINT_SESSION_RUNS
    assert ta.batch_hints(lengths, np.repeat(np.arange(12), 10), False) & ta.HINT_SESSION_RUNS == 0
    assert ta.batch_hints(lengths, np.arange(120) % 7, False) & ta.HINT_SESSION_RUNS == 0
