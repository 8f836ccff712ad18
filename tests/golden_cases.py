"""The committed golden fixtures (tests/golden/*.dccb) as replayable cases.

Each fixture holds a batch in one of BASELINE.json's config shapes plus the
decisions of the oracle's LITERAL replay at the time the fixture was written
(tests/golden/make_fixtures.py): OptCC central_validate / central_finish
(concurrency_control/occ.cpp:116-294) for OCC, and the Row_lock CALVIN
grant / release simulation (concurrency_control/row_lock.cpp:52-381) for
Calvin.  The reference ships no vectors of its own, so
these files are what pins the checker: an edit to oracle/*.c that changes a
decision fails tests/test_golden.py, and the GPU suite compares the engine
with the stored vectors, not only with a live oracle run.
"""
from __future__ import annotations

import os

import numpy as np

import deneva_amd as d

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

OCC_FIXTURES = ["c1_ycsb_theta06_seed7.dccb", "c2_ycsb_theta09_3000.dccb",
                "c3_tpcc_4wh_2048.dccb"]
HIST_FIXTURES = ["occ_hist_epoch0.dccb", "occ_hist_epoch1.dccb"]
CALVIN_FIXTURES = ["c4_calvin_16p_2000.dccb"]
ALL_FIXTURES = OCC_FIXTURES + HIST_FIXTURES + CALVIN_FIXTURES


def load(name):
    """(EpochBatch, info dict, decisions dict) of one fixture."""
    return d.read_batch_file(os.path.join(GOLDEN, name))


def history_of(b, tn):
    """(key, tn) of every write of a committed txn: central_finish pushes the
    committed write set with its tn onto `history` (occ.cpp:277-286)."""
    off = np.asarray(b.offsets, np.int64)
    txn = np.repeat(np.arange(b.n_txn), np.diff(off))
    sel = (np.asarray(b.acctype) == d.WR) & (tn[txn] > 0)
    return np.asarray(b.keys)[sel].copy(), tn[txn][sel].astype(np.uint64)


def history_epochs():
    """The two history-window epochs in order, with the history each one sees:
    [(batch, info, decisions, hist_keys, hist_tn), ...]."""
    b0, i0, d0 = load(HIST_FIXTURES[0])
    b1, i1, d1 = load(HIST_FIXTURES[1])
    hk, ht = history_of(b0, d0["commit_tn"])
    empty = np.zeros(0, np.uint64)
    return [(b0, i0, d0, empty, empty), (b1, i1, d1, hk, ht)]
