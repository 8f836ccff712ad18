"""Captured-snapshot OCC, CPU side: a simulated live
concurrent run (tests/live_sim.py) decides every txn inside its own critical
section; the literal snapshot oracle (oracle_occ_snapshot) must reproduce those
decisions from the capture alone.  Plus hand-derived known answers."""
import numpy as np
import pytest

import _oracle as orc
from deneva_amd import EpochBatch, RD, WR, SCAN
from helpers import make_batch, random_batch
from live_sim import simulate


def live_case(seed, n=400, threads=8, n_keys=200, max_len=12, hist0=None, tnc0=0):
    rng = np.random.default_rng(seed)
    b = random_batch(rng, n, max_len, n_keys, p_write=0.3)
    cap = simulate(b.offsets, b.keys, b.acctype, n_threads=threads, seed=seed, hist0=hist0,
                   tnc0=tnc0)
    b = EpochBatch(b.offsets, b.keys, b.acctype, cap["start_tn"], cap["finish_tn"])
    return b, cap


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("threads", [1, 4, 16])
def test_oracle_reproduces_live_run(seed, threads):
    hist0 = [(tn, [int(k) for k in np.random.default_rng(seed + 100).integers(0, 200, 3)])
             for tn in range(1, 41)]
    b, cap = live_case(seed, threads=threads, hist0=hist0, tnc0=40)
    rc = orc.occ_snapshot(b, cap["active_off"], cap["active_idx"], cap["hist_top"],
                          cap["hist_keys"], cap["hist_tn"])
    assert np.array_equal(rc, cap["rc"])
    if threads > 1:
        assert cap["active_off"][-1] > 0  # the run really was concurrent


def test_single_thread_equals_epoch_replay_decisions():
    # one worker: every txn validates and finishes before the next starts, so
    # the active list is always empty; without a history window, nothing aborts
    b, cap = live_case(7, threads=1)
    assert cap["active_off"][-1] == 0
    b2 = EpochBatch(b.offsets, b.keys, b.acctype)
    rc = orc.occ_snapshot(b2, cap["active_off"], cap["active_idx"])
    assert not rc.any()


def test_known_answers():
    # txn0 writes 5; txn1 reads 5 and saw txn0 active -> abort (W_j ∩ R_i)
    # txn2 writes 5 and saw txn0 active -> abort (W_j ∩ W_i)
    # txn3 reads 5 but saw nobody -> commit; txn4 writes 9, saw txn0 -> commit
    # txn5 reads 7 (SCAN) with window (10, 20]: history tn 15 wrote 7 -> abort
    # txn6 same window but hist_top 12 hides tn 15 -> commit
    # txn7 reads 7, finish <= start: window closed -> commit
    b = make_batch([[(5, WR)], [(5, RD)], [(5, WR)], [(5, RD)], [(9, WR), (5, RD)][:1],
                    [(7, SCAN)], [(7, RD)], [(7, RD)]],
                   start_tn=[0, 0, 0, 0, 0, 10, 10, 20], finish_tn=[0, 0, 0, 0, 0, 20, 20, 20])
    aoff = np.array([0, 0, 1, 2, 2, 3, 3, 3, 3], np.uint32)
    aidx = np.array([0, 0, 0], np.uint32)
    top = np.array([99, 99, 99, 99, 99, 99, 12, 99], np.uint64)
    hk = np.array([7, 3], np.uint64)
    ht = np.array([15, 11], np.uint64)
    rc = orc.occ_snapshot(b, aoff, aidx, top, hk, ht)
    assert rc.tolist() == [0, 2, 2, 0, 0, 2, 0, 0]
