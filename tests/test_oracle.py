"""CPU: the oracle restatements agree with each other and with hand-derived
known-answer cases read off the reference source (see oracle/oracle.h for the
pinning status: the reference ships no golden vectors for this path)."""
import numpy as np
import pytest

import _oracle as orc
import deneva_amd as d
from deneva_amd import RD, SCAN, WR, XP
from helpers import chain_batch, make_batch, random_batch


# ---------------------------------------------------------------- OCC KATs
def both(b, **kw):
    r1, t1, c1 = orc.occ(b, literal=True, **kw)
    r2, t2, c2 = orc.occ(b, literal=False, **kw)
    assert np.array_equal(r1, r2) and np.array_equal(t1, t2) and c1 == c2
    return r1, t1, c1


def test_kat_asymmetric_backward_validation():
    # occ.cpp:185-199 checks an ACTIVE write set against the validating txn's
    # read then write set; a later writer of a row an earlier txn only READ is
    # never checked (backward validation).
    rc, tn, tnc = both(make_batch([[(1, RD), (2, WR)], [(1, WR)], [(2, RD)]]))
    assert list(rc) == [0, 0, 2]
    assert list(tn) == [1, 2, 0] and tnc == 2


def test_kat_readonly_and_aborted_never_kill():
    # read-only txns never enter `active` (occ.cpp:151-154); an aborted txn is
    # unlinked immediately (occ.cpp:219-235)
    rc, tn, _ = both(make_batch([[(1, RD)], [(1, WR)], [(1, RD), (2, WR)], [(2, RD)]]))
    assert list(rc) == [0, 0, 2, 0]
    assert list(tn) == [0, 1, 0, 0]  # read-only commits take no tn (occ.cpp:254)


def test_kat_write_write_conflict():
    rc, _, _ = both(make_batch([[(3, WR)], [(3, WR)], [(4, WR)], [(4, WR), (3, RD)]]))
    assert list(rc) == [0, 2, 0, 2]


def test_kat_xp_and_scan_are_reads():
    # get_rw_set puts every non-WR access into the read set (occ.cpp:296-317)
    rc, tn, _ = both(make_batch([[(7, XP)], [(7, WR)], [(7, SCAN)], [(7, XP)]]))
    assert list(rc) == [0, 0, 2, 2]
    assert list(tn) == [0, 1, 0, 0]


def test_kat_history_window():
    # occ.cpp:160-180: only when finish_tn > start_tn; skip entries with
    # tn > finish_tn; check entries with tn > start_tn against the READ set
    hk = np.array([7, 8, 9], np.uint64)
    ht = np.array([5, 9, 12], np.uint64)
    b = make_batch([[(7, RD)], [(7, RD)], [(8, RD)], [(8, WR)], [(7, RD)], [(9, RD)]],
                   start_tn=[4, 5, 8, 8, 1, 0], finish_tn=[6, 9, 9, 20, 1, 11])
    rc, _, _ = both(b, hist_keys=hk, hist_tn=ht)
    assert list(rc) == [2, 0, 2, 0, 0, 0]


def test_kat_tnc_continues():
    b = make_batch([[(1, WR)], [(2, WR)], [(3, RD)]])
    rc, tn, tnc = both(b, tnc=41)
    assert list(tn) == [42, 43, 0] and tnc == 43


def test_kat_chain():
    rc, _, _ = both(chain_batch(12))
    assert list(rc) == [0, 2] * 6


# --------------------------------------------------------- cross-checks
@pytest.mark.parametrize("theta", [0.0, 0.6, 0.9, 0.99])
def test_replay_equals_hash_ycsb(theta):
    both(d.gen_ycsb(n_txn=3000, zipf_theta=theta, req_per_query=10, table_size=65536))


def test_replay_equals_hash_random():
    rng = np.random.default_rng(5)
    for n_keys in (20, 400, 100000):
        both(random_batch(rng, 600, 24, n_keys, types=(RD, WR, XP, SCAN)))


def test_replay_equals_hash_history_random():
    rng = np.random.default_rng(6)
    b = random_batch(rng, 800, 10, 300)
    st = rng.integers(0, 60, size=b.n_txn).astype(np.uint64)
    b.start_tn = st
    b.finish_tn = (st + rng.integers(0, 20, size=b.n_txn)).astype(np.uint64)
    hk = rng.integers(0, 300, size=300).astype(np.uint64)
    ht = rng.integers(1, 70, size=300).astype(np.uint64)
    both(b, hist_keys=hk, hist_tn=ht, tnc=70)


def test_round_status_fixed_point_equals_serial():
    """The round-based fixed point the GPU runs (per-key min undecided /
    committed writer) converges to the serial decisions."""
    rng = np.random.default_rng(7)
    for b in (d.gen_ycsb(n_txn=4000, zipf_theta=0.9, table_size=1 << 16),
              random_batch(rng, 1500, 16, 300), chain_batch(40)):
        state = np.zeros(b.n_txn, np.uint8)
        rounds = 0
        while (state == 0).any():
            s = orc.occ_round_status(b, state)
            und = state == 0
            state[und & ((s & 2) != 0)] = 2
            state[und & (s == 0)] = 1
            rounds += 1
            assert rounds <= b.n_txn + 1
        rc, _, _ = orc.occ(b)
        assert np.array_equal(np.where(state == 1, 0, 2), rc)


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_rounds_mt_equals_serial(threads):
    """ROUNDS-MT (the multi-core CPU baseline of SURVEY.md §8(d)) decides
    exactly like the serial scan, tn numbering included."""
    rng = np.random.default_rng(8)
    for b in (d.gen_ycsb(n_txn=20000, zipf_theta=0.9, table_size=1 << 16),
              d.gen_ycsb(n_txn=5000, zipf_theta=0.99),
              random_batch(rng, 1500, 16, 300, types=(RD, WR, XP, SCAN)), chain_batch(40),
              make_batch([])):
        rc, tn, tnc = orc.occ(b, tnc=5)
        rc2, tn2, tnc2, rounds = orc.occ_rounds_mt(b, threads, tnc=5)
        assert np.array_equal(rc, rc2) and np.array_equal(tn, tn2) and tnc == tnc2
        assert rounds <= b.n_txn + 1


@pytest.mark.parametrize("threads", [1, 4, 8])
def test_sweep_mt_equals_serial(threads):
    """SWEEP-MT (the multi-core CPU baseline: serial prefixes + parallel
    filters) decides exactly like the serial scan, tn numbering included."""
    rng = np.random.default_rng(12)
    for b in (d.gen_ycsb(n_txn=60000, zipf_theta=0.9, table_size=1 << 16),
              d.gen_ycsb(n_txn=30000, zipf_theta=0.0),
              d.gen_ycsb(n_txn=20000, zipf_theta=0.99),
              random_batch(rng, 3000, 16, 300, types=(RD, WR, XP, SCAN)), chain_batch(3000),
              make_batch([]), make_batch([[], [(1, WR)], [(1, RD)]])):
        rc, tn, tnc = orc.occ(b, tnc=7)
        rc2, tn2, tnc2, levels = orc.occ_sweep_mt(b, threads, tnc=7)
        assert np.array_equal(rc, rc2) and np.array_equal(tn, tn2) and tnc == tnc2
        assert levels >= (1 if b.n_txn else 0)


# ---------------------------------------------------------------- Calvin
def calvin_both(b):
    g1, r1, w1 = orc.calvin(b, literal=True)
    g2, r2, w2 = orc.calvin(b, literal=False)
    assert np.array_equal(g1, g2) and np.array_equal(r1, r2) and np.array_equal(w1, w2)
    return g1, r1, w1


def test_kat_calvin_fifo_no_barging():
    # S1 SH(k), X2 EX(k), S3 SH(k): S3 must wait behind X2 although it is
    # compatible with the SH owner (row_lock.cpp:78-81)
    g, rc, w = calvin_both(make_batch([[(1, RD)], [(1, WR)], [(1, RD)], [(1, RD)], [(1, WR)]]))
    assert list(g) == [0, 1, 2, 2, 3]
    assert list(rc) == [0, 3, 3, 3, 3]
    assert list(w) == [0, 1, 2, 2, 3]


def test_kat_calvin_sh_sharing_and_waves():
    # T0 EX a; T1 SH a, SH b; T2 SH b; T3 EX b -> waits for T1 and T2
    g, rc, w = calvin_both(make_batch([[(10, WR)], [(10, RD), (11, RD)], [(11, RD)], [(11, WR)]]))
    assert list(g) == [0, 1, 0, 0, 1]
    assert list(rc) == [0, 3, 0, 3]
    assert list(w) == [0, 1, 0, 2]


def test_kat_calvin_dedup_and_types():
    # duplicate row in one txn: first access type wins (txn.cpp:778-782);
    # SCAN -> SH, XP -> EX (row.cpp:191)
    g, rc, w = calvin_both(make_batch([[(5, RD), (5, WR)], [(5, SCAN)], [(6, XP)], [(6, SCAN)]]))
    assert g[1] == d.GROUP_NONE
    assert list(g[[0, 2, 3, 4]]) == [0, 0, 0, 1]
    assert list(rc) == [0, 0, 0, 3]


def test_kat_calvin_order():
    # sequence order (epoch, origin, FIFO) from `order`, not index order
    b = make_batch([[(1, WR)], [(1, WR)], [(1, RD)]], order=[(1 << 32) | 5, 0, (1 << 32) | 1])
    g, rc, w = calvin_both(b)
    assert list(g) == [2, 0, 1]
    assert list(rc) == [3, 0, 3]


def test_calvin_replay_equals_formula_random():
    rng = np.random.default_rng(8)
    for n_keys in (8, 200, 100000):
        calvin_both(random_batch(rng, 800, 12, n_keys, types=(RD, WR, XP, SCAN), unique=False))
    b = d.gen_ycsb(n_txn=3000, zipf_theta=0.9, req_per_query=8, table_size=2000)
    b.order = np.random.default_rng(9).permutation(b.n_txn).astype(np.uint64)
    calvin_both(b)


def test_calvin_held_prefix_kat():
    """Held rows (row_lock.cpp:219-372: releases are asynchronous): the literal
    replay of (held requests, then the epoch) and the per-row formula agree,
    and give the hand-worked groups."""
    A, B, C = 10, 20, 30
    b = make_batch([[(A, RD)], [(B, RD)], [(C, RD)], [(B, WR)]])
    hk = np.array([A, B, C, C], np.uint64)
    ha = np.array([WR, RD, RD, WR], np.uint8)
    g, rc = orc.calvin_held(b, hk, ha, literal=True)
    g2, rc2 = orc.calvin_held(b, hk, ha, literal=False)
    assert list(g) == [1, 0, 2, 1] and list(rc) == [3, 0, 3, 3]
    assert np.array_equal(g, g2) and np.array_equal(rc, rc2)
