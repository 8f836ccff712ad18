"""MaaT oracle (oracle/maat_ref.c): the literal replay of Maat::validate /
find_bound / Row_maat (maat.cpp:29-191, row_maat.cpp:38-314) in the epoch
model and the running-bounds formula agree, and hand-worked cases traced to
those lines hold."""
import numpy as np
import pytest

import _oracle as orc
import deneva_amd as d
from deneva_amd import RD, SCAN, WR, XP
from helpers import make_batch, random_batch


def both(b, rows=None, rw_all=False):
    rk, lr, lw = rows if rows is not None else (None, None, None)
    a = orc.maat(b, rk, lr, lw, rw_all=rw_all, literal=True)
    f = orc.maat(b, rk, lr, lw, rw_all=rw_all, literal=False)
    assert np.array_equal(a[0], f[0]) and np.array_equal(a[1], f[1])
    for x, y in zip(a[2], f[2]):
        assert np.array_equal(x, y)
    return a


def test_kat_reader_then_writer():
    # T0 reads k (commits at 1: lower 0 <= gwts 0 -> 1, maat.cpp:46-49); its
    # commit pushes the later writer T1 after it: lower(T1) = 2
    # (row_maat.cpp:254-266); T1 commits at 2; the row's last read / write
    # timestamps become 1 / 2 (row_maat.cpp:249-251, 276-278).
    b = make_batch([[(5, RD)], [(5, WR)]])
    rc, cts, (rk, lr, lw) = both(b)
    assert list(rc) == [0, 0] and list(cts) == [1, 2]
    assert list(lr) == [1] and list(lw) == [2]


def test_kat_writer_then_reader():
    # T0 writes k at 1; its commit caps the later reader T1 at lower(T0) - 1 =
    # 0 (row_maat.cpp:295-305) while T1's lower is >= 1: T1 aborts
    # (maat.cpp:112-115).
    b = make_batch([[(5, WR)], [(5, RD)]])
    rc, cts, _ = both(b)
    assert list(rc) == [0, 2] and list(cts) == [1, 0]


def test_kat_row_timestamps():
    # a row last written at 7 (an earlier epoch): the reader's lower becomes 8
    # (greatest_write_timestamp, row_maat.cpp:115-117; maat.cpp:46-49)
    b = make_batch([[(5, RD)], [(6, WR)]])
    rc, cts, (rk, lr, lw) = both(b, rows=(np.array([5, 6], np.uint64), np.array([0, 3], np.uint64),
                                          np.array([7, 0], np.uint64)))
    assert list(rc) == [0, 0] and list(cts) == [8, 4]
    assert list(lr) == [8, 3] and list(lw) == [7, 4]


def test_kat_xp_scan_untracked():
    # XP / SCAN accesses do nothing in Row_maat::access (row_maat.cpp:42-46)
    b = make_batch([[(5, WR)], [(5, XP)], [(5, SCAN)]])
    rc, cts, _ = both(b)
    assert list(rc) == [0, 0, 0]


@pytest.mark.parametrize("rw_all", [False, True])
def test_random_agree(rw_all):
    rng = np.random.default_rng(3 + rw_all)
    for it in range(40):
        n = int(rng.integers(1, 400))
        nk = int(rng.integers(1, 200))
        types = (RD, WR) if it % 3 else (RD, WR, XP, SCAN)
        b = random_batch(rng, n, int(rng.integers(1, 16)), nk, p_write=float(rng.random()),
                         types=types, unique=bool(it % 2))
        rk = np.arange(nk, dtype=np.uint64)
        both(b, rows=(rk, rng.integers(0, 40, size=nk).astype(np.uint64),
                      rng.integers(0, 40, size=nk).astype(np.uint64)), rw_all=rw_all)


@pytest.mark.parametrize("theta", [0.6, 0.9, 0.99])
def test_ycsb_agree(theta):
    both(d.gen_ycsb(n_txn=3000, zipf_theta=theta, table_size=1 << 14))


def test_tpcc_agree():
    both(d.gen_tpcc(n_txn=2000, num_wh=4), rw_all=True)


def _prefix_level_model(b, P):
    """maat.hip's prefix level restated on the CPU (empty row timestamps):
    the first P txns decided by the formula alone, every later txn aborted
    when its bounds from those commits are already empty, the survivors then
    decided in index order against every commit before them."""
    n = b.n_txn
    off = np.asarray(b.offsets, np.int64)
    keys = np.asarray(b.keys)
    at = np.asarray(b.acctype)
    big = 1 << 62

    def bounds(i, maxr, minw):
        L, U = 1, big
        for x in range(off[i], off[i + 1]):
            k, t = int(keys[x]), int(at[x])
            rd, wr = t == RD, t == WR
            if not (rd or wr):
                continue
            if wr and k in maxr:
                L = max(L, maxr[k] + 1)
            if k in minw:
                U = min(U, minw[k] - 1)
        return L, U

    def commit(i, c, maxr, minw):
        for x in range(off[i], off[i + 1]):
            k, t = int(keys[x]), int(at[x])
            if t == WR:
                minw[k] = min(minw.get(k, big), c)
            elif t == RD:
                maxr[k] = max(maxr.get(k, 0), c)

    rc = np.full(n, 2, np.uint8)  # abort unless committed
    cts = np.zeros(n, np.uint64)
    maxr, minw = {}, {}
    for i in range(min(P, n)):
        L, U = bounds(i, maxr, minw)
        if L < U:
            commit(i, L, maxr, minw)
            rc[i], cts[i] = 0, L
    pre_r, pre_w = dict(maxr), dict(minw)
    surv = [i for i in range(P, n) if (lambda lu: lu[0] < lu[1])(bounds(i, pre_r, pre_w))]
    for i in surv:  # index order: every earlier commit is known
        L, U = bounds(i, maxr, minw)
        if L < U:
            commit(i, L, maxr, minw)
            rc[i], cts[i] = 0, L
    return rc, cts, len(surv)


@pytest.mark.parametrize("theta,P", [(0.9, 64), (0.99, 128), (0.6, 256)])
def test_prefix_level_is_exact(theta, P):
    # the argument behind maat.hip's prefix filter: L only grows and U only
    # shrinks as earlier txns commit, so a txn whose bounds the prefix's
    # commits alone empty is aborted by the full replay too
    b = d.gen_ycsb(n_txn=3000, zipf_theta=theta, seed=0x99 + P)
    rc, cts, nsurv = _prefix_level_model(b, P)
    erc, ects, _ = orc.maat(b)
    assert np.array_equal(rc, erc)
    assert np.array_equal(cts[erc == 0], np.asarray(ects, np.uint64)[erc == 0])
    assert nsurv < b.n_txn - P  # the filter aborts something
