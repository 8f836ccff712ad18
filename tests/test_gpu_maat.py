"""GPU parity of MaaT epoch validation (dcc_maat_validate_epoch, maat.hip)
against the oracle (oracle/maat_ref.c): bit-exact RC, commit timestamps and
row timestamps after the epoch."""
import numpy as np
import pytest

import _oracle as orc
import deneva_amd as d
from deneva_amd import RD, SCAN, WR, XP
from helpers import make_batch, random_batch

pytestmark = pytest.mark.gpu


def run(engine, b, rows=None, rw_all=False, literal=False, dev=False):
    engine.maat_rows_clear()
    rk, lr, lw = rows if rows is not None else (None, None, None)
    if rows is not None:
        engine.maat_rows_set(rk, lr, lw)
    bb = b.to_torch("cuda:0") if dev else b
    rc, cts, st = engine.maat_validate_epoch(bb, read_and_prewrite=rw_all)
    if dev:
        rc, cts = rc.cpu().numpy(), cts.cpu().numpy().view(np.uint64)
    erc, ects, (ek, elr, elw) = orc.maat(b, rk, lr, lw, rw_all=rw_all, literal=literal)
    rc = np.asarray(rc)
    bad = np.nonzero(rc != erc)[0]
    assert bad.size == 0, f"rc mismatch at {bad[:10]} (gpu {rc[bad[:10]]} oracle {erc[bad[:10]]})"
    assert np.array_equal(np.asarray(cts, np.uint64), ects), "commit ts mismatch"
    glr, glw = engine.maat_rows_get(ek)
    assert np.array_equal(glr, elr) and np.array_equal(glw, elw), "row timestamps mismatch"
    assert st["n_commit"] == int((erc == 0).sum())
    return rc, st


def test_kat(engine):
    run(engine, make_batch([[(5, RD)], [(5, WR)]]))
    run(engine, make_batch([[(5, WR)], [(5, RD)]]))
    run(engine, make_batch([[(5, RD)], [(6, WR)]]),
        rows=(np.array([5, 6], np.uint64), np.array([0, 3], np.uint64), np.array([7, 0], np.uint64)))


def test_empty_and_zero_length(engine):
    run(engine, make_batch([]))
    run(engine, make_batch([[], [(1, WR)], [], [(1, RD)]]))


@pytest.mark.parametrize("rw_all", [False, True])
def test_random(engine, rw_all):
    rng = np.random.default_rng(7 + rw_all)
    for it in range(12):
        nk = int(rng.integers(1, 2000))
        types = (RD, WR) if it % 3 else (RD, WR, XP, SCAN)
        b = random_batch(rng, int(rng.integers(1, 5000)), int(rng.integers(1, 64)), nk,
                         p_write=float(rng.random()), types=types, unique=bool(it % 2))
        rk = np.arange(nk, dtype=np.uint64)
        run(engine, b, rows=(rk, rng.integers(0, 100, size=nk).astype(np.uint64),
                             rng.integers(0, 100, size=nk).astype(np.uint64)), rw_all=rw_all,
            literal=it < 4)


@pytest.mark.parametrize("theta", [0.0, 0.6, 0.9, 0.99])
def test_ycsb_c2(engine, theta):
    # BASELINE config C2 shape: 65,536 txns x 16 keys
    run(engine, d.gen_ycsb(n_txn=65536, zipf_theta=theta))


def test_ycsb_device_pointers(engine):
    run(engine, d.gen_ycsb(n_txn=65536, zipf_theta=0.9), dev=True)


def test_tpcc(engine):
    run(engine, d.gen_tpcc(n_txn=16384, num_wh=16), rw_all=True)


def test_epochs_carry_row_timestamps(engine):
    """Row timestamps persist in the context across epochs."""
    engine.maat_rows_clear()
    rk = np.zeros(0, np.uint64)
    lr = np.zeros(0, np.uint64)
    lw = np.zeros(0, np.uint64)
    for e in range(4):
        b = d.gen_ycsb(n_txn=8192, zipf_theta=0.8, table_size=1 << 14, seed=50 + e)
        rc, cts, _ = engine.maat_validate_epoch(b)
        erc, ects, (ek, elr, elw) = orc.maat(b, rk, lr, lw)
        assert np.array_equal(np.asarray(rc), erc) and np.array_equal(np.asarray(cts), ects)
        # the rows known so far, merged with this epoch's
        allk = np.union1d(rk, ek)
        nlr = np.zeros(allk.size, np.uint64)
        nlw = np.zeros(allk.size, np.uint64)
        if rk.size:
            p = np.searchsorted(allk, rk)
            nlr[p], nlw[p] = lr, lw
        p = np.searchsorted(allk, ek)
        nlr[p], nlw[p] = elr, elw
        rk, lr, lw = allk, nlr, nlw
        glr, glw = engine.maat_rows_get(rk)
        assert np.array_equal(glr, lr) and np.array_equal(glw, lw)
    assert engine.maat_rows_size == rk.size
    engine.maat_rows_clear()


def test_row_table_growth(engine):
    """Many distinct rows: the table rehashes, timestamps survive."""
    engine.maat_rows_clear()
    rng = np.random.default_rng(9)
    k = rng.choice(1 << 40, size=200000, replace=False).astype(np.uint64)
    lr = rng.integers(0, 1000, size=k.size).astype(np.uint64)
    lw = rng.integers(0, 1000, size=k.size).astype(np.uint64)
    engine.maat_rows_set(k[:1000], lr[:1000], lw[:1000])
    engine.maat_rows_set(k[1000:], lr[1000:], lw[1000:])
    glr, glw = engine.maat_rows_get(k)
    assert np.array_equal(glr, lr) and np.array_equal(glw, lw)
    engine.maat_rows_clear()


def test_rejected_batch_leaves_rows_unchanged(engine):
    """A batch the engine rejects (reserved key, malformed offsets) changes
    neither the row table's rows nor its timestamps."""
    from deneva_amd._abi import DccError
    engine.maat_rows_clear()
    b = d.gen_ycsb(n_txn=4096, zipf_theta=0.9, table_size=1 << 12, seed=77)
    engine.maat_validate_epoch(b)
    rk = np.unique(np.asarray(b.keys))
    lr0, lw0 = engine.maat_rows_get(rk)
    size0 = engine.maat_rows_size
    c = d.gen_ycsb(n_txn=4096, zipf_theta=0.9, table_size=1 << 16, seed=78)
    keys = np.asarray(c.keys).copy()
    keys[-1] = 0xFFFFFFFFFFFFFFFF
    with pytest.raises(DccError):
        engine.maat_validate_epoch(d.EpochBatch(c.offsets, keys, c.acctype))
    off = np.asarray(c.offsets).copy()
    off[5], off[6] = off[6], off[5]
    with pytest.raises(DccError):
        engine.maat_validate_epoch(d.EpochBatch(off, c.keys, c.acctype))
    assert engine.maat_rows_size == size0
    lr1, lw1 = engine.maat_rows_get(rk)
    assert np.array_equal(lr0, lr1) and np.array_equal(lw0, lw1)
    engine.maat_rows_clear()


@pytest.mark.parametrize("theta,n", [(0.9, 1 << 20), (0.99, 1 << 18), (0.6, 1 << 18), (0.0, 1 << 16)])
def test_prefix_level_full_size(engine, theta, n):
    # epochs of > 4 x 1,024 txns take the prefix level (maat.hip: the first
    # 1,024 decided alone, later txns filtered against their commits, rounds
    # on the survivors); with pre-seeded row timestamps the base bounds join in
    b = d.gen_ycsb(n_txn=n, zipf_theta=theta, seed=0x3A7 + n)
    run(engine, b)
    rng = np.random.default_rng(n)
    rk = np.unique(b.keys[rng.integers(0, b.nnz, size=2000)]).astype(np.uint64)
    lr = rng.integers(0, 50, size=rk.size).astype(np.uint64)
    lw = rng.integers(0, 50, size=rk.size).astype(np.uint64)
    run(engine, b, rows=(rk, lr, lw))


def test_row_table_full_runs_again():
    """A fresh context sizes its row table for a quarter of the epoch's
    accesses; an epoch of all-distinct rows fills it (a walk past MT_WALK),
    and the epoch runs again on a table sized for every access: decisions,
    commit timestamps and row timestamps as the oracle's, and nothing the
    first attempt did leaks into the row timestamps."""
    eng = d.Engine(0)
    try:
        rng = np.random.default_rng(0xF011)
        for e in range(2):
            n, k = 16384, 16
            keys = rng.choice(1 << 40, size=n * k, replace=False).astype(np.uint64)
            at = np.where(rng.random(n * k) < 0.5, WR, RD).astype(np.uint8)
            # one shared row so the epoch has aborts to get right
            keys[k::k] = keys[0]
            run(eng, d.EpochBatch(np.arange(0, n * k + 1, k, dtype=np.uint32), keys, at))
    finally:
        eng.close()
