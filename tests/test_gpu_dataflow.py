"""GPU parity of the dataflow solver (occ_dataflow.hip, DESIGN.md §3, solver
4): level 0 of the sweep, then the survivors -- write and read-only txns --
decided without levels or rounds: each access waits until every writer of its
key with a smaller txn id is decided, a committed one kills it.  Decisions
must be bit-exact against the oracle's serial replay (occ.cpp:116-294),
including keys with many writers (several group words), long dependency
chains, the hand-off of a list too large for the solver, the fallback to the
sweep levels when the solver hits its time limit, and the key table staying
clean across epochs and after a rejected batch."""
import os

import numpy as np
import pytest

import _oracle as orc
import deneva_amd as d
from deneva_amd import RD, WR, XP, SCAN
from deneva_amd._abi import DccError, OPT_SOLVER
from helpers import chain_batch, make_batch, random_batch

pytestmark = pytest.mark.gpu


@pytest.fixture
def dfe(engine):
    engine.set_option(OPT_SOLVER, 4)
    yield engine
    engine.set_option(OPT_SOLVER, 0)


def run(engine, b, hist=None, tnc=0):
    engine.tnc = tnc
    rc, tn, st = engine.occ_validate_epoch(b, want_tn=True)
    hk, ht = (None, None) if hist is None else hist
    erc, etn, etnc = orc.occ(b, hist_keys=hk, hist_tn=ht, tnc=tnc)
    rc = np.asarray(rc)
    bad = np.nonzero(rc != erc)[0]
    assert bad.size == 0, f"rc mismatch at {bad[:10]} (gpu {rc[bad[:10]]} oracle {erc[bad[:10]]})"
    assert np.array_equal(np.asarray(tn).astype(np.uint64), etn), "commit tn mismatch"
    assert engine.tnc == etnc
    assert st["n_commit"] == int((erc == 0).sum())
    return rc, st


@pytest.mark.parametrize("theta", [0.0, 0.6, 0.9, 0.99])
@pytest.mark.parametrize("n", [1, 63, 64, 1025, 3000, 65536])
def test_ycsb(dfe, theta, n):
    run(dfe, d.gen_ycsb(n_txn=n, zipf_theta=theta))


@pytest.mark.parametrize("theta", [0.9, 0.99])
def test_ycsb_1m(dfe, theta):
    b = d.gen_ycsb(n_txn=1 << 20, zipf_theta=theta)
    _, st = run(dfe, b)
    # level 0, then the dataflow solver over its survivors (no fallback)
    assert st["peel_prefix"] > 0 and st["rounds"] == 2 and st["fallback"] == 0, st


def test_chain(dfe):
    # txn i writes key i and reads key i - 1: a dependency chain through the
    # whole list (every decision waits for the one before it)
    rc, st = run(dfe, chain_batch(3000))
    assert st["fallback"] == 0
    assert list(rc[:6]) == [0, 2, 0, 2, 0, 2]


def hot_key_batch(pairs, commit_at=None, readers=64, lead=1100):
    """`lead` independent txns (level 0's serial range), then `pairs` pairs:
    txn 2j writes a fresh key B_j (commits), txn 2j+1 reads B_j (so it aborts)
    and writes the hot key H: H gets `pairs` writers in the survivor list, all
    aborting, spread over many 32-writer groups.  commit_at: one txn writing H
    alone after that many pairs (it commits: every earlier writer of H
    aborted).  Then `readers` txns reading H."""
    H = 1 << 40
    txns = [[(10 + i, WR)] for i in range(lead)]
    for j in range(pairs):
        if commit_at is not None and j == commit_at:
            txns.append([(H, WR)])
        b = 1 << 30 | j
        txns.append([(b, WR)])
        txns.append([(b, RD), (H, WR)])
    txns += [[(H, RD), (5 << 32 | r, WR)] for r in range(readers)]
    return make_batch(txns)


@pytest.mark.parametrize("pairs", [31, 33, 200, 2000])
def test_hot_key_groups(dfe, pairs):
    rc, st = run(dfe, hot_key_batch(pairs))
    # every hot-key writer aborts, the readers after them all commit
    assert (rc[-64:] == 0).all() and st["fallback"] == 0


@pytest.mark.parametrize("at", [0, 40, 1500])
def test_hot_key_commit_mid_groups(dfe, at):
    rc, _ = run(dfe, hot_key_batch(2000, commit_at=at))
    assert (rc[-64:] != 0).all()  # a committed writer of H precedes every reader


def test_low_contention_handoff(dfe):
    # > 1/4 of the epoch survives level 0: the list goes to the round solver
    b = d.gen_ycsb(n_txn=300000, zipf_theta=0.0, table_size=1 << 24)
    _, st = run(dfe, b)
    assert st["n_survivors"] > 65536 and st["fallback"] >= 1


def test_types_ragged_empty(dfe):
    rng = np.random.default_rng(11)
    run(dfe, random_batch(rng, 9000, 64, 4000, types=(RD, WR, XP, SCAN)))
    run(dfe, random_batch(rng, 9000, 5, 300, p_write=0.5))
    run(dfe, random_batch(rng, 6000, 16, 60, types=(RD, WR, XP, SCAN), unique=False))
    run(dfe, make_batch([[] for _ in range(130)]))
    run(dfe, make_batch([[], [(1, WR)], [], [(1, RD)], []] * 500))


def test_hot_single_key_and_max_len(dfe):
    run(dfe, make_batch([[(7, WR if i % 3 == 0 else RD)] for i in range(10000)]))
    rng = np.random.default_rng(3)
    txns = [[(int(k), WR if rng.random() < 0.4 else RD)
             for k in rng.choice(5000, size=64, replace=False)] for _ in range(3000)]
    run(dfe, make_batch(txns))
    # 64-access txns whose chunks overhang their 64-access window
    txns = [[(int(k), WR if rng.random() < 0.3 else RD)
             for k in rng.choice(20000, size=int(L), replace=False)]
            for L in rng.integers(1, 65, size=5000)]
    run(dfe, make_batch(txns))


def test_duplicate_writes_in_txn(dfe):
    # a txn writing (and reading) the same key twice holds two writer entries
    rng = np.random.default_rng(9)
    txns = []
    for i in range(6000):
        k = int(rng.integers(0, 400))
        txns.append([(k, WR), (int(rng.integers(0, 400)), RD), (k, WR), (k, RD)])
    run(dfe, make_batch(txns))


def test_tpcc(dfe):
    run(dfe, d.gen_tpcc(n_txn=65536, num_wh=16))
    run(dfe, d.gen_tpcc(n_txn=262144, num_wh=128))


def test_history_prekill(dfe):
    rng = np.random.default_rng(5)
    b = random_batch(rng, 4000, 12, 600, p_write=0.4)
    n = b.n_txn
    b.start_tn = rng.integers(0, 20, size=n).astype(np.uint64)
    b.finish_tn = (b.start_tn + rng.integers(0, 20, size=n)).astype(np.uint64)
    hk = rng.integers(0, 600, size=300).astype(np.uint64)
    ht = rng.integers(1, 40, size=300).astype(np.uint64)
    dfe.history_clear()
    dfe.history_append(hk, ht)
    try:
        run(dfe, b, hist=(hk, ht), tnc=40)
    finally:
        dfe.history_clear()


def test_table_clean_across_epochs(dfe):
    # different key sets back to back, then the first again: a slot left
    # behind by one epoch would change a later epoch's decisions
    a = d.gen_ycsb(n_txn=200000, zipf_theta=0.9, seed=0xC0FFEE)
    b = d.gen_ycsb(n_txn=200000, zipf_theta=0.9, seed=0xBEEF, table_size=1 << 20)
    ra, _ = run(dfe, a)
    run(dfe, b)
    ra2, _ = run(dfe, a)
    assert np.array_equal(ra, ra2)


def test_rejected_batch_then_clean(dfe):
    # a reserved key fails the epoch after the solver touched the table; the
    # next epoch starts from a clean table again
    b = d.gen_ycsb(n_txn=50000, zipf_theta=0.9)
    keys = np.asarray(b.keys).copy()
    keys[len(keys) // 2] = 0xFFFFFFFFFFFFFFFF
    bad = d.EpochBatch(b.offsets, keys, b.acctype)
    with pytest.raises(DccError):
        dfe.occ_validate_epoch(bad)
    run(dfe, b)


def test_time_limit_falls_back(dfe):
    # the solver gives up at once (a 0 us limit): the epoch is decided again by
    # the sweep's levels, and the next epoch (normal limit) cleans the table
    b = d.gen_ycsb(n_txn=200000, zipf_theta=0.9, seed=0xFA11)
    os.environ["DCC_DF_LIMIT_US"] = "0"
    try:
        _, st = run(dfe, b)
        assert st["fallback"] >= 1
    finally:
        os.environ["DCC_DF_LIMIT_US"] = "500000"
    _, st = run(dfe, b)
    assert st["fallback"] == 0


def test_device_batch_repeat(dfe):
    # the captured epoch replayed (graph), device pointers
    import torch
    b = d.gen_ycsb(n_txn=300000, zipf_theta=0.9, seed=0xD00D)
    db = b.to_torch("cuda:0")
    erc, _, _ = orc.occ(b)
    for _ in range(4):
        rc, _, _ = dfe.occ_validate_epoch(db)
        torch.cuda.synchronize()
        assert np.array_equal(rc.cpu().numpy(), erc)
