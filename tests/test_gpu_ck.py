"""GPU parity of the commit/kill round solver (occ_ck.hip, DESIGN.md §3b,
solver 4): the sweep's first levels, then rounds over their survivors in
which a txn commits when no earlier undecided or committed txn writes one of
its keys and aborts when an earlier committed txn does (this round's commits
included).  Decisions must be bit-exact
against the oracle's serial replay (occ.cpp:116-294), including the rounds
past the captured ones, the hand-off of a list too large for the solver, and
the key table staying clean across epochs and after a rejected batch."""
import numpy as np
import pytest

import _oracle as orc
import deneva_amd as d
from deneva_amd import RD, WR, XP, SCAN
from deneva_amd._abi import DccError, OPT_CK_LEVEL, OPT_SOLVER
from helpers import chain_batch, make_batch, random_batch

pytestmark = pytest.mark.gpu


@pytest.fixture(params=[1, 2])
def ck(engine, request):
    # the rounds after level 0 (ck_level 1) and after levels 0-1 (the default)
    engine.set_option(OPT_SOLVER, 4)
    engine.set_option(OPT_CK_LEVEL, request.param)
    engine.ck_level = request.param
    yield engine
    engine.set_option(OPT_SOLVER, 0)
    engine.set_option(OPT_CK_LEVEL, 2)


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
def test_ycsb(ck, theta, n):
    run(ck, d.gen_ycsb(n_txn=n, zipf_theta=theta))


@pytest.mark.parametrize("theta", [0.9, 0.99])
def test_ycsb_1m(ck, theta):
    b = d.gen_ycsb(n_txn=1 << 20, zipf_theta=theta)
    _, st = run(ck, b)
    # level 0 plus a handful of commit/kill rounds (8 at theta 0.9)
    assert st["peel_prefix"] > 0 and 1 < st["rounds"] <= 20, st["rounds"]


def test_chain_past_captured_rounds(ck):
    # two decisions per round: ~1,000 rounds, far past the captured ones
    # (the list after level 0 holds 1,976 chain txns; level 1's serial pass
    # decides 2,048, so only the level-0 variant reaches the rounds)
    rc, st = run(ck, chain_batch(3000 if ck.ck_level == 1 else 5000))
    assert st["rounds"] > 400
    assert list(rc[:6]) == [0, 2, 0, 2, 0, 2]


def test_low_contention_handoff(ck):
    # > 1/4 of the epoch survives level 0: the list goes to the round solver
    b = d.gen_ycsb(n_txn=300000, zipf_theta=0.0, table_size=1 << 24)
    _, st = run(ck, b)
    assert st["n_survivors"] > 65536 and st["fallback"] >= 1


def test_types_ragged_empty(ck):
    rng = np.random.default_rng(11)
    run(ck, random_batch(rng, 9000, 64, 4000, types=(RD, WR, XP, SCAN)))
    run(ck, random_batch(rng, 9000, 5, 300, p_write=0.5))
    run(ck, random_batch(rng, 6000, 16, 60, types=(RD, WR, XP, SCAN), unique=False))
    run(ck, make_batch([[] for _ in range(130)]))
    run(ck, make_batch([[], [(1, WR)], [], [(1, RD)], []] * 500))


def test_hot_single_key_and_max_len(ck):
    run(ck, make_batch([[(7, WR if i % 3 == 0 else RD)] for i in range(10000)]))
    rng = np.random.default_rng(3)
    txns = [[(int(k), WR if rng.random() < 0.4 else RD)
             for k in rng.choice(5000, size=64, replace=False)] for _ in range(3000)]
    run(ck, make_batch(txns))


def test_tpcc(ck):
    run(ck, d.gen_tpcc(n_txn=65536, num_wh=16))
    run(ck, d.gen_tpcc(n_txn=262144, num_wh=128))


def test_history_prekill(ck):
    rng = np.random.default_rng(5)
    b = random_batch(rng, 4000, 12, 600, p_write=0.4)
    n = b.n_txn
    b.start_tn = rng.integers(0, 20, size=n).astype(np.uint64)
    b.finish_tn = (b.start_tn + rng.integers(0, 20, size=n)).astype(np.uint64)
    hk = rng.integers(0, 600, size=300).astype(np.uint64)
    ht = rng.integers(1, 40, size=300).astype(np.uint64)
    ck.history_clear()
    ck.history_append(hk, ht)
    try:
        run(ck, b, hist=(hk, ht), tnc=40)
    finally:
        ck.history_clear()


def test_table_clean_across_epochs(ck):
    # different key sets back to back, then the first again: a slot left
    # behind by one epoch would change a later epoch's decisions
    a = d.gen_ycsb(n_txn=200000, zipf_theta=0.9, seed=0xC0FFEE)
    b = d.gen_ycsb(n_txn=200000, zipf_theta=0.9, seed=0xBEEF, table_size=1 << 20)
    ra, _ = run(ck, a)
    run(ck, b)
    ra2, _ = run(ck, a)
    assert np.array_equal(ra, ra2)


def test_rejected_batch_then_clean(ck):
    # a reserved key fails the epoch after the solver touched the table; the
    # next epoch starts from a clean table again
    b = d.gen_ycsb(n_txn=50000, zipf_theta=0.9)
    keys = np.asarray(b.keys).copy()
    keys[len(keys) // 2] = 0xFFFFFFFFFFFFFFFF
    bad = d.EpochBatch(b.offsets, keys, b.acctype)
    with pytest.raises(DccError):
        ck.occ_validate_epoch(bad)
    run(ck, b)


def test_device_batch_repeat(ck):
    # the captured epoch replayed (graph), device pointers
    import torch
    b = d.gen_ycsb(n_txn=300000, zipf_theta=0.9, seed=0xD00D)
    db = b.to_torch("cuda:0")
    erc, _, _ = orc.occ(b)
    for _ in range(4):
        rc, _, _ = ck.occ_validate_epoch(db)
        torch.cuda.synchronize()
        assert np.array_equal(rc.cpu().numpy(), erc)
