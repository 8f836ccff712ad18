"""GPU parity of the OCC sweep solver (occ_sweep.hip), the
default unsharded solver: per level, 64-txn tile records, one serial pass in
one CU with the committed write keys in LDS, and a filter + compaction pass
over the rest of the list.  The cases drive every path — level-0 access-budget
stops, many levels and host continuations (one level per synchronisation),
the hand-off of a low-contention list to the round solver, history-aborted
txns inside tiles, empty and maximum-length txns, tiles with 4096 accesses —
and the decisions must be bit-exact against the oracle's serial replay."""
import numpy as np
import pytest

import _oracle as orc
import deneva_amd as d
from deneva_amd import RD, WR, XP, SCAN
from deneva_amd._abi import OPT_SOLVER, OPT_SWEEP_LEVELS
from helpers import chain_batch, make_batch, random_batch

pytestmark = pytest.mark.gpu


@pytest.fixture
def sw(engine):
    engine.set_option(OPT_SOLVER, 3)
    yield engine
    engine.set_option(OPT_SOLVER, 0)
    engine.set_option(OPT_SWEEP_LEVELS, 0)


def run(engine, b, levels=4, hist=None, tnc=0):
    engine.set_option(OPT_SWEEP_LEVELS, levels)
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
    assert st["n_abort"] == int((erc == 2).sum())
    return rc, st


@pytest.mark.parametrize("theta", [0.0, 0.6, 0.9, 0.99])
@pytest.mark.parametrize("n", [1, 63, 64, 65, 1025, 20000, 65536])
def test_ycsb(sw, theta, n):
    run(sw, d.gen_ycsb(n_txn=n, zipf_theta=theta))


@pytest.mark.parametrize("theta", [0.9, 0.99])
def test_ycsb_1m(sw, theta):
    b = d.gen_ycsb(n_txn=1 << 20, zipf_theta=theta)
    _, st = run(sw, b)
    assert st["peel_prefix"] > 0 and st["n_survivors"] < b.n_txn // 4


@pytest.mark.parametrize("levels", [1, 2, 7])
def test_levels_per_sync(sw, levels):
    # the same decisions whatever the number of levels between host syncs
    b = d.gen_ycsb(n_txn=200000, zipf_theta=0.9, seed=0x5EED)
    run(sw, b, levels=levels)


def test_low_contention_handoff(sw):
    # uniform keys on a large table: the committed keys kill little, the
    # survivors are handed to the round solver after level 0
    b = d.gen_ycsb(n_txn=300000, zipf_theta=0.0, table_size=1 << 24)
    _, st = run(sw, b)
    assert st["n_survivors"] > 65536


def test_level0_budget_stop(sw):
    # 64 fresh keys per txn: the level-0 key table holds 16,384 accesses, so
    # the serial pass stops after 256 txns, long before p_max (1,024)
    n = 5000
    txns = [[(i * 64 + q, WR if q % 2 else RD) for q in range(64)] for i in range(n)]
    _, st = run(sw, make_batch(txns))
    assert st["peel_prefix"] == 256


def test_max_len_tiles(sw):
    # 64 accesses per txn: 4096-access tiles
    rng = np.random.default_rng(3)
    txns = [[(int(k), WR if rng.random() < 0.4 else RD)
             for k in rng.choice(5000, size=64, replace=False)] for _ in range(3000)]
    run(sw, make_batch(txns))


def test_ragged_types_and_empty(sw):
    rng = np.random.default_rng(11)
    run(sw, random_batch(rng, 9000, 64, 4000, types=(RD, WR, XP, SCAN)))
    run(sw, random_batch(rng, 9000, 5, 300, p_write=0.5))
    run(sw, make_batch([[] for _ in range(130)]))
    run(sw, make_batch([[], [(1, WR)], [], [(1, RD)], []] * 50))


def test_chain(sw):
    # dependencies inside every tile and across tiles
    run(sw, chain_batch(3000))


def test_hot_single_key(sw):
    txns = [[(7, WR if i % 3 == 0 else RD)] for i in range(10000)]
    run(sw, make_batch(txns))


def test_history_prekill(sw):
    # history-window aborts decided before the solver stay aborted and never
    # add their keys to C
    rng = np.random.default_rng(5)
    b = random_batch(rng, 4000, 12, 600, p_write=0.4)
    n = b.n_txn
    b.start_tn = rng.integers(0, 20, size=n).astype(np.uint64)
    b.finish_tn = (b.start_tn + rng.integers(0, 20, size=n)).astype(np.uint64)
    hk = rng.integers(0, 600, size=300).astype(np.uint64)
    ht = rng.integers(1, 40, size=300).astype(np.uint64)
    sw.history_clear()
    sw.history_append(hk, ht)
    try:
        run(sw, b, hist=(hk, ht), tnc=40)
    finally:
        sw.history_clear()


def test_tpcc(sw):
    run(sw, d.gen_tpcc(n_txn=65536, num_wh=16))


@pytest.mark.parametrize("levels", [2, 4])
def test_device_batch_and_repeat(sw, levels):
    # graph-captured epochs; at 2 levels per synchronisation the serial-only
    # last level leaves list txns past its serial range, so every replay
    # resumes with that level's filter and more levels
    import torch
    sw.set_option(OPT_SWEEP_LEVELS, levels)
    b = d.gen_ycsb(n_txn=100000, zipf_theta=0.9)
    db = b.to_torch("cuda:0")
    erc, _, _ = orc.occ(b)
    for _ in range(3):
        rc, _, _ = sw.occ_validate_epoch(db)
        torch.cuda.synchronize()
        assert np.array_equal(rc.cpu().numpy(), erc)


@pytest.mark.parametrize("device", [False, True])
def test_adaptive_two_level_schedule(device):
    """Auto schedule (DCC_OPT_SWEEP_LEVELS 0, read-only split): an epoch whose
    last predecessor's level-1 list was short runs two levels per graph
    (level 1 a serial tail of 8,192); one whose list then overflows the tail
    continues exactly through more levels after a host round trip, and the
    next epoch goes back to three.  Every epoch bit-exact against the oracle,
    graph replays included (C2, then the headline size, then C2 again)."""
    import torch
    small = d.gen_ycsb(n_txn=65536, zipf_theta=0.9, seed=0x2C2)
    big = d.gen_ycsb(n_txn=1 << 20, zipf_theta=0.9, seed=0x2C3)
    exp = {id(small): orc.occ(small)[0], id(big): orc.occ(big)[0]}
    with d.Engine(0) as eng:
        rounds = []
        for b in [small, small, small, big, big, small, small]:
            bb = b.to_torch("cuda:0") if device else b
            rc, _, st = eng.occ_validate_epoch(bb)
            rc = rc.cpu().numpy() if device else np.asarray(rc)
            assert np.array_equal(rc, exp[id(b)])
            rounds.append(st["rounds"])
        # C2's level-1 list fits the tail: two levels from the second epoch on
        assert rounds[1] == 2 and rounds[2] == 2
