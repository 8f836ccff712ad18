"""GPU parity of the OCC prefix peel (occ_peel.hip): the
prefix is solved first, later txns touching a committed prefix write key are
killed by the filter pass, the survivors are compacted and decided (recursively
peeled).  Forced small prefixes drive every path — LDS and global committed-key
sets, several peel levels, empty survivor sets, history-aborted txns — and the
decisions must stay bit-exact against the oracle's serial replay."""
import numpy as np
import pytest

import _oracle as orc
import deneva_amd as d
from deneva_amd import RD, WR, XP, SCAN
from deneva_amd._abi import OPT_PEEL, OPT_PEEL_MIN, OPT_SOLVER
from helpers import chain_batch, make_batch, random_batch

pytestmark = pytest.mark.gpu


@pytest.fixture
def peel_engine(engine):
    # the default solver is the sweep (test_gpu_sweep.py); pin the peel path
    engine.set_option(OPT_SOLVER, 2)
    yield engine
    engine.set_option(OPT_SOLVER, 0)
    engine.set_option(OPT_PEEL, -1)
    engine.set_option(OPT_PEEL_MIN, 32768)


def run(engine, b, prefix, peel_min=32768, hist=None, tnc=0):
    engine.set_option(OPT_PEEL, prefix)
    engine.set_option(OPT_PEEL_MIN, peel_min)
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


@pytest.mark.parametrize("prefix", [1, 7, 64, 1000])
@pytest.mark.parametrize("theta", [0.0, 0.6, 0.9, 0.99])
def test_ycsb_forced_prefix(peel_engine, theta, prefix):
    b = d.gen_ycsb(n_txn=20000, zipf_theta=theta, table_size=1 << 18)
    rc, st = run(peel_engine, b, prefix)
    assert st["peel_prefix"] == prefix


@pytest.mark.parametrize("theta", [0.9, 0.99])
def test_ycsb_multilevel(peel_engine, theta):
    # auto prefix with a low threshold: the survivors are peeled again
    b = d.gen_ycsb(n_txn=200000, zipf_theta=theta, seed=0xD3E7A005)
    rc, st = run(peel_engine, b, -1, peel_min=2048)
    assert st["peel_prefix"] > 0


def test_auto_headline_shape(peel_engine):
    b = d.gen_ycsb(n_txn=1 << 20, zipf_theta=0.9)
    rc, st = run(peel_engine, b, -1)
    assert st["peel_prefix"] == 16384
    assert 0 < st["n_survivors"] < b.n_txn // 10


def test_global_committed_set(peel_engine):
    # > 4096 committed prefix write keys: the filter probes the global set
    rng = np.random.default_rng(11)
    b = random_batch(rng, 30000, 16, 1 << 30, p_write=0.8)
    rc, st = run(peel_engine, b, 8000)
    assert st["peel_prefix"] == 8000


@pytest.mark.parametrize("prefix", [1, 3, 50])
def test_random_ragged_types(peel_engine, prefix):
    rng = np.random.default_rng(prefix)
    run(peel_engine, random_batch(rng, 6000, 64, 3000, types=(RD, WR, XP, SCAN)), prefix)
    run(peel_engine, random_batch(rng, 6000, 20, 200, p_write=0.5), prefix, peel_min=500)


def test_everything_killed(peel_engine):
    # txn 0 writes the key everybody touches: no survivors
    n = 5000
    b = make_batch([[(42, WR)]] + [[(42, RD), (i + 100, WR)] for i in range(n)])
    rc, st = run(peel_engine, b, 1)
    assert st["n_survivors"] == 0
    assert rc[0] == 0 and (rc[1:] == 2).all()


def test_nothing_killed(peel_engine):
    # disjoint keys: every txn survives the filter and commits
    b = make_batch([[(i, WR), (i + 1_000_000, RD)] for i in range(4000)])
    rc, st = run(peel_engine, b, 16)
    assert st["n_survivors"] == 4000 - 16
    assert (rc == 0).all()


def test_prefix_aborts_are_inert(peel_engine):
    # T0 commits k1; T1 (prefix) is killed by it and writes k2; T2 reads k2
    # (written only by an aborted prefix txn) and must commit
    b = make_batch([[(1, WR)], [(1, RD), (2, WR)], [(2, RD)], [(1, RD)], [(3, WR)], [(3, RD)]])
    rc, _ = run(peel_engine, b, 2)
    assert list(rc) == [0, 2, 0, 2, 0, 2]


def test_chain_peeled(peel_engine):
    b = chain_batch(3000)
    rc, st = run(peel_engine, b, 100, peel_min=200)
    assert list(rc[:4]) == [0, 2, 0, 2]


def test_history_with_peel(peel_engine):
    rng = np.random.default_rng(5)
    b = random_batch(rng, 4000, 8, 500, p_write=0.4)
    n = b.n_txn
    b.start_tn = rng.integers(0, 20, size=n).astype(np.uint64)
    b.finish_tn = (b.start_tn + rng.integers(0, 20, size=n)).astype(np.uint64)
    hk = rng.integers(0, 500, size=300).astype(np.uint64)
    ht = rng.integers(1, 40, size=300).astype(np.uint64)
    peel_engine.history_clear()
    peel_engine.history_append(hk, ht)
    try:
        run(peel_engine, b, 64, peel_min=500, hist=(hk, ht), tnc=40)
    finally:
        peel_engine.history_clear()


def test_tpcc_peel(peel_engine):
    b = d.gen_tpcc(n_txn=65536, num_wh=16)
    rc, st = run(peel_engine, b, -1)
    assert st["peel_prefix"] > 0


def test_device_pointers_peel(peel_engine):
    import torch
    b = d.gen_ycsb(n_txn=100000, zipf_theta=0.9)
    peel_engine.set_option(OPT_PEEL, -1)
    rc, tn, st = peel_engine.occ_validate_epoch(b.to_torch("cuda:0"), want_tn=True)
    torch.cuda.synchronize()
    erc, etn, _ = orc.occ(b)
    assert np.array_equal(rc.cpu().numpy(), erc)
    assert st["peel_prefix"] > 0


def test_peel_matches_rounds(peel_engine):
    # same decisions with the peel on and off, twice (determinism)
    b = d.gen_ycsb(n_txn=300000, zipf_theta=0.9, seed=0xD3E7A009)
    peel_engine.set_option(OPT_PEEL, 0)
    rc0, _, st0 = peel_engine.occ_validate_epoch(b)
    peel_engine.set_option(OPT_PEEL, -1)
    rc1, _, st1 = peel_engine.occ_validate_epoch(b)
    rc2, _, _ = peel_engine.occ_validate_epoch(b)
    assert st0["peel_prefix"] == 0 and st1["peel_prefix"] > 0
    assert np.array_equal(np.asarray(rc0), np.asarray(rc1))
    assert np.array_equal(np.asarray(rc1), np.asarray(rc2))
