"""GPU parity of the OCC epoch validator against the oracle: bit-exact RC and
commit tn (central_finish numbering) on identical batches."""
import numpy as np
import pytest

import _oracle as orc
import deneva_amd as d
from deneva_amd import RD, WR, XP, SCAN
from helpers import chain_batch, make_batch, random_batch

pytestmark = pytest.mark.gpu


def run(engine, b, tnc=0, hist=None, literal=False, append=False):
    engine.tnc = tnc
    rc, tn, st = engine.occ_validate_epoch(b, want_tn=True, append_history=append)
    hk, ht = (None, None) if hist is None else hist
    erc, etn, etnc = orc.occ(b, hist_keys=hk, hist_tn=ht, tnc=tnc, literal=literal)
    rc = np.asarray(rc)
    bad = np.nonzero(rc != erc)[0]
    assert bad.size == 0, f"rc mismatch at txns {bad[:10]} (gpu {rc[bad[:10]]} oracle {erc[bad[:10]]})"
    assert np.array_equal(np.asarray(tn).astype(np.uint64), etn), "commit tn mismatch"
    assert engine.tnc == etnc
    assert st["n_commit"] == int((erc == 0).sum())
    assert st["n_abort"] == int((erc == 2).sum())
    return rc, st


@pytest.mark.parametrize("theta", [0.0, 0.6, 0.9, 0.99])
@pytest.mark.parametrize("n", [1, 1000, 65536])
def test_ycsb_parity(engine, theta, n):
    run(engine, d.gen_ycsb(n_txn=n, zipf_theta=theta))


@pytest.mark.parametrize("k", [1, 4, 10, 33, 64])
def test_ycsb_keys_per_txn(engine, k):
    run(engine, d.gen_ycsb(n_txn=20000, zipf_theta=0.9, req_per_query=k, table_size=1 << 20))


def test_ycsb_small_table_literal(engine):
    b = d.gen_ycsb(n_txn=4000, zipf_theta=0.6, req_per_query=10, table_size=65536,
                   seed=7)  # config C1 shape (REQ_PER_QUERY=10, theta 0.6, 64K table)
    run(engine, b, literal=True)


@pytest.mark.parametrize("theta", [0.9, 0.99])
def test_ycsb_1m_parity(engine, theta):
    run(engine, d.gen_ycsb(n_txn=1 << 20, zipf_theta=theta, seed=0xD3E7A002))


def test_empty_batch(engine):
    b = make_batch([])
    rc, tn, st = engine.occ_validate_epoch(b, want_tn=True)
    assert st["n_commit"] == 0 and st["n_abort"] == 0


def test_empty_and_readonly_txns(engine):
    b = make_batch([[], [(5, RD)], [], [(5, WR)], [(5, RD)], [], [(5, SCAN), (6, XP)]])
    rc, _ = run(engine, b)
    # XP is not WR: the last txn is read-only for OCC (get_rw_set, occ.cpp:296-317: only WR joins the write set)
    assert list(rc) == [0, 0, 0, 0, 2, 0, 2]


def test_hand_case_asymmetric(engine):
    # T0 reads k1, writes k2.  T1 writes k1 (a row T0 only READ): not checked
    # by backward validation -> commits.  T2 reads k2 (T0 wrote): aborts.
    # T3 writes k3 and reads k9; T4 read-only on k3: aborts (T3 active).
    b = make_batch([[(1, RD), (2, WR)], [(1, WR)], [(2, RD)], [(3, WR), (9, RD)], [(3, RD)]])
    rc, _ = run(engine, b, literal=True)
    assert list(rc) == [0, 0, 2, 0, 2]


def test_aborted_never_kill(engine):
    # T1 is killed by T0; T2 conflicts only with T1 (aborted) -> commits
    b = make_batch([[(1, WR)], [(1, RD), (2, WR)], [(2, RD)]])
    rc, _ = run(engine, b, literal=True)
    assert list(rc) == [0, 2, 0]


def test_same_key_writers(engine):
    n = 5000
    b = make_batch([[(42, WR)] for _ in range(n)])
    rc, _ = run(engine, b)
    assert rc[0] == 0 and (rc[1:] == 2).all()


def test_max_len_and_ragged(engine):
    rng = np.random.default_rng(1)
    for n_keys in (50, 5000, 10 ** 7):
        run(engine, random_batch(rng, 3000, 64, n_keys, p_write=0.4))


def test_types_mix(engine):
    rng = np.random.default_rng(2)
    run(engine, random_batch(rng, 5000, 20, 2000, types=(RD, WR, XP, SCAN)))


def test_keys_near_reserved(engine):
    top = 0xFFFFFFFFFFFFFFFE
    b = make_batch([[(top, WR)], [(top, RD), (0, WR)], [(0, RD)], [(top - 1, WR)]])
    rc, _ = run(engine, b)
    assert list(rc) == [0, 2, 0, 0]


def test_chain_many_rounds(engine):
    # ~n rounds: crosses the 61-round tag space several times (retag path)
    from deneva_amd._abi import OPT_SOLVER
    b = chain_batch(300)
    engine.set_option(OPT_SOLVER, 1)
    try:
        rc, st = run(engine, b)
    finally:
        engine.set_option(OPT_SOLVER, 0)
    assert st["rounds"] > 130
    assert list(rc[:6]) == [0, 2, 0, 2, 0, 2]


@pytest.mark.parametrize("solver", [1, 3])
def test_solvers_agree(engine, solver):
    # every batch shape through the round solver (the sweep's hand-off) and
    # the sweep explicitly
    from deneva_amd._abi import OPT_SOLVER
    rng = np.random.default_rng(33)
    engine.set_option(OPT_SOLVER, solver)
    try:
        run(engine, chain_batch(2000))
        run(engine, random_batch(rng, 5000, 64, 300, p_write=0.5))
        run(engine, random_batch(rng, 5000, 16, 40, types=(RD, WR, XP, SCAN), unique=False))
        run(engine, d.gen_ycsb(n_txn=30000, zipf_theta=0.99, table_size=1 << 16))
        run(engine, make_batch([[(7, WR)] for _ in range(40000)]))  # one segment > 32K writers
    finally:
        engine.set_option(OPT_SOLVER, 0)


def test_history_window(engine):
    # history: tn 5 wrote k7, tn 9 wrote k8
    hist = (np.array([7, 8], np.uint64), np.array([5, 9], np.uint64))
    b = make_batch([[(7, RD)], [(7, RD)], [(8, RD)], [(8, WR)], [(7, RD)]],
                   start_tn=[4, 5, 8, 8, 1], finish_tn=[6, 9, 9, 20, 1])
    engine.history_clear()
    engine.history_append(*hist)
    rc, _ = run(engine, b, hist=hist, literal=True)
    # t0: 4<5<=6 hit; t1: window (5,9] excludes 5; t2: (8,9] hits 9;
    # t3: only WRITES k8 (history checks the read set only); t4: finish<=start
    assert list(rc) == [2, 0, 2, 0, 0]
    engine.history_clear()


def test_history_random(engine):
    rng = np.random.default_rng(3)
    hk = rng.integers(0, 500, size=400).astype(np.uint64)
    ht = rng.integers(1, 100, size=400).astype(np.uint64)
    b = random_batch(rng, 2000, 12, 800, p_write=0.3)
    st = rng.integers(0, 100, size=b.n_txn).astype(np.uint64)
    b.start_tn = st
    b.finish_tn = (st + rng.integers(0, 30, size=b.n_txn)).astype(np.uint64)
    engine.history_clear()
    engine.history_append(hk, ht)
    run(engine, b, hist=(hk, ht), tnc=100)
    engine.history_clear()


def test_multi_epoch_history_append(engine):
    """Epoch replay across epochs: epoch 2 sees epoch 1's committed writes in
    its history window (central_finish pushes them with tn = tnc+1...)."""
    rng = np.random.default_rng(4)
    b1 = random_batch(rng, 1500, 8, 600, p_write=0.5)
    b2 = random_batch(rng, 1500, 8, 600, p_write=0.5)
    n2 = b2.n_txn
    b2.start_tn = np.zeros(n2, np.uint64)
    b2.finish_tn = np.full(n2, 10 ** 9, np.uint64)
    engine.history_clear()
    engine.tnc = 0
    rc1, tn1, _ = engine.occ_validate_epoch(b1, want_tn=True, append_history=True)
    erc1, etn1, tnc1 = orc.occ(b1)
    assert np.array_equal(rc1, erc1) and np.array_equal(tn1, etn1)
    assert engine.tnc == tnc1
    hk, ht = [], []
    for t in range(b1.n_txn):
        if etn1[t]:
            for x in range(b1.offsets[t], b1.offsets[t + 1]):
                if b1.acctype[x] == WR:
                    hk.append(b1.keys[x])
                    ht.append(etn1[t])
    assert engine.history_size == len(hk)
    rc2, tn2, _ = engine.occ_validate_epoch(b2, want_tn=True)
    erc2, etn2, _ = orc.occ(b2, hist_keys=np.array(hk, np.uint64), hist_tn=np.array(ht, np.uint64),
                            tnc=tnc1, literal=True)
    assert np.array_equal(rc2, erc2) and np.array_equal(tn2, etn2)
    engine.history_clear()


def test_device_pointers(engine):
    import torch
    b = d.gen_ycsb(n_txn=50000, zipf_theta=0.9)
    db = b.to_torch("cuda:0")
    engine.tnc = 0
    rc, tn, st = engine.occ_validate_epoch(db, want_tn=True)
    torch.cuda.synchronize()
    erc, etn, _ = orc.occ(b)
    assert np.array_equal(rc.cpu().numpy(), erc)
    assert np.array_equal(tn.cpu().numpy().astype(np.uint64), etn)


def test_repeat_deterministic(engine):
    b = d.gen_ycsb(n_txn=200000, zipf_theta=0.99, seed=11)
    r0 = np.asarray(engine.occ_validate_epoch(b)[0]).copy()
    for _ in range(3):
        assert np.array_equal(np.asarray(engine.occ_validate_epoch(b)[0]), r0)


def test_errors(engine):
    with pytest.raises(d.DccError) as e:
        engine.occ_validate_epoch(make_batch([[(d.KEY_RESERVED, WR)]]))
    assert e.value.code == -22
    with pytest.raises(d.DccError) as e:
        engine.occ_validate_epoch(make_batch([[(i, RD) for i in range(65)]]))
    assert e.value.code == -34
    bad = make_batch([[(1, RD)], [(2, RD)]])
    bad.offsets = np.array([0, 2, 1], np.uint32)
    with pytest.raises(d.DccError) as e:
        engine.occ_validate_epoch(bad)
    assert e.value.code == -22
    # the engine stays usable after errors
    run(engine, make_batch([[(1, WR)], [(1, RD)]]))


@pytest.mark.parametrize("num_wh,wh_update", [(128, 1), (4, 1), (16, 0)])
def test_tpcc_parity(engine, num_wh, wh_update):
    # C3: TPC-C NewOrder + Payment, 262,144-txn batch at 128 warehouses
    n = 262144 if num_wh == 128 else 50000
    run(engine, d.gen_tpcc(n_txn=n, num_wh=num_wh, wh_update=wh_update))
