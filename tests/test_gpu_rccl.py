"""GPU: the RCCL call path on a one-GPU box.  A one-rank RCCL clique
(DCC_OPT_COMM_SOLO: ncclCommInitRank with nranks = 1) makes the context run
the key-sharded paths of SURVEY.md §8(e) with their collectives --
ncclAllReduce (ncclMax) of the per-txn status, has-write and Calvin readiness
bytes, ncclAllGather of the sweep filters' kill words
(worker_thread.cpp:326-335's AND of votes, dcc_comm.hip) -- over that one
rank.  Decisions and commit tns equal the oracle's, and dcc_comm_calls
records that the collectives ran.  This executes the RCCL calls; it does not
measure multi-GPU scaling (the 8-GPU node is the driver's)."""
import numpy as np
import pytest

import _oracle as orc
import deneva_amd as d
from deneva_amd._abi import OPT_COMM_SOLO, OPT_SOLVER

pytestmark = pytest.mark.gpu


@pytest.fixture
def solo():
    eng = d.Engine(0)
    eng.set_option(OPT_COMM_SOLO, 1)
    eng.comm_init(0, 1, d.comm_unique_id())
    yield eng
    eng.close()


@pytest.mark.parametrize("shard_self", [False, True])
@pytest.mark.parametrize("n,theta", [(65536, 0.9), (1 << 20, 0.99)])
def test_solo_rccl_occ(solo, n, theta, shard_self):
    """The key-sharded sweep: with the whole batch (DCC_SHARD_SELF) the
    ranks exchange only kill words (ncclAllGather per level); with the
    rank's own accesses, record counts and records as well."""
    b = d.gen_ycsb(n_txn=n, zipf_theta=theta, seed=0xCC01 + n)
    erc, etn, etnc = orc.occ(b)
    solo.tnc = 0
    c0 = solo.comm_calls
    rc, tn, st = solo.occ_validate_epoch(b, want_tn=True, shard_self=shard_self)
    assert np.array_equal(np.asarray(rc), erc)
    assert np.array_equal(np.asarray(tn, np.uint64), etn)
    assert solo.tnc == etnc and st["n_shards"] == 1
    assert solo.comm_calls > c0  # the collectives were enqueued on RCCL


def test_solo_rccl_round_solver_and_history(solo):
    """The fixed-point round solver's per-round status all-reduce, with
    TS_CAS windows (their abort bytes all-reduced too) and history appends."""
    rng = np.random.default_rng(41)
    solo.set_option(OPT_SOLVER, 1)
    solo.tnc = 0
    solo.history_clear()
    hk, ht = np.zeros(0, np.uint64), np.zeros(0, np.uint64)
    tnc = 0
    for e in range(3):
        b = d.gen_ycsb(n_txn=30000, zipf_theta=0.8, table_size=1 << 15, seed=0xCC10 + e)
        b.start_tn = rng.integers(0, tnc + 1, size=b.n_txn).astype(np.uint64)
        b.finish_tn = (b.start_tn + rng.integers(0, 500, size=b.n_txn)).astype(np.uint64)
        erc, etn, etnc = orc.occ(b, hist_keys=hk, hist_tn=ht, tnc=tnc)
        c0 = solo.comm_calls
        rc, tn, _ = solo.occ_validate_epoch(b, want_tn=True, append_history=True)
        assert np.array_equal(np.asarray(rc), erc) and np.array_equal(np.asarray(tn), etn)
        assert solo.comm_calls > c0
        off = np.asarray(b.offsets, np.int64)
        owner = np.repeat(np.arange(b.n_txn), np.diff(off))
        sel = (np.asarray(b.acctype) == d.WR) & (etn[owner] != 0)
        hk = np.concatenate([hk, np.asarray(b.keys)[sel]])
        ht = np.concatenate([ht, etn[owner[sel]]])
        tnc = etnc
    assert solo.history_size == hk.size


def test_solo_rccl_calvin(solo):
    """Calvin: grant groups per row, readiness all-reduced (ncclMax)."""
    c = d.gen_ycsb(n_txn=100000, zipf_theta=0.9, part_cnt=16, chunk_txns=4096, seed=0xCC20)
    eg, erc, _ = orc.calvin(c)
    c0 = solo.comm_calls
    g, rc, _, _ = solo.calvin_order_epoch(c, want_group=True)
    assert np.array_equal(np.asarray(g).astype(np.uint32), eg)
    assert np.array_equal(np.asarray(rc), erc)
    assert solo.comm_calls > c0


def test_solo_option_after_init_is_rejected(solo):
    with pytest.raises(d.DccError):
        solo.set_option(OPT_COMM_SOLO, 0)
