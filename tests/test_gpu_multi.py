"""GPU: the single-process multi-GPU context (dcc_init_multi, SURVEY.md
§8(b): one process, the node's GPUs internal to the context).  On a one-GPU
box the shards share the GPU and exchange in-process (the path is the one
ncclCommInitAll drives on an 8-GPU node, only the transport differs).
Decisions, commit tns, history and Calvin groups must equal one GPU / the
oracle bit for bit, at the full C5 size."""
import numpy as np
import pytest

import _oracle as orc
import deneva_amd as d
from deneva_amd import RD, WR

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c5():
    b = d.gen_ycsb(n_txn=1 << 20, zipf_theta=0.99, seed=0xD3E7A002)
    erc, etn, etnc = orc.occ(b)
    return b, erc, etn, etnc


@pytest.mark.parametrize("shards", [2, 4, 8])
def test_multi_occ_c5_full(c5, shards):
    b, erc, etn, etnc = c5
    with d.Engine(devices=[0] * shards) as eng:
        assert eng.comm_size == shards
        eng.tnc = 0
        rc, tn, st = eng.occ_validate_epoch(b, want_tn=True)
        assert np.array_equal(np.asarray(rc), erc)
        assert np.array_equal(np.asarray(tn, np.uint64), etn)
        assert eng.tnc == etnc and st["n_shards"] == shards


def test_multi_history_and_calvin():
    rng = np.random.default_rng(3)
    with d.Engine(devices=[0, 0, 0]) as eng:
        eng.tnc = 0
        eng.history_clear()
        hk, ht = np.zeros(0, np.uint64), np.zeros(0, np.uint64)
        tnc = 0
        for e in range(3):
            b = d.gen_ycsb(n_txn=20000, zipf_theta=0.7, table_size=1 << 14, seed=40 + e)
            b.start_tn = rng.integers(0, tnc + 1, size=b.n_txn).astype(np.uint64)
            b.finish_tn = (b.start_tn + rng.integers(0, 200, size=b.n_txn)).astype(np.uint64)
            erc, etn, etnc = orc.occ(b, hist_keys=hk, hist_tn=ht, tnc=tnc)
            rc, tn, _ = eng.occ_validate_epoch(b, want_tn=True, append_history=True)
            assert np.array_equal(np.asarray(rc), erc) and np.array_equal(np.asarray(tn), etn)
            off = np.asarray(b.offsets, np.int64)
            owner = np.repeat(np.arange(b.n_txn), np.diff(off))
            sel = (np.asarray(b.acctype) == WR) & (etn[owner] != 0)
            hk = np.concatenate([hk, np.asarray(b.keys)[sel]])
            ht = np.concatenate([ht, etn[owner[sel]]])
            tnc = etnc
        assert eng.history_size == hk.size
        c = d.gen_ycsb(n_txn=50000, zipf_theta=0.9, part_cnt=4, chunk_txns=4096)
        c.order = rng.integers(0, 1 << 20, size=c.n_txn).astype(np.uint64)
        g, crc, _, _ = eng.calvin_order_epoch(c, want_group=True)
        eg, erc2, _ = orc.calvin(c)
        assert np.array_equal(np.asarray(g).astype(np.uint32), eg)
        assert np.array_equal(np.asarray(crc), erc2)
        hk2 = np.asarray(c.keys[:3000], np.uint64)
        ha2 = np.where(np.arange(3000) % 3 == 0, WR, RD).astype(np.uint8)
        g, crc, _, _ = eng.calvin_order_epoch(c, want_group=True, held=(hk2, ha2))
        eg, erc2 = orc.calvin_held(c, hk2, ha2)
        assert np.array_equal(np.asarray(g).astype(np.uint32), eg)
        assert np.array_equal(np.asarray(crc), erc2)


@pytest.mark.parametrize("dev", [False, True])
def test_multi_maat_on_rank0(dev):
    """MaaT on a multi-GPU context runs the whole epoch on rank 0 (its row
    table holds every row's timestamps): rc, commit timestamps and the row
    timestamps equal the oracle's, across two epochs."""
    with d.Engine(devices=[0, 0, 0]) as eng:
        eng.maat_rows_clear()
        rk = lr = lw = None
        for e in range(2):
            b = d.gen_ycsb(n_txn=20000, zipf_theta=0.9, table_size=1 << 15, seed=0x3A0 + e)
            bb = b.to_torch("cuda:0") if dev else b
            rc, cts, _ = eng.maat_validate_epoch(bb)
            if dev:
                rc, cts = rc.cpu().numpy(), cts.cpu().numpy().view(np.uint64)
            erc, ects, (rk, lr, lw) = orc.maat(b, rk, lr, lw)
            assert np.array_equal(np.asarray(rc), erc), f"epoch {e}"
            assert np.array_equal(np.asarray(cts, np.uint64), ects), f"epoch {e}"
            glr, glw = eng.maat_rows_get(rk)
            assert np.array_equal(glr, lr) and np.array_equal(glw, lw)
        assert eng.maat_rows_size == rk.size


@pytest.mark.parametrize("dev", [False, True])
def test_multi_snapshot_key_sharded(dev):
    """Captured-snapshot validation on a multi-GPU context: each rank decides
    its key shard against its history shard (the history is sharded by key,
    dcc_occ_history_append) and the captured active lists; a txn commits iff
    every rank commits it -- equal to the literal snapshot oracle."""
    import torch
    from test_snapshot_oracle import live_case
    hist0 = [(tn, [int(k) for k in np.random.default_rng(3).integers(0, 200, 3)]) for tn in range(1, 41)]
    b, cap = live_case(2, n=2000, threads=16, hist0=hist0, tnc0=40)
    want = orc.occ_snapshot(b, cap["active_off"], cap["active_idx"], cap["hist_top"], cap["hist_keys"],
                            cap["hist_tn"])
    assert np.array_equal(want, cap["rc"])
    with d.Engine(devices=[0, 0, 0]) as eng:
        eng.history_clear()
        eng.history_append(cap["hist_keys"], cap["hist_tn"])
        if dev:
            cv = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(
                np.int64 if a.dtype == np.uint64 else np.int32)).cuda()
            aidx = cap["active_idx"]
            rc, st = eng.occ_validate_snapshot(b.to_torch(), cv(cap["active_off"]),
                                               cv(aidx) if len(aidx) else torch.zeros(1, dtype=torch.int32,
                                                                                      device="cuda"),
                                               cv(cap["hist_top"]))
            rc = rc.cpu().numpy()
        else:
            rc, st = eng.occ_validate_snapshot(b, cap["active_off"], cap["active_idx"], cap["hist_top"])
            rc = np.asarray(rc)
        assert np.array_equal(rc, want)
        assert st["n_commit"] == int((want == 0).sum()) and st["n_shards"] == 3
        eng.history_clear()


def test_multi_calvin_held_device_batch():
    """Held rows with a device batch on a multi-GPU context (the held arrays
    are device arrays too): sharded by row like the host form, equal to the
    literal Row_lock replay of the held prefix then the epoch."""
    import torch
    c = d.gen_ycsb(n_txn=50000, zipf_theta=0.9, part_cnt=4, chunk_txns=4096, seed=0x4E1D)
    c.order = np.random.default_rng(9).integers(0, 1 << 20, size=c.n_txn).astype(np.uint64)
    hk = np.asarray(c.keys[:3000], np.uint64)
    ha = np.where(np.arange(3000) % 3 == 0, WR, RD).astype(np.uint8)
    eg, erc = orc.calvin_held(c, hk, ha)
    dh = (torch.from_numpy(hk.view(np.int64)).cuda(), torch.from_numpy(ha).cuda())
    with d.Engine(devices=[0, 0, 0]) as eng:
        g, rc, _, _ = eng.calvin_order_epoch(c.to_torch("cuda:0"), want_group=True, held=dh)
        torch.cuda.synchronize()
        assert np.array_equal(g.cpu().numpy().view(np.uint32), eg)
        assert np.array_equal(rc.cpu().numpy(), erc)


@pytest.mark.parametrize("shards", [2, 4])
def test_multi_device_batch_occ(c5, shards):
    """A device batch (DCC_DEVICE_PTRS): every rank partitions it on its own
    GPU (shard_dev.hip) instead of the host splitting it; decisions and commit
    tns land in the caller's device arrays, equal to the oracle's."""
    import torch
    b, erc, etn, etnc = c5
    db = b.to_torch("cuda:0")
    with d.Engine(devices=[0] * shards) as eng:
        eng.tnc = 0
        rc, tn, st = eng.occ_validate_epoch(db, want_tn=True)
        torch.cuda.synchronize()
        assert np.array_equal(rc.cpu().numpy(), erc)
        assert np.array_equal(tn.cpu().numpy().view(np.uint64), etn)
        assert eng.tnc == etnc and st["n_shards"] == shards


def test_multi_device_batch_calvin():
    import torch
    c = d.gen_ycsb(n_txn=60000, zipf_theta=0.9, part_cnt=4, chunk_txns=4096)
    c.order = np.random.default_rng(5).integers(0, 1 << 20, size=c.n_txn).astype(np.uint64)
    eg, erc, _ = orc.calvin(c)
    with d.Engine(devices=[0, 0, 0]) as eng:
        g, rc, _, _ = eng.calvin_order_epoch(c.to_torch("cuda:0"), want_group=True)
        torch.cuda.synchronize()
        assert np.array_equal(g.cpu().numpy().view(np.uint32), eg)
        assert np.array_equal(rc.cpu().numpy(), erc)


@pytest.fixture(scope="module")
def c4():
    from helpers import c4_batch
    b = c4_batch()
    eg, erc, _ = orc.calvin(b)
    return b, eg, erc


def test_multi_calvin_c4_full_8_shards(c4):
    """BASELINE config C4 at full size, key-sharded 8 ways in one multi-GPU
    context (each shard locks only its own rows, ycsb_txn.cpp:62-63); the
    scattered grant groups and the all-reduced readiness equal the oracle's
    literal Row_lock order and the one-GPU engine's."""
    b, eg, erc = c4
    with d.Engine(0) as one:
        g1, rc1, _, _ = one.calvin_order_epoch(b, want_group=True)
    g1 = np.asarray(g1).astype(np.uint32)
    assert np.array_equal(g1, eg) and np.array_equal(np.asarray(rc1), erc)
    with d.Engine(devices=[0] * 8) as eng:
        assert eng.comm_size == 8
        g, rc, _, st = eng.calvin_order_epoch(b, want_group=True)
        assert np.array_equal(np.asarray(g).astype(np.uint32), eg)
        assert np.array_equal(np.asarray(rc), erc)
        assert st["n_shards"] == 8 and st["n_commit"] == int((erc == 0).sum())


def test_multi_calvin_waves_on_rank0():
    """Wave levels on a multi-GPU context: the whole epoch runs on rank 0's
    GPU (the levels chain through every row); groups, readiness and waves
    equal the oracle's, host and device batches."""
    import torch
    from helpers import c4_batch
    b = c4_batch(40000)
    eg, erc, ew = orc.calvin(b)
    with d.Engine(devices=[0, 0, 0]) as eng:
        g, rc, w, st = eng.calvin_order_epoch(b, want_group=True, want_wave=True)
        assert np.array_equal(np.asarray(g).astype(np.uint32), eg)
        assert np.array_equal(np.asarray(rc), erc)
        assert np.array_equal(np.asarray(w).astype(np.uint32), ew)
        assert st["rounds"] == int(ew.max()) + 1
        g2, rc2, w2, _ = eng.calvin_order_epoch(b.to_torch("cuda:0"), want_group=True, want_wave=True)
        torch.cuda.synchronize()
        assert np.array_equal(w2.cpu().numpy().view(np.uint32)[:b.n_txn], ew)
        assert np.array_equal(rc2.cpu().numpy()[:b.n_txn], erc)


@pytest.mark.parametrize("bad_rank", [0, 2])
def test_multi_rank_failure_does_not_hang(bad_rank):
    """One rank fails before its first exchange (fault injection): every
    rank returns instead of waiting for it (the exchange is poisoned), the
    failing rank's error is reported, and the next epoch runs normally."""
    from deneva_amd._abi import OPT_FAIL_RANK
    b = d.gen_ycsb(n_txn=30000, zipf_theta=0.9, table_size=1 << 16)
    erc, _, _ = orc.occ(b)
    c = d.gen_ycsb(n_txn=20000, zipf_theta=0.9, part_cnt=4, chunk_txns=4096)
    eg, ecrc, _ = orc.calvin(c)
    with d.Engine(devices=[0] * 4) as eng:
        eng.set_option(OPT_FAIL_RANK, bad_rank)
        with pytest.raises(d.DccError, match="injected"):
            eng.occ_validate_epoch(b)
        rc, _, _ = eng.occ_validate_epoch(b)
        assert np.array_equal(np.asarray(rc), erc)
        eng.set_option(OPT_FAIL_RANK, 3)
        with pytest.raises(d.DccError, match="injected"):
            eng.calvin_order_epoch(c, want_group=True)
        g, crc, _, _ = eng.calvin_order_epoch(c, want_group=True)
        assert np.array_equal(np.asarray(g).astype(np.uint32), eg)
        assert np.array_equal(np.asarray(crc), ecrc)


@pytest.mark.parametrize("fault", ["decreasing", "first", "last", "too_long"])
def test_multi_rejects_malformed_device_batch(fault):
    """A malformed device batch is rejected by every rank before any exchange
    (rank 0 validates the caller's arrays; the shards' own offsets are always
    well formed, so no rank could notice alone); the context stays usable."""
    import torch
    b = d.gen_ycsb(n_txn=4096, zipf_theta=0.9, table_size=1 << 14)
    off = np.asarray(b.offsets, np.uint32).copy()
    keys, at = np.asarray(b.keys), np.asarray(b.acctype)
    if fault == "decreasing":
        off[100] = off[99] - 1
    elif fault == "first":
        off[0] = 1
    elif fault == "last":
        off[-1] = off[-1] - 3
    else:  # one txn of 80 accesses (> MAX_ROW_PER_TXN)
        off = np.concatenate([[0], np.arange(80, keys.size + 1, 16, dtype=np.int64)])
        off[-1] = keys.size
        off = off.astype(np.uint32)
    bad = d.EpochBatch(off, keys, at).to_torch("cuda:0")
    erc, _, _ = orc.occ(b)
    with d.Engine(devices=[0, 0, 0]) as eng:
        with pytest.raises(d.DccError):
            eng.occ_validate_epoch(bad)
        with pytest.raises(d.DccError):
            eng.calvin_order_epoch(bad, want_group=True)
        rc, _, _ = eng.occ_validate_epoch(b.to_torch("cuda:0"))
        torch.cuda.synchronize()
        assert np.array_equal(rc.cpu().numpy(), erc)


def test_multi_occ_growing_epochs_share_one_gpu():
    """Two shards of one context on one GPU, commit tn wanted, epochs growing
    from one to the next (every epoch reallocates the central_finish
    look-back words; the allocator may hand a shard memory the other shard
    just freed, holding words with the same tag sequence).  Round 5's
    intermittent 'central_finish numbered 339 txns, 480 committed writers'
    was a grown buffer whose tail was never cleared (occ_begin); every
    epoch's commit tns must equal the oracle's (occ.cpp:277-286)."""
    with d.Engine(devices=[0, 0]) as eng, d.Engine(0) as other:
        eng.tnc = 0
        tnc = 0
        for e, n in enumerate([700, 3000, 9000, 40000, 150000, 600000]):
            b = d.gen_ycsb(n_txn=n, zipf_theta=0.99, table_size=1 << 18, seed=0x61A0 + e)
            erc, etn, etnc = orc.occ(b, tnc=tnc)
            rc, tn, _ = eng.occ_validate_epoch(b, want_tn=True)
            assert np.array_equal(np.asarray(rc), erc), f"epoch {e}"
            assert np.array_equal(np.asarray(tn, np.uint64), etn), f"epoch {e}"
            assert eng.tnc == etnc
            tnc = etnc
            # a third context on the same GPU churns the allocator in between
            other.tnc = 0
            other.occ_validate_epoch(b, want_tn=True)


@pytest.mark.parametrize("solver", [1, 3])
def test_multi_shard_self_history_per_solver(solver):
    """Every solver shards the batch by key: with the round solver too, a
    rank appends only its own keys' committed writes, so the context's
    history holds each pair once (the round solver used to stage
    the whole batch as its shard)."""
    from deneva_amd._abi import OPT_SOLVER
    rng = np.random.default_rng(19)
    with d.Engine(devices=[0, 0, 0]) as eng:
        eng.set_option(OPT_SOLVER, solver)
        eng.tnc = 0
        eng.history_clear()
        hk, ht = np.zeros(0, np.uint64), np.zeros(0, np.uint64)
        tnc = 0
        for e in range(3):
            b = d.gen_ycsb(n_txn=12000, zipf_theta=0.8, table_size=1 << 14, seed=70 + e)
            b.start_tn = rng.integers(0, tnc + 1, size=b.n_txn).astype(np.uint64)
            b.finish_tn = (b.start_tn + rng.integers(0, 300, size=b.n_txn)).astype(np.uint64)
            erc, etn, etnc = orc.occ(b, hist_keys=hk, hist_tn=ht, tnc=tnc)
            rc, tn, _ = eng.occ_validate_epoch(b, want_tn=True, append_history=True)
            assert np.array_equal(np.asarray(rc), erc) and np.array_equal(np.asarray(tn), etn)
            off = np.asarray(b.offsets, np.int64)
            owner = np.repeat(np.arange(b.n_txn), np.diff(off))
            sel = (np.asarray(b.acctype) == WR) & (etn[owner] != 0)
            hk = np.concatenate([hk, np.asarray(b.keys)[sel]])
            ht = np.concatenate([ht, etn[owner[sel]]])
            tnc = etnc
            assert eng.history_size == hk.size
