"""GPU: the key-sharded engine path end to end.

Ranks are separate processes sharing the box's one GPU; each owns the keys
with dcc_key_shard(key, world) == rank and exchanges the per-round status
through dcc_comm_init_host (gloo all-reduce MAX on the host).  The engine
code path is the one RCCL drives on an 8-GPU node — only the all-reduce
transport differs.  OCC runs the key-sharded sweep in both forms: ranks
given only their accesses (dcc_shard_filter; the serial range's records
all-gathered and merged on every rank) and ranks given the whole epoch
(DCC_SHARD_SELF; each keeps its key shard on the device and gathers the
serial ranges from its copy of the batch); the filters' kill bits are
all-gathered.  Decisions, commit tn, history across epochs, and Calvin
grant groups / readiness must equal the unsharded oracle bit for bit."""
import os
import socket

import numpy as np
import pytest

import _oracle as orc
import deneva_amd as d

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _occ_batches():
    yield d.gen_ycsb(n_txn=1, zipf_theta=0.9)
    yield d.gen_ycsb(n_txn=20000, zipf_theta=0.9, req_per_query=16, table_size=1 << 16)
    yield d.gen_ycsb(n_txn=65536, zipf_theta=0.99)
    yield d.gen_ycsb(n_txn=5000, zipf_theta=0.6, req_per_query=33, table_size=1 << 12)


def _occ(eng, b, rank, world, whole, **kw):
    """One key-sharded OCC epoch: the rank's accesses only, or the whole batch."""
    if whole:
        return eng.occ_validate_epoch(b, shard_self=True, **kw)
    return eng.occ_validate_epoch(d.shard_filter(b, rank, world), **kw)


def _worker(rank, world, port, out, whole=False):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def allreduce_max(buf):
        t = torch.from_numpy(buf)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)

    eng = d.Engine(0)
    eng.comm_init_host(rank, world, allreduce_max)
    assert eng.comm_rank == rank and eng.comm_size == world
    res = {"occ": [], "hist": [], "calvin": []}
    for b in _occ_batches():
        eng.tnc = 0  # each batch is checked as a fresh epoch
        rc, tn, st = _occ(eng, b, rank, world, whole, want_tn=True)
        res["occ"].append((np.asarray(rc).copy(), np.asarray(tn).copy(), st["rounds"],
                           st["n_shards"], st["peel_prefix"], b.n_txn))
    # three epochs with history (start/finish windows) appended across epochs
    eng.tnc = 0
    eng.history_clear()
    for e in range(3):
        b = d.gen_ycsb(n_txn=4000, zipf_theta=0.8, req_per_query=8, table_size=3000, seed=100 + e)
        n = b.n_txn
        b.start_tn = np.full(n, 0, np.uint64)
        b.finish_tn = np.full(n, 1 << 40, np.uint64)
        rc, tn, st = _occ(eng, b, rank, world, whole, want_tn=True, append_history=True)
        res["hist"].append((np.asarray(rc).copy(), np.asarray(tn).copy(), eng.tnc))
    for theta in (0.0, 0.9):
        b = d.gen_ycsb(n_txn=30000, zipf_theta=theta, req_per_query=16, table_size=1 << 14)
        g, crc, _, st = eng.calvin_order_epoch(d.shard_filter(b, rank, world), want_group=True)
        res["calvin"].append((np.asarray(g).copy(), np.asarray(crc).copy()))
    out[rank] = res
    dist.destroy_process_group()


@pytest.mark.parametrize("whole", [False, True])
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_engine_matches_unsharded(world, whole):
    import torch.multiprocessing as mp
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out, whole), nprocs=world, join=True)
    for bi, b in enumerate(_occ_batches()):
        erc, etn, _ = orc.occ(b)
        for r in range(world):
            rc, tn, rounds, nsh, prefix, n = out[r]["occ"][bi]
            assert nsh == world
            if n > 1024:
                assert prefix > 0, "the key-sharded sweep decided the serial prefix"
            assert np.array_equal(rc, erc), f"rank {r} batch {bi}: rc differs from unsharded"
            assert np.array_equal(tn.astype(np.uint64), etn), f"rank {r} batch {bi}: tn differs"
    # history epochs: replay the oracle epoch by epoch with the same windows
    hk = np.zeros(0, np.uint64)
    ht = np.zeros(0, np.uint64)
    tnc = 0
    for e in range(3):
        b = d.gen_ycsb(n_txn=4000, zipf_theta=0.8, req_per_query=8, table_size=3000, seed=100 + e)
        b.start_tn = np.full(b.n_txn, 0, np.uint64)
        b.finish_tn = np.full(b.n_txn, 1 << 40, np.uint64)
        erc, etn, etnc = orc.occ(b, hist_keys=hk, hist_tn=ht, tnc=tnc)
        for r in range(world):
            rc, tn, rtnc = out[r]["hist"][e]
            assert np.array_equal(rc, erc), f"rank {r} epoch {e}: history rc differs"
            assert np.array_equal(tn.astype(np.uint64), etn)
            assert rtnc == etnc
        # committed writes join the history
        off = b.offsets
        for t in np.nonzero(etn)[0]:
            for x in range(off[t], off[t + 1]):
                if b.acctype[x] == d.WR:
                    hk = np.append(hk, b.keys[x])
                    ht = np.append(ht, etn[t])
        tnc = etnc
    for ci, theta in enumerate((0.0, 0.9)):
        b = d.gen_ycsb(n_txn=30000, zipf_theta=theta, req_per_query=16, table_size=1 << 14)
        eg, ecrc, _ = orc.calvin(b)
        owner = np.array([d.key_shard(int(k), world) for k in b.keys])
        got = np.full(b.nnz, 0xFFFFFFFE, np.uint32)
        for r in range(world):
            g, crc = out[r]["calvin"][ci]
            got[owner == r] = g.astype(np.uint32)
            assert np.array_equal(crc, ecrc), f"rank {r}: calvin readiness differs"
        assert np.array_equal(got, eg), "calvin grant groups differ"


def _c5_worker(rank, world, port, out, whole=False):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def allreduce_max(buf):
        t = torch.from_numpy(buf)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)

    eng = d.Engine(0)
    eng.comm_init_host(rank, world, allreduce_max)
    b = d.gen_ycsb(n_txn=1 << 20, zipf_theta=0.99, seed=0xD3E7A002)
    eng.tnc = 0
    rc, tn, st = _occ(eng, b, rank, world, whole, want_tn=True)
    out[rank] = (np.asarray(rc).copy(), np.asarray(tn).copy(), st["n_shards"], eng.tnc)
    eng.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("whole", [False, True])
@pytest.mark.parametrize("world", [4, 8])
def test_sharded_c5_full_size(world, whole):
    """BASELINE config C5 (1,048,576 YCSB txns, theta=0.99) key-sharded over
    4 and 8 ranks (processes sharing the GPU, gloo exchange)."""
    import torch.multiprocessing as mp
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_c5_worker, args=(world, _free_port(), out, whole), nprocs=world, join=True)
    b = d.gen_ycsb(n_txn=1 << 20, zipf_theta=0.99, seed=0xD3E7A002)
    erc, etn, etnc = orc.occ(b)
    for r in range(world):
        rc, tn, nsh, tnc = out[r]
        assert nsh == world and tnc == etnc
        assert np.array_equal(rc, erc), f"rank {r}: rc differs from the oracle"
        assert np.array_equal(tn.astype(np.uint64), etn), f"rank {r}: tn differs"


def _c4_worker(rank, world, port, out):
    import torch
    import torch.distributed as dist
    from helpers import c4_batch
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def allreduce_max(buf):
        t = torch.from_numpy(buf)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)

    eng = d.Engine(0)
    eng.comm_init_host(rank, world, allreduce_max)
    b = c4_batch()
    g, crc, _, st = eng.calvin_order_epoch(d.shard_filter(b, rank, world), want_group=True)
    out[rank] = (np.asarray(g).astype(np.uint32).copy(), np.asarray(crc).copy(), st["n_shards"])
    eng.close()
    dist.destroy_process_group()


def test_sharded_calvin_c4_full_size_8_ranks():
    """BASELINE config C4 (1,048,576 txns, 16 partitions, sequencer (origin,
    FIFO) order) key-sharded over 8 rank processes: each locks only its own
    rows (ycsb_txn.cpp:62-63), readiness is the MAX all-reduce of the WAIT
    bytes; the scattered groups and readiness equal the oracle's literal
    Row_lock order (row_lock.cpp:52-216)."""
    import torch.multiprocessing as mp
    from helpers import c4_batch
    world = 8
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_c4_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    b = c4_batch()
    eg, erc, _ = orc.calvin(b)
    owner = d.shard_of_keys(np.asarray(b.keys), world)
    got = np.full(b.nnz, 0xFFFFFFFE, np.uint32)
    for r in range(world):
        g, crc, nsh = out[r]
        assert nsh == world
        got[owner == r] = g[: int((owner == r).sum())]
        assert np.array_equal(crc, erc), f"rank {r}: calvin readiness differs"
    assert np.array_equal(got, eg), "calvin grant groups differ"
