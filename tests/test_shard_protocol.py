"""CPU, multi-process (gloo, world size 2 and 3): the key-sharded round
protocol of SURVEY.md §8(e) decides exactly what one unsharded epoch decides.

Each rank holds the full offsets but only the accesses whose key it owns
(dcc_shard_filter); per round it computes the per-txn status of its own keys
(oracle_occ_round_status: 1 blocked, 2 killed), the ranks all-reduce it with
MAX, and every rank applies the same verdict (>= 2 abort, 0 commit, 1 stay).
This is the exchange the GPU engine performs with RCCL (dcc_comm.hip), and
the Calvin readiness all-reduce is checked the same way."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import _oracle as orc
import deneva_amd as d


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batches():
    yield d.gen_ycsb(n_txn=6000, zipf_theta=0.9, req_per_query=16, table_size=1 << 16)
    yield d.gen_ycsb(n_txn=4000, zipf_theta=0.99, req_per_query=10, table_size=1 << 12)
    yield d.gen_ycsb(n_txn=3000, zipf_theta=0.6, req_per_query=4, table_size=1 << 10)


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = []
    for b in _batches():
        sb = d.shard_filter(b, rank, world)
        n = b.n_txn
        state = np.zeros(n, np.uint8)
        rounds = 0
        while (state == 0).any():
            st = orc.occ_round_status(sb, state)
            t = torch.from_numpy(st.astype(np.uint8))
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            g = t.numpy()
            und = state == 0
            state[und & (g >= 2)] = 2
            state[und & (g == 0)] = 1
            rounds += 1
            assert rounds <= n + 1
        # Calvin readiness: per-row groups are shard-local; WAIT on any shard wins
        _, crc, _ = orc.calvin(sb)
        t = torch.from_numpy(crc.astype(np.uint8))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        res.append((state.copy(), rounds, t.numpy().copy()))
    out[rank] = res
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_round_protocol_matches_unsharded(world):
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for bi, b in enumerate(_batches()):
        erc, _, _ = orc.occ(b)
        _, ecrc, _ = orc.calvin(b)
        states = [out[r][bi][0] for r in range(world)]
        for r in range(1, world):
            assert np.array_equal(states[r], states[0]), "ranks disagree"
            assert out[r][bi][1] == out[0][bi][1]
        rc = np.where(states[0] == 1, 0, 2).astype(np.uint8)
        assert np.array_equal(rc, erc), f"batch {bi}: sharded decisions differ from unsharded"
        for r in range(world):
            assert np.array_equal(out[r][bi][2], ecrc), f"batch {bi}: calvin readiness differs"


def test_shard_filter_groups_are_shard_local():
    # every row lives on one shard, so each request's grant group computed on
    # its shard equals the unsharded group
    b = d.gen_ycsb(n_txn=3000, zipf_theta=0.9, req_per_query=8, table_size=4000)
    eg, _, _ = orc.calvin(b)
    world = 4
    got = np.full(b.nnz, 0xFFFFFFFE, np.uint32)
    owner = np.array([d.key_shard(int(k), world) for k in b.keys])
    for r in range(world):
        sb = d.shard_filter(b, r, world)
        g, _, _ = orc.calvin(sb)
        got[owner == r] = g
    assert np.array_equal(got, eg)
