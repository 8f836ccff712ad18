"""GPU parity of the Calvin epoch lock-ordering engine against the oracle:
bit-exact grant group per request, acquire_locks RC per txn and wave level
per txn, on identical batches."""
import numpy as np
import pytest

import _oracle as orc
import deneva_amd as d
from deneva_amd import RD, WR, XP, SCAN
from helpers import make_batch, random_batch

pytestmark = pytest.mark.gpu


def run(engine, b, waves=True, literal=False):
    g, rc, w, st = engine.calvin_order_epoch(b, want_group=True, want_wave=waves)
    eg, erc, ew = orc.calvin(b, literal=literal)
    g = np.asarray(g).astype(np.uint32)
    rc = np.asarray(rc)
    bad = np.nonzero(g != eg)[0]
    assert bad.size == 0, f"group mismatch at requests {bad[:10]} (gpu {g[bad[:10]]} oracle {eg[bad[:10]]})"
    bad = np.nonzero(rc != erc)[0]
    assert bad.size == 0, f"rc mismatch at txns {bad[:10]}"
    if waves:
        w = np.asarray(w).astype(np.uint32)
        bad = np.nonzero(w != ew)[0]
        assert bad.size == 0, f"wave mismatch at txns {bad[:10]} (gpu {w[bad[:10]]} oracle {ew[bad[:10]]})"
        if b.n_txn:
            assert st["rounds"] == int(ew.max()) + 1
    assert st["n_commit"] == int((erc == 0).sum())
    assert st["n_abort"] == int((erc == 3).sum())
    return g, rc, st


def c4_order(b):
    """Sequencer order of a partitioned YCSB batch: (origin = home partition,
    FIFO seq within the origin) — sched_dequeue's (epoch, origin, FIFO)."""
    home = b.meta["home"].astype(np.uint64)
    seq = np.zeros(b.n_txn, np.uint64)
    for h in np.unique(home):
        idx = np.nonzero(home == h)[0]
        seq[idx] = np.arange(idx.size, dtype=np.uint64)
    return (home << np.uint64(32)) | seq


def test_kat_fifo_no_barging(engine):
    g, rc, _ = run(engine, make_batch([[(1, RD)], [(1, WR)], [(1, RD)], [(1, RD)], [(1, WR)]]),
                   literal=True)
    assert list(g) == [0, 1, 2, 2, 3]
    assert list(rc) == [0, 3, 3, 3, 3]


def test_kat_dedup_and_types(engine):
    g, rc, _ = run(engine, make_batch([[(5, RD), (5, WR)], [(5, SCAN)], [(6, XP)], [(6, SCAN)]]),
                   literal=True)
    assert g[1] == d.GROUP_NONE


def test_kat_order(engine):
    b = make_batch([[(1, WR)], [(1, WR)], [(1, RD)]], order=[(1 << 32) | 5, 0, (1 << 32) | 1])
    g, rc, _ = run(engine, b, literal=True)
    assert list(g) == [2, 0, 1]


def test_empty_and_zero_length(engine):
    run(engine, make_batch([]))
    run(engine, make_batch([[], [], []]))
    run(engine, make_batch([[], [(3, WR)], [], [(3, RD)]]))
    run(engine, make_batch([[(7, RD)]]))


@pytest.mark.parametrize("n_keys", [1, 8, 200, 100000])
def test_random_dups_all_types(engine, n_keys):
    rng = np.random.default_rng(n_keys)
    b = random_batch(rng, 3000, 20, n_keys, types=(RD, WR, XP, SCAN), unique=False)
    run(engine, b, literal=True)


def test_random_max_len(engine):
    rng = np.random.default_rng(3)
    run(engine, random_batch(rng, 2000, 64, 5000, types=(RD, WR, XP, SCAN), unique=False))


@pytest.mark.parametrize("theta", [0.0, 0.9, 0.99])
@pytest.mark.parametrize("n", [1, 1000, 65536])
def test_ycsb_index_order(engine, theta, n):
    run(engine, d.gen_ycsb(n_txn=n, zipf_theta=theta, req_per_query=16))


@pytest.mark.parametrize("theta", [0.6, 0.9])
def test_ycsb_c4_order(engine, theta):
    b = d.gen_ycsb(n_txn=65536, zipf_theta=theta, part_cnt=16, chunk_txns=4096, want_home=True)
    b.order = c4_order(b)
    run(engine, b)


def test_random_order_with_ties(engine):
    rng = np.random.default_rng(11)
    b = d.gen_ycsb(n_txn=20000, zipf_theta=0.9, req_per_query=8, table_size=5000)
    b.order = rng.integers(0, 50, size=b.n_txn).astype(np.uint64)  # many equal keys: index order
    run(engine, b)


def test_order_wide_bits(engine):
    # > 32 varying order bits: 64-bit order sort path
    rng = np.random.default_rng(12)
    b = d.gen_ycsb(n_txn=30000, zipf_theta=0.9, req_per_query=8, table_size=20000)
    b.order = rng.integers(0, 2**63, size=b.n_txn, dtype=np.uint64)
    run(engine, b)


def test_wide_keys(engine):
    # canonical TPC-C style keys (table << 56 | key) and random 64-bit keys:
    # more than 32 varying bits -> 64-bit key sort path
    rng = np.random.default_rng(13)
    b = random_batch(rng, 5000, 16, 3000, types=(RD, WR), unique=False)
    tbl = rng.integers(1, 9, size=b.nnz).astype(np.uint64)
    b.keys = (tbl << np.uint64(56)) | (b.keys * np.uint64(0x9E3779B1) & np.uint64((1 << 40) - 1))
    run(engine, b)
    b.keys = rng.integers(0, 2**64 - 1, size=b.nnz, dtype=np.uint64)
    run(engine, b)


def test_single_key_all_txns(engine):
    # one hot row, alternating SH runs and EX: deep group chain
    rng = np.random.default_rng(14)
    txns = [[(42, WR if rng.random() < 0.3 else RD)] for _ in range(20000)]
    run(engine, make_batch(txns))


def test_c4_full_size(engine):
    # C4: 1,048,576 txns x 16 keys, 16 partitions, sequencer order
    b = d.gen_ycsb(n_txn=1 << 20, zipf_theta=0.9, part_cnt=16, chunk_txns=65536, want_home=True)
    b.order = c4_order(b)
    run(engine, b, waves=False)


def test_c4_full_size_waves_and_dispatch(engine):
    # the C4 epoch with wave levels (row_lock.cpp:317-357 grant chains,
    # 49,489 levels: the one-CU walk with its helper workgroups, ~18 ms at this size,
    # DESIGN.md §8) and the dispatch
    # lists built from them (txn_table.cpp:151-176), against the oracle
    b = d.gen_ycsb(n_txn=1 << 20, zipf_theta=0.9, part_cnt=16, chunk_txns=65536, want_home=True)
    b.order = c4_order(b)
    g, rc, w, st = engine.calvin_order_epoch(b, want_group=True, want_wave=True)
    eg, erc, ew = orc.calvin(b)
    w = np.asarray(w).astype(np.uint32)
    assert np.array_equal(np.asarray(g).astype(np.uint32), eg)
    assert np.array_equal(np.asarray(rc), erc)
    assert np.array_equal(w, ew) and st["rounds"] == int(ew.max()) + 1
    print(f"C4 waves: {int(ew.max()) + 1} levels, device {st['device_ms']:.2f} ms")
    off, txn = engine.calvin_dispatch(w, b.order)
    seq = np.argsort(b.order, kind="stable")
    want = seq[np.argsort(w[seq], kind="stable")]
    assert np.array_equal(np.asarray(txn), want.astype(np.uint32))
    counts = np.bincount(w, minlength=int(w.max()) + 1)
    assert np.array_equal(np.diff(np.asarray(off, np.int64)), counts)


def test_device_pointers(engine):
    import torch
    b = d.gen_ycsb(n_txn=50000, zipf_theta=0.9)
    g, rc, _ = run(engine, b)
    db = b.to_torch("cuda:0")
    g2, rc2, w2, st = engine.calvin_order_epoch(db, want_group=True, want_wave=True)
    assert np.array_equal(g2.cpu().numpy().astype(np.uint32)[:b.nnz], g)
    assert np.array_equal(rc2.cpu().numpy()[:b.n_txn], rc)


def test_repeat_deterministic(engine):
    b = d.gen_ycsb(n_txn=100000, zipf_theta=0.99)
    g1, rc1, _ = run(engine, b, waves=False)
    g2, rc2, _, _ = engine.calvin_order_epoch(b, want_group=True, want_wave=False)
    assert np.array_equal(np.asarray(g2), g1) and np.array_equal(np.asarray(rc2), rc1)


@pytest.mark.parametrize("num_wh", [128, 4])
def test_tpcc_calvin(engine, num_wh):
    # canonical TPC-C keys: table id in the top byte, packed to the bits that vary
    b = d.gen_tpcc(n_txn=50000 if num_wh == 4 else 262144, num_wh=num_wh)
    run(engine, b, waves=num_wh == 4)
    if num_wh == 128:  # the sort path by default (the hashed bucket path is slower here)
        _, _, _, st = engine.calvin_order_epoch(b, want_group=True)
        assert st["fallback"] == 0, "TPC-C took the bucket path by default"


# ---------------------------------------------------------------- held prefix
def run_held(engine, b, hk, ha, dev=False):
    """Grant groups / readiness against a pre-seeded lock table vs the literal
    Row_lock replay of (held requests, then the epoch)."""
    bb = b.to_torch("cuda:0") if dev else b
    if dev:
        import torch
        held = (torch.from_numpy(np.ascontiguousarray(hk, np.uint64).view(np.int64)).cuda(),
                torch.from_numpy(np.ascontiguousarray(ha, np.uint8)).cuda())
    else:
        held = (hk, ha)
    g, rc, _, st = engine.calvin_order_epoch(bb, want_group=True, held=held)
    if dev:
        g, rc = g.cpu().numpy(), rc.cpu().numpy()
    eg, erc = orc.calvin_held(b, hk, ha)
    assert np.array_equal(np.asarray(g).astype(np.uint32), eg), "group mismatch"
    assert np.array_equal(np.asarray(rc), erc), "rc mismatch"
    assert st["n_commit"] == int((erc == 0).sum())
    return eg, erc


def test_held_kat(engine):
    # A held EX: a reader waits (group 1).  B held SH: a reader joins (group 0).
    # C held SH with an EX waiter: a reader waits behind it (group 2, no barging).
    A, B, C = 10, 20, 30
    b = make_batch([[(A, RD)], [(B, RD)], [(C, RD)], [(B, WR)]])
    hk = np.array([A, B, C, C], np.uint64)
    ha = np.array([WR, RD, RD, WR], np.uint8)
    eg, erc = run_held(engine, b, hk, ha)
    assert list(eg) == [1, 0, 2, 1]
    assert list(erc) == [3, 0, 3, 3]


@pytest.mark.parametrize("dev", [False, True])
@pytest.mark.parametrize("ordered", [False, True])
def test_held_random(engine, dev, ordered):
    rng = np.random.default_rng(21 + dev + 2 * ordered)
    b = random_batch(rng, 20000, 12, 3000, types=(RD, WR, XP, SCAN), unique=False)
    if ordered:
        b.order = rng.integers(0, 5000, size=b.n_txn).astype(np.uint64)
    h = 4000
    hk = rng.integers(0, 3000, size=h).astype(np.uint64)
    ha = rng.choice(np.array([RD, WR, XP, SCAN], np.uint8), size=h)
    run_held(engine, b, hk, ha, dev=dev)


def test_held_ycsb_full(engine):
    b = d.gen_ycsb(n_txn=1 << 18, zipf_theta=0.9, part_cnt=16, chunk_txns=16384, want_home=True)
    b.order = c4_order(b)
    rng = np.random.default_rng(5)
    # the previous epoch's hot rows are still held (owners + queued writers)
    hot = np.unique(b.keys[: 1 << 14])
    hk = np.repeat(hot[:2000], 2)
    ha = np.tile(np.array([RD, WR], np.uint8), 2000)
    eg, erc = run_held(engine, b, hk, ha)
    _, erc0, _ = orc.calvin(b)
    assert (erc == 0).sum() < (erc0 == 0).sum()  # held rows delay some txns


def test_held_rejects_waves(engine):
    b = make_batch([[(1, RD)]])
    with pytest.raises(d.DccError):
        engine.calvin_order_epoch(b, want_wave=True, held=(np.array([1], np.uint64),
                                                            np.array([WR], np.uint8)))


@pytest.mark.parametrize("sequenced", [False, True])
def test_graph_replay_new_contents(engine, sequenced):
    """Caller-owned outputs: the second epoch of a shape is captured as a HIP
    graph and later ones replay it.  A replay over new batch contents in the
    same buffers (same key bits, then wider keys: a new capture) still
    matches the oracle on every call."""
    import torch
    n = 20000
    seeds = [11, 11, 11, 12, 13]
    b0 = d.gen_ycsb(n_txn=n, zipf_theta=0.9, part_cnt=4, chunk_txns=4096, want_home=True, seed=11)
    if sequenced:
        b0.order = c4_order(b0)
    db = b0.to_torch("cuda:0")
    g_out = torch.empty(b0.nnz, dtype=torch.int32, device="cuda:0")
    rc_out = torch.empty(n, dtype=torch.uint8, device="cuda:0")

    def put(dst, a):  # new contents, same device buffer
        dst.copy_(torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0"))
        torch.cuda.synchronize()  # the engine reads on its own stream

    for i, sd in enumerate(seeds + [14]):
        b = d.gen_ycsb(n_txn=n, zipf_theta=0.9, part_cnt=4, chunk_txns=4096, want_home=True, seed=sd)
        keys = np.asarray(b.keys, np.uint64)
        if i == len(seeds):  # wider keys: more varying bits, a different packing
            keys = keys * np.uint64(1 << 20) + np.uint64(7)
        order = c4_order(b) if sequenced else None
        b = d.EpochBatch(b.offsets, keys, b.acctype, None, None, order, dict(b.meta))
        put(db.keys, keys)
        put(db.acctype, np.asarray(b.acctype))
        if sequenced:
            put(db.order, order)
        g, rc, _, st = engine.calvin_order_epoch(db, want_group=True, out_group=g_out, out_rc=rc_out)
        torch.cuda.synchronize()
        eg, erc, _ = orc.calvin(b)
        assert np.array_equal(g.cpu().numpy().astype(np.uint32), eg), f"groups, call {i}"
        assert np.array_equal(rc.cpu().numpy(), erc), f"readiness, call {i}"
        assert st["n_commit"] == int((erc == 0).sum())


def test_rejects_malformed_batches(engine):
    """The batch validation (offsets monotone and inside the accesses, at most
    MAX_ROW_PER_TXN per txn) rides in the key-bit reduction's launch; a bad
    batch is rejected before any ordering work."""
    b = make_batch([[(1, RD), (2, WR)], [(3, WR)], [(4, RD)]])
    off = np.asarray(b.offsets).copy()
    off[1], off[2] = 3, 2  # not monotone
    with pytest.raises(d.DccError):
        engine.calvin_order_epoch(d.EpochBatch(off, b.keys, b.acctype))
    big = make_batch([[(k + 1, RD) for k in range(70)]])  # > MAX_ROW_PER_TXN
    with pytest.raises(d.DccError):
        engine.calvin_order_epoch(big)
    # the engine still decides a good batch afterwards
    run(engine, random_batch(np.random.default_rng(5), 300, 12, 200), waves=False)
