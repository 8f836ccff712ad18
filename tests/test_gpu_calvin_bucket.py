"""GPU parity of the Calvin bucket path (calvin_bucket.hip: one stable
partition of the sequence-order requests into key buckets, then per bucket an
LDS sort + grant-group scan with each row's state carried from chunk to chunk,
and the windowed group write-out with readiness) against the oracle
(`orc.calvin`, the Row_lock CALVIN replay restated: row_lock.cpp:78-81,
152-170, 317-357).  DCC_OPT_CALVIN_PATH=2 takes the path at every size it applies
to (txn lengths <= 64, uniform or ragged, packed keys <= 28 bits -- past 24
the carry table is hashed on the row bits, TPC-C's canonical keys among
them); the cases cover one-row
buckets, a single key, duplicates of a row inside a txn (also where a txn
straddles a chunk boundary), hot rows spanning many chunks, sequencer orders
with ties, txn lengths 1..64, ragged txns (random lengths with empty txns, a
key-sharded rank's share of C4), 25- to 28-bit keys and TPC-C on the hashed
carry table, a bucket with more rows than that table holds (the epoch is
redone on the sort path), and the fallback for wider keys."""
import numpy as np
import pytest

import _oracle as orc
import deneva_amd as d
from deneva_amd import RD, WR, XP, SCAN
from helpers import c4_batch

pytestmark = pytest.mark.gpu


@pytest.fixture
def bucket(engine):
    engine.set_option(d._abi.OPT_CALVIN_PATH, 2)
    yield
    engine.set_option(d._abi.OPT_CALVIN_PATH, 0)


def uniform_batch(rng, n, L, n_keys, p_write=0.5, types=None, order=False, zipf=None):
    if zipf:
        keys = (rng.zipf(zipf, size=n * L) - 1) % n_keys
    else:
        keys = rng.integers(0, n_keys, size=n * L)
    if types:
        at = rng.choice(np.asarray(types, np.uint8), size=n * L)
    else:
        at = np.where(rng.random(n * L) < p_write, WR, RD).astype(np.uint8)
    off = (np.arange(n + 1) * L).astype(np.uint32)
    od = rng.integers(0, max(2, n // 4), size=n).astype(np.uint64) if order else None
    return d.EpochBatch(off, keys.astype(np.uint64), at, None, None, od)


def check(engine, b):
    g, rc, _, st = engine.calvin_order_epoch(b, want_group=True)
    eg, erc, _ = orc.calvin(b)
    g = np.asarray(g).astype(np.uint32)
    bad = np.nonzero(g != eg)[0]
    assert bad.size == 0, f"group mismatch at {bad[:8]}: gpu {g[bad[:8]]} oracle {eg[bad[:8]]}"
    bad = np.nonzero(np.asarray(rc) != erc)[0]
    assert bad.size == 0, f"rc mismatch at txns {bad[:8]}"
    assert st["n_commit"] == int((erc == 0).sum())
    return g


@pytest.mark.parametrize("n,L,n_keys,order", [
    (1, 1, 1, False), (5, 3, 7, True), (3000, 16, 1, False), (3000, 16, 8, True),
    (5000, 10, 200, True), (20000, 64, 5000, False), (40000, 1, 300, True),
    (20000, 8, 1 << 24, True), (30000, 16, 1 << 16, False), (12345, 7, 1 << 20, True)])
def test_uniform_random(engine, bucket, n, L, n_keys, order):
    rng = np.random.default_rng(n + L)
    check(engine, uniform_batch(rng, n, L, n_keys, types=(RD, WR, XP, SCAN), order=order))


def ragged_batch(rng, n, maxlen, n_keys, order=False, zipf=None, p_empty=0.05):
    lens = rng.integers(1, maxlen + 1, size=n)
    lens[rng.random(n) < p_empty] = 0
    off = np.zeros(n + 1, np.uint32)
    off[1:] = np.cumsum(lens)
    m = int(off[-1])
    keys = ((rng.zipf(zipf, size=m) - 1) % n_keys) if zipf else rng.integers(0, n_keys, size=m)
    at = rng.choice(np.array([RD, WR, XP, SCAN], np.uint8), size=m, p=[0.5, 0.3, 0.1, 0.1])
    od = rng.integers(0, max(2, n // 4), size=n).astype(np.uint64) if order else None
    return d.EpochBatch(off, keys.astype(np.uint64), at, None, None, od)


@pytest.mark.parametrize("n,maxlen,n_keys,order", [
    (7, 3, 5, True), (3000, 64, 50, False), (20000, 17, 4096, True), (50000, 5, 1 << 18, True),
    (40000, 2, 300, False), (30000, 40, 1 << 22, True), (100000, 9, 1 << 20, False)])
def test_ragged_random(engine, bucket, n, maxlen, n_keys, order):
    # ragged txns take the bucket path too (element -> request map per wave,
    # offsets staged per output window)
    rng = np.random.default_rng(n * 7 + maxlen)
    b = ragged_batch(rng, n, maxlen, n_keys, order=order, zipf=1.2 if n_keys > 1000 else None)
    g, rc, _, st = engine.calvin_order_epoch(b, want_group=True)
    assert st["fallback"] == 1, "the ragged epoch did not take the bucket path"
    check(engine, b)


def test_ragged_key_shard_of_c4(engine):
    # one key shard's share of a sequenced YCSB epoch (what a key-sharded rank
    # of C4 orders: 2 requests per txn on average, empty txns common) at 8
    # shards, with the default path choice (the bucket path from 2^21 requests)
    b = d.gen_ycsb(n_txn=1 << 20, zipf_theta=0.9, part_cnt=16, chunk_txns=4096, want_home=True)
    home = b.meta["home"].astype(np.uint64)
    seq = np.zeros(b.n_txn, np.uint64)
    for h in np.unique(home):
        idx = np.nonzero(home == h)[0]
        seq[idx] = np.arange(idx.size, dtype=np.uint64)
    keys = np.asarray(b.keys, np.uint64)
    keep = np.asarray(d.shard_of_keys(keys, 8)) == 3
    off = np.asarray(b.offsets, np.int64)
    own = np.repeat(np.arange(b.n_txn), np.diff(off))
    cnt = np.bincount(own[keep], minlength=b.n_txn)
    noff = np.zeros(b.n_txn + 1, np.uint32)
    noff[1:] = np.cumsum(cnt)
    sb = d.EpochBatch(noff, keys[keep], np.asarray(b.acctype)[keep], None, None,
                      (home << np.uint64(32)) | seq)
    engine.set_option(d._abi.OPT_CALVIN_PATH, 2)
    try:
        _, _, _, st = engine.calvin_order_epoch(sb, want_group=True)
        assert st["fallback"] == 1
        check(engine, sb)
    finally:
        engine.set_option(d._abi.OPT_CALVIN_PATH, 0)


def test_chunk_straddling_duplicates(engine, bucket):
    # 64 rows (one-row buckets of ~5,000 requests: two chunks each), 16
    # requests per txn drawn with repeats: a txn often holds a row twice, also
    # across the 4,096-request chunk boundary
    rng = np.random.default_rng(5)
    check(engine, uniform_batch(rng, 20000, 16, 64, types=(RD, WR, XP, SCAN), order=True))
    # the same with row bits inside the bucket (4,096 rows: 2 rows per bucket)
    check(engine, uniform_batch(rng, 60000, 16, 4096, types=(RD, WR), order=True))


@pytest.mark.parametrize("n,L,nrow", [(40000, 2, 200), (20000, 4, 64), (30000, 3, 500)])
def test_rows_of_one_class(engine, bucket, n, L, nrow):
    # every row in bucket 0 and row class 0 (keys i * 8192 with all 21 low
    # bits varying): rows go untouched for whole 64-request rounds while txns
    # straddle the round boundaries -- the carry table's one-round "same txn"
    # flag must not outlive its round
    rng = np.random.default_rng(n + nrow)
    keys = rng.choice(np.arange(nrow, dtype=np.uint64) * np.uint64(8192), size=n * L)
    keys[0] = (1 << 21) - 1
    at = rng.choice(np.array([RD, WR, SCAN, XP], np.uint8), size=n * L, p=[0.6, 0.2, 0.1, 0.1])
    od = rng.integers(0, n // 8, size=n).astype(np.uint64)
    check(engine, d.EpochBatch((np.arange(n + 1) * L).astype(np.uint32), keys, at, None, None, od))


def test_single_hot_row(engine, bucket):
    rng = np.random.default_rng(14)
    at = np.where(rng.random(20000) < 0.3, WR, RD).astype(np.uint8)
    b = d.EpochBatch(np.arange(20001, dtype=np.uint32), np.full(20000, 42, np.uint64), at)
    check(engine, b)


@pytest.mark.parametrize("theta", [0.9, 0.99])
@pytest.mark.parametrize("n", [65536, 262144])
def test_ycsb_sequenced(engine, bucket, theta, n):
    # zipf hot rows: buckets of many chunks, rows spanning chunks
    b = d.gen_ycsb(n_txn=n, zipf_theta=theta, part_cnt=16, chunk_txns=4096, want_home=True)
    home = b.meta["home"].astype(np.uint64)
    seq = np.zeros(b.n_txn, np.uint64)
    for h in np.unique(home):
        idx = np.nonzero(home == h)[0]
        seq[idx] = np.arange(idx.size, dtype=np.uint64)
    b.order = (home << np.uint64(32)) | seq
    check(engine, b)


def test_zipf_hot_rows_with_row_bits(engine, bucket):
    rng = np.random.default_rng(21)
    check(engine, uniform_batch(rng, 100000, 16, 1 << 20, zipf=1.3, order=True))


def test_wide_keys_fall_back(engine, bucket):
    rng = np.random.default_rng(22)
    check(engine, uniform_batch(rng, 5000, 16, 1 << 30, order=True))


def test_paths_agree_c4(engine):
    # C4 (1,048,576 x 16): the bucket path (the default at this size) and the
    # global sort + scan produce the same groups and readiness
    b = c4_batch()
    engine.set_option(d._abi.OPT_CALVIN_PATH, 1)
    try:
        g0, rc0, _, _ = engine.calvin_order_epoch(b, want_group=True)
    finally:
        engine.set_option(d._abi.OPT_CALVIN_PATH, 0)
    engine.set_option(d._abi.OPT_CALVIN_PATH, 2)
    try:
        g1, rc1, _, _ = engine.calvin_order_epoch(b, want_group=True)
    finally:
        engine.set_option(d._abi.OPT_CALVIN_PATH, 0)
    assert np.array_equal(np.asarray(g0), np.asarray(g1))
    assert np.array_equal(np.asarray(rc0), np.asarray(rc1))


def test_graph_replay(engine, bucket):
    """The bucket path inside the captured graph: repeated epochs of one shape
    over new contents in the same device buffers."""
    import torch
    n = 30000
    b0 = d.gen_ycsb(n_txn=n, zipf_theta=0.9, part_cnt=4, chunk_txns=4096, seed=3)
    db = b0.to_torch("cuda:0")
    g_out = torch.empty(b0.nnz, dtype=torch.int32, device="cuda:0")
    rc_out = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    for i, sd in enumerate([3, 3, 4, 5, 6]):
        b = d.gen_ycsb(n_txn=n, zipf_theta=0.9, part_cnt=4, chunk_txns=4096, seed=sd)
        db.keys.copy_(torch.from_numpy(np.ascontiguousarray(b.keys)).to("cuda:0"))
        db.acctype.copy_(torch.from_numpy(np.ascontiguousarray(b.acctype)).to("cuda:0"))
        torch.cuda.synchronize()  # the engine reads on its own stream
        g, rc, _, _ = engine.calvin_order_epoch(db, want_group=True, out_group=g_out, out_rc=rc_out)
        torch.cuda.synchronize()
        eg, erc, _ = orc.calvin(b)
        assert np.array_equal(g.cpu().numpy().astype(np.uint32), eg), f"groups, call {i}"
        assert np.array_equal(rc.cpu().numpy(), erc), f"readiness, call {i}"


def test_sorted_order_skips_rank_and_matches(engine):
    """A sequencer hands its epoch over origin by origin in FIFO order, so the
    order is non-decreasing in index order (ties included): the engine ranks
    it as the identity without sorting.  The same txns with the order shuffled
    take the rank sort; both equal the Row_lock replay."""
    rng = np.random.default_rng(41)
    b = uniform_batch(rng, 60000, 16, 1 << 14, zipf=1.3)
    b.order = np.sort(rng.integers(0, 3000, size=b.n_txn)).astype(np.uint64)  # ties
    check(engine, b)
    b.order = rng.permutation(b.order)
    check(engine, b)


def test_speculative_replay_and_miss(engine):
    """The bucket-path graph of a shape is launched right behind the prep on
    the packing it was captured with; the host checks it afterwards and redoes
    the epoch when the key universe changed (here: a key with a new high bit),
    and a malformed batch is still rejected."""
    import torch
    n = 1 << 17
    dev = "cuda:0"
    kw = dict(n_txn=n, zipf_theta=0.9, part_cnt=16, chunk_txns=8192, table_size=1 << 18, want_home=True)
    b0 = d.gen_ycsb(seed=5, **kw)
    db = b0.to_torch(dev)
    g_out = torch.empty(b0.nnz, dtype=torch.int32, device=dev)
    rc_out = torch.empty(n, dtype=torch.uint8, device=dev)
    engine.set_option(d._abi.OPT_CALVIN_PATH, 2)
    try:
        for i, mutate in enumerate([None, None, None, "seed", "highbit", None, "highbit"]):
            b = d.gen_ycsb(seed=5 if mutate is None else 6, **kw)
            keys = np.asarray(b.keys, np.uint64).copy()
            if mutate == "highbit":
                keys[12345] |= np.uint64(1 << 21)  # a new packed bit (still <= 24)
            b.keys = keys
            db.keys.copy_(torch.from_numpy(keys.view(np.int64)).to(dev))
            db.acctype.copy_(torch.from_numpy(np.ascontiguousarray(b.acctype)).to(dev))
            torch.cuda.synchronize()  # the engine reads on its own stream
            g, rc, _, st = engine.calvin_order_epoch(db, want_group=True, out_group=g_out, out_rc=rc_out)
            torch.cuda.synchronize()
            eg, erc, _ = orc.calvin(b)
            assert st["fallback"] == 1, "bucket path"
            assert np.array_equal(g.cpu().numpy().astype(np.uint32), eg), f"groups, epoch {i}"
            assert np.array_equal(rc.cpu().numpy(), erc), f"readiness, epoch {i}"
        off = np.asarray(b0.offsets, np.uint32).copy()
        off[7] = off[8] + 1  # offsets decrease
        bad = d.EpochBatch(torch.from_numpy(off).to(dev), db.keys, db.acctype)
        with pytest.raises(d.DccError):
            engine.calvin_order_epoch(bad, want_group=True, out_group=g_out, out_rc=rc_out)
    finally:
        engine.set_option(d._abi.OPT_CALVIN_PATH, 0)


def test_c4_interleaved_origins_full_size(engine):
    # C4 captured with its 16 origins interleaved (txn i from origin i % 16):
    # the order must be ranked before the bucket path
    b = c4_batch()
    home = (np.arange(b.n_txn) % 16).astype(np.uint64)
    b.order = (home << np.uint64(32)) | (np.arange(b.n_txn, dtype=np.uint64) // np.uint64(16))
    g, rc, _, st = engine.calvin_order_epoch(b, want_group=True)
    eg, erc, _ = orc.calvin(b)
    assert st["fallback"] == 1
    assert np.array_equal(np.asarray(g).astype(np.uint32), eg)
    assert np.array_equal(np.asarray(rc), erc)


@pytest.mark.parametrize("n,L,kbits,order", [(20000, 16, 25, True), (30000, 8, 26, False),
                                             (50000, 16, 28, True), (4000, 64, 27, True)])
def test_hashed_carry_table(engine, bucket, n, L, kbits, order):
    """Packed keys of 25-28 bits: row bits 14-17 above the 11 bucket bits,
    the carry table hashed on them."""
    rng = np.random.default_rng(kbits * 7 + L)
    b = uniform_batch(rng, n, L, 1 << kbits, order=order)
    b.keys[0] = (1 << kbits) - 1  # every bit varies: the packing keeps kbits
    b.keys[1] = 0
    check(engine, b)
    _, _, _, st = engine.calvin_order_epoch(b, want_group=True)
    assert st["fallback"] == 1, "not on the bucket path"


@pytest.mark.parametrize("num_wh,n", [(4, 50000), (128, 262144)])
def test_tpcc_on_bucket_path(engine, bucket, num_wh, n):
    """Canonical TPC-C keys (28 bits packed at 128 warehouses, ragged
    NewOrder / Payment txns) on the bucket path with the hashed carry table."""
    b = d.gen_tpcc(n_txn=n, num_wh=num_wh)
    check(engine, b)
    _, _, _, st = engine.calvin_order_epoch(b, want_group=True)
    assert st["fallback"] == 1, "not on the bucket path"


def test_hashed_table_overflow_redoes_on_sort_path():
    """20,000 rows in one bucket (more than the 8,192-slot hashed table): the
    epoch is redone on the sort path, exactly, and the context keeps the sort
    path for such epochs (a fresh context: the switch is per context)."""
    eng = d.Engine(0)
    eng.set_option(d._abi.OPT_CALVIN_PATH, 2)
    rng = np.random.default_rng(33)
    n, L = 20000, 4
    rows = rng.permutation(1 << 15)[: n * L // 2].astype(np.uint64)
    keys = np.concatenate([(rows << np.uint64(11)) | np.uint64(5),
                           rng.integers(0, 1 << 26, size=n * L - rows.size).astype(np.uint64)])
    keys[-1] = (1 << 26) - 1  # 26 varying bits: hashed
    keys[-2] = 0
    at = np.where(rng.random(n * L) < 0.5, WR, RD).astype(np.uint8)
    off = (np.arange(n + 1) * L).astype(np.uint32)
    b = d.EpochBatch(off, keys, at)
    check(eng, b)
    _, _, _, st = eng.calvin_order_epoch(b, want_group=True)
    assert st["fallback"] == 0, "the overflowing epoch should end on the sort path"
