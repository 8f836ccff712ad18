"""GPU index probe and Calvin wave dispatch lists.

Index: restated IndexHash semantics (index_hash.cpp:58-231) — a key inserted
more than once reads as its newest insert, a missing key is DCC_ROW_NONE.
Dispatch: the txns of each wave in sequence order, against a stable numpy
sort of the oracle's wave levels."""
import numpy as np
import pytest

import _oracle as orc
import deneva_amd as d
from deneva_amd._abi import ROW_NONE

pytestmark = pytest.mark.gpu


def index_oracle(inserts, probe):
    """BucketHeader::insert_item / read_item: the newest item of a key."""
    m = {}
    for keys, rows in inserts:
        for k, r in zip(keys.tolist(), rows.tolist()):
            m[k] = r
    return np.array([m.get(k, ROW_NONE) for k in probe.tolist()], np.uint64)


def test_index_build_probe_duplicates_growth():
    rng = np.random.default_rng(1)
    with d.Engine(0) as eng:
        inserts = []
        for step in range(4):  # appends with duplicates inside and across steps
            k = rng.integers(0, 300000, size=120000).astype(np.uint64)
            r = rng.integers(0, 1 << 40, size=k.size).astype(np.uint64)
            eng.index_insert(k, r)
            inserts.append((k, r))
        probe = rng.integers(0, 400000, size=500000).astype(np.uint64)
        got, miss = eng.index_probe(probe)
        want = index_oracle(inserts, probe)
        assert np.array_equal(got, want)
        assert miss == int((want == ROW_NONE).sum())
        assert eng.index_size == len(np.unique(np.concatenate([k for k, _ in inserts])))


def test_index_probe_epoch_device():
    """Every access of a resident 1M-txn YCSB epoch (16M probes)."""
    import torch
    b = d.gen_ycsb(n_txn=1 << 20, zipf_theta=0.9)
    table = np.arange(1 << 24, dtype=np.uint64)
    rows = table * 7 + 3  # row id of each key (the table's item location)
    with d.Engine(0) as eng:
        eng.index_insert(table, rows)
        dk = torch.from_numpy(np.asarray(b.keys).view(np.int64)).cuda()
        out, miss = eng.index_probe(dk)
        torch.cuda.synchronize()
        assert miss == 0
        assert np.array_equal(out.cpu().numpy().view(np.uint64), np.asarray(b.keys) * 7 + 3)
        assert eng.index_last_ms > 0


@pytest.mark.parametrize("ordered", [False, True])
def test_dispatch_lists(engine, ordered):
    rng = np.random.default_rng(7)
    b = d.gen_ycsb(n_txn=20000, zipf_theta=0.8, table_size=1 << 14)
    if ordered:
        b.order = rng.integers(0, 4000, size=b.n_txn).astype(np.uint64)
    _, _, w, _ = engine.calvin_order_epoch(b, want_group=False, want_wave=True)
    _, _, ew = orc.calvin(b)
    assert np.array_equal(np.asarray(w).astype(np.uint32), ew)
    off, txn = engine.calvin_dispatch(np.asarray(w), b.order)
    seq = np.arange(b.n_txn) if b.order is None else np.argsort(b.order, kind="stable")
    want = seq[np.argsort(ew[seq], kind="stable")]
    assert np.array_equal(np.asarray(txn), want.astype(np.uint32))
    counts = np.bincount(ew, minlength=int(ew.max()) + 1)
    assert np.array_equal(np.diff(np.asarray(off, np.int64)), counts)
    # every txn of wave w+1 has a predecessor in wave w (the schedule is tight)
    assert off[0] == 0 and off[-1] == b.n_txn


def test_repeated_host_calls_keep_memory_flat():
    """Probe and dispatch with host pointers stage through the context's
    grow-only scratch: after the first call, repeated calls allocate nothing
    (device free memory stays flat)."""
    import torch
    rng = np.random.default_rng(9)
    with d.Engine(0) as eng:
        k = rng.integers(0, 1 << 20, size=200000).astype(np.uint64)
        eng.index_insert(k, k * 3)
        probe = rng.integers(0, 1 << 21, size=1 << 20).astype(np.uint64)
        wave = rng.integers(0, 500, size=1 << 18).astype(np.uint32)
        order = rng.permutation(wave.size).astype(np.uint64)
        eng.index_probe(probe)
        eng.calvin_dispatch(wave, order)
        torch.cuda.synchronize()
        free0 = torch.cuda.mem_get_info(0)[0]
        for _ in range(40):
            eng.index_probe(probe)
            eng.calvin_dispatch(wave, order)
            eng.index_insert(k[:1000], k[:1000])
        torch.cuda.synchronize()
        free1 = torch.cuda.mem_get_info(0)[0]
        # 40 leaked probe buffers alone would be 40 x 16 MiB
        assert free0 - free1 < (8 << 20), (free0, free1)
