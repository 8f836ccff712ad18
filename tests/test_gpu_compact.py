"""GPU parity of the compact transfer forms (dcc.h DCC_KEYS_U32,
DCC_ACCTYPE_2BIT, DCC_TN_U32) and pinned host batches (dcc_host_alloc): the
shim's host path moves u32 keys, 2-bit access types and u32 timestamps and
the engine widens them on the device (k_widen), so every decision must equal
the full-width batch's and the oracle's -- OCC with history windows and
commit tn, Calvin grant groups, MaaT, device batches, odd access counts,
unaligned device arrays and a key-sharded context."""
import numpy as np
import pytest

import _oracle as orc
import deneva_amd as d
from deneva_amd import RD, WR
from deneva_amd.engine import pack_acctype
from helpers import make_batch, random_batch

pytestmark = pytest.mark.gpu


def compact_plain(b):
    """The compact form in ordinary (pageable) numpy arrays."""
    at = pack_acctype(b.acctype)
    st = None if b.start_tn is None else np.asarray(b.start_tn, np.uint32)
    ft = None if b.finish_tn is None else np.asarray(b.finish_tn, np.uint32)
    return d.EpochBatch(np.asarray(b.offsets, np.uint32), np.asarray(b.keys, np.uint32), at, st, ft,
                        b.order, {"acctype_2bit": True})


@pytest.mark.parametrize("n", [1, 5, 1001, 65536])
@pytest.mark.parametrize("pinned", [False, True])
def test_occ_compact_matches(engine, n, pinned):
    b = d.gen_ycsb(n_txn=n, zipf_theta=0.9, table_size=1 << 20)
    erc, etn, _ = orc.occ(b)
    cb = engine.compact_host_batch(b) if pinned else compact_plain(b)
    engine.tnc = 0
    rc, tn, _ = engine.occ_validate_epoch(cb, want_tn=True)
    assert np.array_equal(np.asarray(rc), erc)
    assert np.array_equal(np.asarray(tn).astype(np.uint64), etn)


def test_occ_compact_history_windows(engine):
    # u32 TS_CAS windows against a device history (the SHIM config's call)
    rng = np.random.default_rng(8)
    b = random_batch(rng, 30001, 13, 3000, p_write=0.4)  # odd nnz: packed tail byte
    b.start_tn = rng.integers(0, 50, size=b.n_txn).astype(np.uint64)
    b.finish_tn = (b.start_tn + rng.integers(0, 30, size=b.n_txn)).astype(np.uint64)
    hk = rng.integers(0, 3000, size=500).astype(np.uint64)
    ht = rng.integers(1, 80, size=500).astype(np.uint64)
    erc, etn, etnc = orc.occ(b, hist_keys=hk, hist_tn=ht, tnc=80)
    for cb in (engine.compact_host_batch(b), compact_plain(b)):
        engine.history_clear()
        engine.history_append(hk, ht)
        engine.tnc = 80
        try:
            rc, tn, _ = engine.occ_validate_epoch(cb, want_tn=True)
        finally:
            engine.history_clear()
        assert np.array_equal(np.asarray(rc), erc)
        assert np.array_equal(np.asarray(tn).astype(np.uint64), etn)
        assert engine.tnc == etnc


def test_compact_device_batch_unaligned(engine):
    # device arrays in the compact form, sliced so the u32 keys start 4 B past
    # a 16-B boundary and the packed types 1 B past a word (k_widen's scalar path)
    import torch
    b = d.gen_ycsb(n_txn=20000, zipf_theta=0.9, table_size=1 << 18)
    erc, _, _ = orc.occ(b)
    keys = torch.from_numpy(np.concatenate([[7], np.asarray(b.keys, np.uint32)]).astype(np.int32)).cuda()[1:]
    at = torch.from_numpy(np.concatenate([[0], pack_acctype(b.acctype)]).astype(np.uint8)).cuda()[1:]
    off = torch.from_numpy(np.asarray(b.offsets, np.uint32).view(np.int32)).cuda()
    db = d.EpochBatch(off, keys, at, meta={"acctype_2bit": True})
    rc, _, _ = engine.occ_validate_epoch(db)
    torch.cuda.synchronize()
    assert np.array_equal(rc.cpu().numpy(), erc)


def test_calvin_and_maat_compact(engine):
    c = d.gen_ycsb(n_txn=40000, zipf_theta=0.9, part_cnt=4, chunk_txns=4096)
    c.order = np.random.default_rng(2).integers(0, 1 << 20, size=c.n_txn).astype(np.uint64)
    eg, erc, _ = orc.calvin(c)
    cc = engine.compact_host_batch(c)
    g, rc, _, _ = engine.calvin_order_epoch(cc, want_group=True)
    assert np.array_equal(np.asarray(g).astype(np.uint32), eg)
    assert np.array_equal(np.asarray(rc), erc)
    m = d.gen_ycsb(n_txn=20000, zipf_theta=0.9)
    mrc, mcts, _ = orc.maat(m)
    engine.maat_rows_clear()
    rc, cts, _ = engine.maat_validate_epoch(engine.compact_host_batch(m))
    engine.maat_rows_clear()
    assert np.array_equal(np.asarray(rc), mrc)
    assert np.array_equal(np.asarray(cts).astype(np.uint64), mcts)


def test_sharded_context_compact(engine):
    b = d.gen_ycsb(n_txn=50000, zipf_theta=0.99, table_size=1 << 18)
    erc, etn, _ = orc.occ(b)
    with d.Engine(devices=[0, 0, 0]) as m:
        m.tnc = 0
        rc, tn, _ = m.occ_validate_epoch(m.compact_host_batch(b), want_tn=True)
        assert np.array_equal(np.asarray(rc), erc)
        assert np.array_equal(np.asarray(tn).astype(np.uint64), etn)


def test_host_offsets_checked_on_device(engine):
    # the sweep skips the host scan of a host batch's offsets: a decrease in
    # the middle (first and last offsets valid) is rejected by the device pass
    b = make_batch([[(i, WR), (i + 1, RD)] for i in range(5000)])
    off = np.asarray(b.offsets, np.uint32).copy()
    off[2500] = off[2499] - 1
    bad = d.EpochBatch(off, b.keys, b.acctype)
    with pytest.raises(d.DccError) as e:
        engine.occ_validate_epoch(bad)
    assert e.value.code == -22
    rc, _, _ = engine.occ_validate_epoch(b)  # usable afterwards
    assert np.array_equal(np.asarray(rc), orc.occ(b)[0])
