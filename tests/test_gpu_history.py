"""Device-resident OCC history (occ_history.h): epochs append their committed
write sets on the device (central_finish, occ.cpp:277-286) and later epochs'
history windows (occ.cpp:160-180) see them.  Checked against the oracle with
the history accumulated on the host from the oracle's own commit tns."""
import numpy as np
import pytest

import _oracle as orc
import deneva_amd as d
from deneva_amd import WR
from deneva_amd._abi import OPT_HIST_MERGE
from helpers import random_batch

pytestmark = pytest.mark.gpu


def committed_writes(b, tn):
    """(key, tn) of every write of a txn with a commit tn (central_finish)."""
    off = np.asarray(b.offsets, np.int64)
    at = np.asarray(b.acctype)
    keys = np.asarray(b.keys, np.uint64)
    lens = np.diff(off)
    owner = np.repeat(np.arange(b.n_txn), lens)
    sel = (at == WR) & (np.asarray(tn)[owner] != 0)
    return keys[sel], np.asarray(tn, np.uint64)[owner[sel]]


def windows(rng, n, tnc, spread):
    """TS_CAS-like windows straddling the commit counter."""
    st = (tnc - rng.integers(0, spread, size=n)).clip(0).astype(np.uint64)
    ft = (st + rng.integers(0, 2 * spread, size=n)).astype(np.uint64)
    return st, ft


def sorted_pairs(k, t):
    k = np.asarray(k, np.uint64)
    t = np.asarray(t, np.uint64)
    o = np.lexsort((t, k))
    return k[o], t[o]


@pytest.mark.parametrize("device_ptrs", [False, True])
@pytest.mark.parametrize("merge_min", [500, 65536])
def test_many_epochs(engine, device_ptrs, merge_min):
    import torch
    rng = np.random.default_rng(11 + merge_min + device_ptrs)
    engine.history_clear()
    engine.tnc = 0
    engine.set_option(OPT_HIST_MERGE, merge_min)
    hk = np.zeros(0, np.uint64)
    ht = np.zeros(0, np.uint64)
    tnc = 0
    try:
        for e in range(6):
            b = d.gen_ycsb(n_txn=20000, zipf_theta=0.6, table_size=1 << 16, seed=100 + e)
            b.start_tn, b.finish_tn = windows(rng, b.n_txn, tnc, 400)
            erc, etn, etnc = orc.occ(b, hist_keys=hk, hist_tn=ht, tnc=tnc)
            bb = b.to_torch("cuda:0") if device_ptrs else b
            rc, tn, st = engine.occ_validate_epoch(bb, want_tn=True, append_history=True)
            if device_ptrs:
                torch.cuda.synchronize()
                rc = rc.cpu().numpy()
                tn = tn.cpu().numpy().view(np.uint64)
            assert np.array_equal(rc, erc), f"epoch {e}: rc differs"
            assert np.array_equal(np.asarray(tn, np.uint64), etn), f"epoch {e}: tn differs"
            assert engine.tnc == etnc
            nk, nt = committed_writes(b, etn)
            hk = np.concatenate([hk, nk])
            ht = np.concatenate([ht, nt])
            tnc = etnc
            assert engine.history_size == hk.size
        gk, gt = engine.history_export()
        wk, wt = sorted_pairs(hk, ht)
        assert np.array_equal(gk, wk) and np.array_equal(gt, wt)
    finally:
        engine.set_option(OPT_HIST_MERGE, 65536)
        engine.history_clear()


@pytest.mark.parametrize("device_ptrs", [False, True])
def test_appends_of_handed_off_epochs(engine, device_ptrs):
    """Low-contention epochs (theta 0) whose lists stop shrinking go to the
    round solver after the captured graph ran: central_finish runs a second
    time on the fully decided epoch (a fresh look-back tag), and the delta's
    chains pushed by the first, partly decided run are dropped (the level is
    rebuilt from the flat pairs).  Every later window must see exactly the
    oracle's history; the second and third passes replay the graph."""
    import torch
    rng = np.random.default_rng(0x4AD0 + device_ptrs)
    engine.set_option(OPT_HIST_MERGE, 1 << 22)  # keep everything in the delta
    bs = [d.gen_ycsb(n_txn=65536, zipf_theta=0.0, table_size=1 << 18, seed=0x4AD0 + e) for e in range(3)]
    try:
        for rep in range(3):
            engine.history_clear()
            engine.tnc = 0
            hk = np.zeros(0, np.uint64)
            ht = np.zeros(0, np.uint64)
            tnc = 0
            for e, b in enumerate(bs):
                b.start_tn, b.finish_tn = windows(np.random.default_rng(e), b.n_txn, tnc, 30000)
                erc, etn, etnc = orc.occ(b, hist_keys=hk, hist_tn=ht, tnc=tnc)
                bb = b.to_torch("cuda:0") if device_ptrs else b
                rc, tn, st = engine.occ_validate_epoch(bb, want_tn=True, append_history=True)
                if device_ptrs:
                    torch.cuda.synchronize()
                    rc = rc.cpu().numpy()
                    tn = tn.cpu().numpy().view(np.uint64)
                assert np.array_equal(rc, erc), f"pass {rep} epoch {e}: rc differs"
                assert np.array_equal(np.asarray(tn, np.uint64), etn), f"pass {rep} epoch {e}: tn differs"
                nk, nt = committed_writes(b, etn)
                hk = np.concatenate([hk, nk])
                ht = np.concatenate([ht, nt])
                tnc = etnc
            gk, gt = engine.history_export()
            wk, wt = sorted_pairs(hk, ht)
            assert np.array_equal(gk, wk) and np.array_equal(gt, wt)
    finally:
        engine.set_option(OPT_HIST_MERGE, 65536)
        engine.history_clear()
        engine.tnc = 0


def test_out_of_order_appends(engine):
    """Host appends with tns below earlier ones: levels re-sorted by (key, tn)."""
    rng = np.random.default_rng(5)
    engine.history_clear()
    engine.set_option(OPT_HIST_MERGE, 300)
    try:
        hk, ht = [], []
        for _ in range(8):
            k = rng.integers(0, 200, size=250).astype(np.uint64)
            t = rng.integers(1, 5000, size=250).astype(np.uint64)
            engine.history_append(k, t)
            hk.append(k)
            ht.append(t)
            hk_a, ht_a = np.concatenate(hk), np.concatenate(ht)
            b = random_batch(rng, 3000, 10, 200, p_write=0.3)
            b.start_tn = rng.integers(0, 5000, size=b.n_txn).astype(np.uint64)
            b.finish_tn = (b.start_tn + rng.integers(0, 300, size=b.n_txn)).astype(np.uint64)
            engine.tnc = 5000
            rc, tn, _ = engine.occ_validate_epoch(b, want_tn=True)
            erc, etn, _ = orc.occ(b, hist_keys=hk_a, hist_tn=ht_a, tnc=5000)
            assert np.array_equal(np.asarray(rc), erc)
            assert np.array_equal(np.asarray(tn, np.uint64), etn)
        gk, gt = engine.history_export()
        wk, wt = sorted_pairs(np.concatenate(hk), np.concatenate(ht))
        assert np.array_equal(gk, wk) and np.array_equal(gt, wt)
    finally:
        engine.set_option(OPT_HIST_MERGE, 65536)
        engine.history_clear()


def test_trim(engine):
    """dcc_occ_history_trim drops tn <= floor; windows opening at or after the
    floor decide exactly as with the whole history."""
    rng = np.random.default_rng(6)
    engine.history_clear()
    k = rng.integers(0, 300, size=3000).astype(np.uint64)
    t = rng.integers(1, 2000, size=3000).astype(np.uint64)
    engine.history_append(k, t)
    floor = 1200
    engine.history_trim(floor)
    keep = t > floor
    gk, gt = engine.history_export()
    wk, wt = sorted_pairs(k[keep], t[keep])
    assert np.array_equal(gk, wk) and np.array_equal(gt, wt)
    assert engine.history_size == int(keep.sum())
    b = random_batch(rng, 4000, 8, 300, p_write=0.4)
    b.start_tn = rng.integers(floor, 2000, size=b.n_txn).astype(np.uint64)
    b.finish_tn = (b.start_tn + rng.integers(0, 200, size=b.n_txn)).astype(np.uint64)
    engine.tnc = 2000
    rc, _, _ = engine.occ_validate_epoch(b, want_tn=True)
    erc, _, _ = orc.occ(b, hist_keys=k, hist_tn=t, tnc=2000)
    assert np.array_equal(np.asarray(rc), erc)
    # then appends continue on top of the trimmed base
    rc2, tn2, _ = engine.occ_validate_epoch(b, want_tn=True, append_history=True)
    nk, nt = committed_writes(b, np.asarray(tn2, np.uint64))
    gk, gt = engine.history_export()
    wk, wt = sorted_pairs(np.concatenate([k[keep], nk]), np.concatenate([t[keep], nt]))
    assert np.array_equal(gk, wk) and np.array_equal(gt, wt)
    engine.history_clear()


def test_snapshot_sees_epoch_history(engine):
    """Captured-snapshot validation reads the same device history levels."""
    rng = np.random.default_rng(8)
    engine.history_clear()
    engine.tnc = 0
    b1 = random_batch(rng, 3000, 8, 500, p_write=0.5)
    _, tn1, _ = engine.occ_validate_epoch(b1, want_tn=True, append_history=True)
    hk, ht = committed_writes(b1, np.asarray(tn1, np.uint64))
    b2 = random_batch(rng, 2000, 8, 500, p_write=0.5)
    n = b2.n_txn
    b2.start_tn = rng.integers(0, int(engine.tnc) + 1, size=n).astype(np.uint64)
    b2.finish_tn = (b2.start_tn + rng.integers(0, 50, size=n)).astype(np.uint64)
    aoff = np.zeros(n + 1, np.uint32)
    top = rng.integers(0, int(engine.tnc) + 1, size=n).astype(np.uint64)
    rc, _ = engine.occ_validate_snapshot(b2, aoff, np.zeros(1, np.uint32), top)
    want = orc.occ_snapshot(b2, aoff, np.zeros(0, np.uint32), top, hk, ht)
    assert np.array_equal(np.asarray(rc), want)
    engine.history_clear()


@pytest.mark.parametrize("device_ptrs", [False, True])
def test_failed_append_retry_then_window(engine, device_ptrs):
    """central_finish pushes an epoch's pairs onto the delta's chains before
    the host checks the epoch.  An epoch that fails afterwards (one txn holds
    the reserved key: rejected with DCC_EINVAL once the epoch ran) must leave
    no trace: tnc and the history stay as they were, the retry without that
    txn pushes the same flat positions again, and the windows of the epoch
    after it -- reaching below the retried epoch's tns, so they walk the
    chains -- decide exactly as the oracle (a pair pushed twice
    linked to itself and the walk never ended)."""
    import torch
    rng = np.random.default_rng(0xFA11 + device_ptrs)
    engine.history_clear()
    engine.tnc = 0
    engine.set_option(OPT_HIST_MERGE, 1 << 22)  # every append stays in the chained delta
    try:
        hk, ht = np.zeros(0, np.uint64), np.zeros(0, np.uint64)
        tnc = 0
        as_dev = (lambda b: b.to_torch("cuda:0")) if device_ptrs else (lambda b: b)
        for e in range(4):
            b = d.gen_ycsb(n_txn=20000, zipf_theta=0.8, table_size=1 << 12, seed=0xFA00 + e)
            b.start_tn, b.finish_tn = windows(rng, b.n_txn, tnc, 3000)
            if e == 2:
                bad = d.EpochBatch(b.offsets, np.asarray(b.keys, np.uint64).copy(), b.acctype,
                                   b.start_tn, b.finish_tn)
                bad.keys[-1] = d.KEY_RESERVED
                with pytest.raises(d.DccError):
                    engine.occ_validate_epoch(as_dev(bad), want_tn=True, append_history=True)
                if device_ptrs:
                    torch.cuda.synchronize()
                assert engine.tnc == tnc and engine.history_size == hk.size
            erc, etn, etnc = orc.occ(b, hist_keys=hk, hist_tn=ht, tnc=tnc)
            rc, tn, _ = engine.occ_validate_epoch(as_dev(b), want_tn=True, append_history=True)
            if device_ptrs:
                torch.cuda.synchronize()
                rc, tn = rc.cpu().numpy(), tn.cpu().numpy().view(np.uint64)
            assert np.array_equal(np.asarray(rc), erc), f"epoch {e}: rc differs"
            assert np.array_equal(np.asarray(tn, np.uint64), etn), f"epoch {e}: tn differs"
            nk, nt = committed_writes(b, etn)
            hk, ht = np.concatenate([hk, nk]), np.concatenate([ht, nt])
            tnc = etnc
        gk, gt = engine.history_export()
        wk, wt = sorted_pairs(hk, ht)
        assert np.array_equal(gk, wk) and np.array_equal(gt, wt)
    finally:
        engine.set_option(OPT_HIST_MERGE, 65536)
        engine.history_clear()
        engine.tnc = 0
