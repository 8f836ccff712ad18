"""GPU parity of captured-snapshot validation (dcc_occ_validate_snapshot)
against the literal snapshot oracle and against the simulated live run that
made the capture: bit-exact RCs."""
import numpy as np
import pytest

import _oracle as orc
import deneva_amd as d
from deneva_amd import EpochBatch, RD, WR, SCAN
from helpers import make_batch, random_batch
from live_sim import simulate
from test_snapshot_oracle import live_case

pytestmark = pytest.mark.gpu


def check(engine, b, aoff, aidx, top=None, hk=None, ht=None, device=False, expect=None):
    engine.history_clear()
    if hk is not None and len(hk):
        engine.history_append(hk, ht)
    want = orc.occ_snapshot(b, aoff, aidx, top, hk, ht)
    if device:
        import torch
        bb = b.to_torch()
        cv = lambda a: None if a is None else torch.from_numpy(
            np.ascontiguousarray(a).view(np.int64 if a.dtype == np.uint64 else np.int32)).cuda()
        rc, st = engine.occ_validate_snapshot(bb, cv(aoff), cv(aidx) if len(aidx) else
                                              torch.zeros(1, dtype=torch.int32, device="cuda"),
                                              cv(top))
        rc = rc.cpu().numpy()
    else:
        rc, st = engine.occ_validate_snapshot(b, aoff, aidx, top)
        rc = np.asarray(rc)
    bad = np.nonzero(rc != want)[0]
    assert bad.size == 0, f"rc mismatch at {bad[:10]}: gpu {rc[bad[:10]]} oracle {want[bad[:10]]}"
    if expect is not None:
        assert np.array_equal(rc, expect)
    assert st["n_commit"] == int((want == 0).sum())
    assert st["n_abort"] == int((want == 2).sum())
    return rc, st


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("threads", [4, 32])
@pytest.mark.parametrize("device", [False, True])
def test_live_capture_parity(engine, seed, threads, device):
    hist0 = [(tn, [int(k) for k in np.random.default_rng(seed).integers(0, 200, 3)])
             for tn in range(1, 41)]
    b, cap = live_case(seed, n=600, threads=threads, hist0=hist0, tnc0=40)
    check(engine, b, cap["active_off"], cap["active_idx"], cap["hist_top"], cap["hist_keys"],
          cap["hist_tn"], device=device, expect=cap["rc"])


def test_known_answers(engine):
    b = make_batch([[(5, WR)], [(5, RD)], [(5, WR)], [(5, RD)], [(9, WR)],
                    [(7, SCAN)], [(7, RD)], [(7, RD)]],
                   start_tn=[0, 0, 0, 0, 0, 10, 10, 20], finish_tn=[0, 0, 0, 0, 0, 20, 20, 20])
    aoff = np.array([0, 0, 1, 2, 2, 3, 3, 3, 3], np.uint32)
    aidx = np.array([0, 0, 0], np.uint32)
    top = np.array([99, 99, 99, 99, 99, 99, 12, 99], np.uint64)
    check(engine, b, aoff, aidx, top, np.array([7, 3], np.uint64), np.array([15, 11], np.uint64),
          expect=np.array([0, 2, 2, 0, 0, 2, 0, 0], np.uint8))


def synthetic_capture(rng, n, max_active, hist=True):
    """Large capture without a run: txn i saw up to max_active earlier txns."""
    b = d.gen_ycsb(n_txn=n, zipf_theta=0.9, table_size=1 << 20)
    cnt = rng.integers(0, max_active + 1, size=n)
    cnt = np.minimum(cnt, np.arange(n))
    aoff = np.zeros(n + 1, np.uint32)
    aoff[1:] = np.cumsum(cnt)
    t = np.repeat(np.arange(n), cnt)
    aidx = (t - 1 - rng.integers(0, 64, size=t.size) % np.maximum(t, 1)).clip(0).astype(np.uint32)
    st = ft = top = hk = ht = None
    if hist:
        st = rng.integers(0, 1000, size=n).astype(np.uint64)
        ft = (st + rng.integers(0, 200, size=n)).astype(np.uint64)
        top = rng.integers(0, 1200, size=n).astype(np.uint64)
        hk = rng.integers(0, 1 << 20, size=20000).astype(np.uint64)
        ht = rng.integers(1, 1200, size=20000).astype(np.uint64)
    return EpochBatch(b.offsets, b.keys, b.acctype, st, ft), aoff, aidx, top, hk, ht


@pytest.mark.parametrize("hist", [False, True])
def test_synthetic_large(engine, hist):
    rng = np.random.default_rng(5)
    b, aoff, aidx, top, hk, ht = synthetic_capture(rng, 100000, 8, hist)
    rc, st = check(engine, b, aoff, aidx, top, hk, ht)
    assert 0 < st["n_abort"] < b.n_txn


def test_no_hist_top_sees_whole_history(engine):
    rng = np.random.default_rng(9)
    b, aoff, aidx, top, hk, ht = synthetic_capture(rng, 20000, 4, True)
    check(engine, b, aoff, aidx, None, hk, ht)


def test_edges(engine):
    # empty batch, empty txns, no active entries at all, max-length txns
    empty = make_batch([])
    rc, st = engine.occ_validate_snapshot(empty, np.zeros(1, np.uint32), np.zeros(0, np.uint32))
    assert st["n_commit"] == 0
    txns = [[], [(1, WR)], [(k, RD if k % 2 else WR) for k in range(64)], [(1, RD)]]
    b = make_batch(txns)
    check(engine, b, np.zeros(5, np.uint32), np.zeros(0, np.uint32),
          expect=np.zeros(4, np.uint8))
    aoff = np.array([0, 0, 0, 2, 4], np.uint32)
    aidx = np.array([0, 1, 2, 1], np.uint32)
    check(engine, b, aoff, aidx, expect=np.array([0, 0, 2, 2], np.uint8))


def test_malformed_capture_rejected(engine):
    b = make_batch([[(1, WR)], [(1, RD)]])
    with pytest.raises(Exception):
        engine.occ_validate_snapshot(b, np.array([0, 0, 1], np.uint32), np.array([5], np.uint32))
    with pytest.raises(Exception):
        engine.occ_validate_snapshot(b, np.array([0, 1, 0], np.uint32), np.array([0], np.uint32))
