"""GPU parity of pipelined epochs (dcc_occ_submit_epoch / dcc_occ_wait_epoch,
occ_pipe.cpp): consecutive epochs run on separate lanes of one GPU and must
decide exactly what dcc_occ_validate_epoch decides on them one after another
in submit order -- central_validate per epoch (occ.cpp:116-239), with the
commit counter tnc (occ.cpp:283-284) advancing in submit order.

Cases: 2, 3 and 4 lanes over distinct device batches (graph-replayed after
each lane's first epoch), host batches, out-of-order waits, an epoch asking
for commit tn in the middle of the stream (numbered from the tnc of every
epoch before it), streams of epochs with commit tn and the history append
(central_finish, occ.cpp:277-286, run by the context as each epoch
completes, or chained on the device behind each decision: DCC_OPT_PIPE_CHAIN)
checked tn by tn and pair by pair -- also when chained finishes fall back to
the host (epochs not final inside their graph, a malformed epoch in the
stream, epochs without tn between them) -- a history window behind
appends still in flight (it drains the lanes), a malformed batch (its error
comes back from its own wait; the others are unaffected), the synchronous
entry point draining the lanes first, and every epoch of a full-size (1M)
stream checked against the oracle."""
import numpy as np
import pytest

import _oracle as orc
import deneva_amd as d
from deneva_amd._abi import OPT_PIPE_CHAIN, OPT_PIPE_PARTITION, OPT_PIPELINE, OPT_SWEEP_LEVELS, DccError

pytestmark = pytest.mark.gpu


@pytest.fixture
def eng(engine):
    engine.tnc = 0
    yield engine
    engine.set_option(OPT_PIPELINE, 2)
    engine.set_option(OPT_PIPE_PARTITION, 0)
    engine.set_option(OPT_PIPE_CHAIN, 1)
    engine.set_option(OPT_SWEEP_LEVELS, 0)
    engine.tnc = 0


def batches(n, count, theta=0.9, seed=0x51DE):
    return [d.gen_ycsb(n_txn=n, zipf_theta=theta, seed=seed + i) for i in range(count)]


def expected(bs, tnc=0):
    out = []
    for b in bs:
        rc, tn, tnc = orc.occ(b, tnc=tnc)
        out.append((rc, tn, tnc))
    return out


@pytest.mark.parametrize("lanes,part", [(1, 0), (2, 0), (3, 0), (4, 0), (2, 1), (3, 1), (4, 1), (8, 1)])
def test_device_stream_matches_serial(eng, lanes, part):
    """part 1: each lane on its own XCDs (CU-masked streams, grids sized to
    the lane's CUs)."""
    import torch
    eng.set_option(OPT_PIPELINE, lanes)
    eng.set_option(OPT_PIPE_PARTITION, part)
    bs = batches(65536, 7)
    exp = expected(bs)
    dbs = [b.to_torch("cuda:0") for b in bs]
    outs = [torch.empty(b.n_txn, dtype=torch.uint8, device="cuda:0") for b in bs]
    # twice over the same buffers: the second pass replays every lane's graph
    for rep in range(2):
        eng.tnc = 0
        ts = [eng.occ_submit_epoch(db, o) for db, o in zip(dbs, outs)]
        sts = [eng.occ_wait_epoch(t) for t in ts]
        for i, (o, (erc, _, _)) in enumerate(zip(outs, exp)):
            assert np.array_equal(o.cpu().numpy(), erc), f"epoch {i}, pass {rep}"
            assert sts[i]["n_commit"] == int(np.count_nonzero(erc == d.RC_RCOK))
        assert eng.tnc == exp[-1][2]


def test_host_batches_and_out_of_order_waits(eng):
    eng.set_option(OPT_PIPELINE, 3)
    bs = batches(20000, 5, seed=0x77)
    exp = expected(bs)
    outs = [np.full(b.n_txn, 0xEE, np.uint8) for b in bs]
    ts = [eng.occ_submit_epoch(b, o) for b, o in zip(bs, outs)]
    order = [3, 0, 4, 2, 1]
    for k in order:
        eng.occ_wait_epoch(ts[k])
    for i, (o, (erc, _, _)) in enumerate(zip(outs, exp)):
        assert np.array_equal(o, erc), f"epoch {i}"
    with pytest.raises(DccError):
        eng.occ_wait_epoch(ts[0])  # each ticket is waited once
    assert eng.tnc == exp[-1][2]


def test_commit_tn_epoch_in_stream_numbers_in_order(eng):
    """An epoch asking for commit tn in the middle of the stream stays on its
    lane; the context numbers it when it completes, from the tnc of every
    epoch before it (occ.cpp:283-284)."""
    import torch
    eng.set_option(OPT_PIPELINE, 2)
    bs = batches(30000, 5, seed=0x99)
    exp = expected(bs)
    dbs = [b.to_torch("cuda:0") for b in bs]
    outs = [torch.empty(b.n_txn, dtype=torch.uint8, device="cuda:0") for b in bs]
    tn2 = torch.empty(bs[2].n_txn, dtype=torch.int64, device="cuda:0")
    ts = []
    for i, (db, o) in enumerate(zip(dbs, outs)):
        ts.append(eng.occ_submit_epoch(db, o, tn2 if i == 2 else None))
    for t in ts:
        eng.occ_wait_epoch(t)
    for i, (o, (erc, _, _)) in enumerate(zip(outs, exp)):
        assert np.array_equal(o.cpu().numpy(), erc), f"epoch {i}"
    assert np.array_equal(tn2.cpu().numpy().astype(np.uint64), exp[2][1])
    assert eng.tnc == exp[-1][2]


def test_malformed_epoch_reports_at_its_wait(eng):
    eng.set_option(OPT_PIPELINE, 2)
    bs = batches(10000, 3, seed=0x31)
    exp = expected([bs[0], bs[2]])
    bad = d.EpochBatch(bs[1].offsets.copy(), bs[1].keys, bs[1].acctype)
    bad.offsets[100] = bad.offsets[101] + 1  # offsets decrease
    outs = [np.zeros(b.n_txn, np.uint8) for b in bs]
    ts = [eng.occ_submit_epoch(b, o) for b, o in zip([bs[0], bad, bs[2]], outs)]
    eng.occ_wait_epoch(ts[0])
    with pytest.raises(DccError):
        eng.occ_wait_epoch(ts[1])
    eng.occ_wait_epoch(ts[2])
    assert np.array_equal(outs[0], exp[0][0])
    assert np.array_equal(outs[2], exp[1][0])


def test_sync_call_drains_first(eng):
    import torch
    eng.set_option(OPT_PIPELINE, 2)
    bs = batches(40000, 3, seed=0x45)
    exp = expected(bs)
    dbs = [b.to_torch("cuda:0") for b in bs]
    outs = [torch.empty(b.n_txn, dtype=torch.uint8, device="cuda:0") for b in bs]
    t0 = eng.occ_submit_epoch(dbs[0], outs[0])
    t1 = eng.occ_submit_epoch(dbs[1], outs[1])
    rc, tn, _ = eng.occ_validate_epoch(dbs[2], want_tn=True, out_rc=outs[2])
    assert np.array_equal(tn.cpu().numpy().astype(np.uint64), exp[2][1])
    eng.occ_wait_epoch(t1)
    eng.occ_wait_epoch(t0)
    for i, (o, (erc, _, _)) in enumerate(zip(outs, exp)):
        assert np.array_equal(o.cpu().numpy(), erc), f"epoch {i}"


@pytest.mark.parametrize("lanes,part", [(4, 0), (4, 1), (8, 1)])
def test_full_size_stream(eng, lanes, part):
    """The bench's pipelined headline: 1M-txn theta=0.9 epochs on the bench's
    lanes (one more epoch than lanes, so one lane takes two), unmasked or
    each lane on its own XCDs; every epoch in flight checked."""
    import torch
    eng.set_option(OPT_PIPELINE, lanes)
    eng.set_option(OPT_PIPE_PARTITION, part)
    bs = batches(1 << 20, lanes + 1, seed=0xD3E7A001)
    exp = expected(bs)
    dbs = [b.to_torch("cuda:0") for b in bs]
    outs = [torch.empty(b.n_txn, dtype=torch.uint8, device="cuda:0") for b in bs]
    for rep in range(3):
        eng.tnc = 0
        ts = [eng.occ_submit_epoch(db, o) for db, o in zip(dbs, outs)]
        for t in ts:
            eng.occ_wait_epoch(t)
        for i, (o, (erc, _, _)) in enumerate(zip(outs, exp)):
            assert np.array_equal(o.cpu().numpy(), erc), f"epoch {i}, pass {rep}"
        assert eng.tnc == exp[-1][2]


def test_option_change_keeps_outstanding_tickets(eng):
    """DCC_OPT_PIPELINE while epochs are in flight: they complete on their
    lanes and keep their results until waited (dcc.h); tickets keep counting
    up, so an old ticket never aliases a new epoch."""
    import torch
    eng.set_option(OPT_PIPELINE, 3)
    bs = batches(30000, 6, seed=0x5E7)
    exp = expected(bs)
    dbs = [b.to_torch("cuda:0") for b in bs]
    outs = [torch.empty(b.n_txn, dtype=torch.uint8, device="cuda:0") for b in bs]
    ts = [eng.occ_submit_epoch(dbs[i], outs[i]) for i in range(3)]
    eng.set_option(OPT_PIPELINE, 2)
    ts += [eng.occ_submit_epoch(dbs[i], outs[i]) for i in range(3, 6)]
    assert len(set(ts)) == 6 and ts == sorted(ts)
    sts = [eng.occ_wait_epoch(t) for t in ts]
    for i, (o, (erc, _, _)) in enumerate(zip(outs, exp)):
        assert np.array_equal(o.cpu().numpy(), erc), f"epoch {i}"
        assert sts[i]["n_commit"] == int(np.count_nonzero(erc == d.RC_RCOK))
    assert eng.tnc == exp[-1][2]


def committed_pairs(b, tn):
    off = np.asarray(b.offsets, np.int64)
    owner = np.repeat(np.arange(b.n_txn), np.diff(off))
    sel = (np.asarray(b.acctype) == d.WR) & (np.asarray(tn)[owner] != 0)
    return np.asarray(b.keys, np.uint64)[sel], np.asarray(tn, np.uint64)[owner[sel]]


def sorted_pairs(k, t):
    k, t = np.asarray(k, np.uint64), np.asarray(t, np.uint64)
    o = np.lexsort((t, k))
    return k[o], t[o]


@pytest.mark.parametrize("lanes,device,chain", [(2, True, 1), (4, True, 1), (3, False, 1), (4, True, 0),
                                               (3, False, 0)])
def test_tn_and_history_stream(eng, lanes, device, chain):
    """Every epoch of the stream wants commit tn and appends its committed
    writes (the reference's central_finish under TS_CLOCK); the lanes only
    decide, the context numbers and appends in submit order.  Each epoch's
    tns, tnc and the final history equal the oracle's serial chain; then an
    epoch with TS_CAS windows behind two appends still in flight drains the
    lanes and sees all of them."""
    import torch
    eng.set_option(OPT_PIPELINE, lanes)
    eng.set_option(OPT_PIPE_CHAIN, chain)
    eng.history_clear()
    try:
        bs = batches(40000, 7, seed=0x7A1)
        tnc, exp, hk, ht = 0, [], np.zeros(0, np.uint64), np.zeros(0, np.uint64)
        for b in bs:
            rc, tn, tnc = orc.occ(b, tnc=tnc)
            exp.append((rc, tn, tnc))
            k, t = committed_pairs(b, tn)
            hk, ht = np.concatenate([hk, k]), np.concatenate([ht, t])
        if device:
            ins = [b.to_torch("cuda:0") for b in bs]
            rcs = [torch.empty(b.n_txn, dtype=torch.uint8, device="cuda:0") for b in bs]
            tns = [torch.empty(b.n_txn, dtype=torch.int64, device="cuda:0") for b in bs]
        else:
            ins = bs
            rcs = [np.zeros(b.n_txn, np.uint8) for b in bs]
            tns = [np.zeros(b.n_txn, np.uint64) for b in bs]
        for rep in range(2):  # the second pass replays every lane's graph
            eng.history_clear()
            eng.tnc = 0
            ts = [eng.occ_submit_epoch(x, r, t, append_history=True) for x, r, t in zip(ins, rcs, tns)]
            where = [eng.occ_wait_epoch(t)["fin_where"] for t in ts]
            assert all(w == 2 for w in where) if not chain else where.count(1) >= 4, where
            for i, (r, t, (erc, etn, _)) in enumerate(zip(rcs, tns, exp)):
                r = r.cpu().numpy() if device else r
                t = t.cpu().numpy().view(np.uint64) if device else t
                assert np.array_equal(r, erc), f"pass {rep} epoch {i}: rc"
                assert np.array_equal(t, etn), f"pass {rep} epoch {i}: tn"
            assert eng.tnc == exp[-1][2]
            assert eng.history_size == hk.size
            gk, gt = eng.history_export()
            wk, wt = sorted_pairs(hk, ht)
            assert np.array_equal(gk, wk) and np.array_equal(gt, wt)
        # a window epoch behind appends still in flight
        eng.history_clear()
        eng.tnc = 0
        w = d.gen_ycsb(n_txn=30000, zipf_theta=0.9, seed=0x7A9)
        rng = np.random.default_rng(5)
        t2 = exp[1][2]
        w.start_tn = rng.integers(0, t2 + 1, size=w.n_txn).astype(np.uint64)
        w.finish_tn = (w.start_tn + rng.integers(0, t2 + 1, size=w.n_txn)).astype(np.uint64)
        k01 = [committed_pairs(bs[i], exp[i][1]) for i in range(2)]
        wrc, wtn, wtnc = orc.occ(w, hist_keys=np.concatenate([k01[0][0], k01[1][0]]),
                                 hist_tn=np.concatenate([k01[0][1], k01[1][1]]), tnc=t2)
        ow = np.zeros(w.n_txn, np.uint8)
        otw = np.zeros(w.n_txn, np.uint64)
        keep = [(np.zeros(bs[i].n_txn, np.uint8), np.zeros(bs[i].n_txn, np.uint64)) for i in range(2)]
        ts = [eng.occ_submit_epoch(bs[i], keep[i][0], keep[i][1], append_history=True) for i in range(2)]
        tw = eng.occ_submit_epoch(w, ow, otw, append_history=True)
        for t in ts + [tw]:
            eng.occ_wait_epoch(t)
        assert np.array_equal(ow, wrc) and np.array_equal(otw, wtn) and eng.tnc == wtnc
    finally:
        eng.history_clear()


def test_full_size_tn_history_stream(eng):
    """Five 1M-txn theta=0.9 epochs on 4 lanes, each with commit tn and the
    history append: every epoch's tns and the history against the oracle."""
    import torch
    eng.set_option(OPT_PIPELINE, 4)
    eng.history_clear()
    try:
        bs = batches(1 << 20, 5, seed=0xD3E7A001)
        tnc, exp = 0, []
        hk, ht = [], []
        for b in bs:
            rc, tn, tnc = orc.occ(b, tnc=tnc)
            exp.append((rc, tn, tnc))
            k, t = committed_pairs(b, tn)
            hk.append(k)
            ht.append(t)
        dbs = [b.to_torch("cuda:0") for b in bs]
        rcs = [torch.empty(b.n_txn, dtype=torch.uint8, device="cuda:0") for b in bs]
        tns = [torch.empty(b.n_txn, dtype=torch.int64, device="cuda:0") for b in bs]
        eng.tnc = 0
        ts = [eng.occ_submit_epoch(x, r, t, append_history=True) for x, r, t in zip(dbs, rcs, tns)]
        for t in ts:
            eng.occ_wait_epoch(t)
        for i, (r, t, (erc, etn, _)) in enumerate(zip(rcs, tns, exp)):
            assert np.array_equal(r.cpu().numpy(), erc), f"epoch {i}: rc"
            assert np.array_equal(t.cpu().numpy().view(np.uint64), etn), f"epoch {i}: tn"
        assert eng.tnc == exp[-1][2]
        gk, gt = eng.history_export()
        wk, wt = sorted_pairs(np.concatenate(hk), np.concatenate(ht))
        assert np.array_equal(gk, wk) and np.array_equal(gt, wt)
    finally:
        eng.history_clear()


def run_mixed(eng, bs, want, app, device):
    """Submit every batch (want[i]: commit tn, app[i]: history append), wait
    for all; returns (rcs, tns or None, errors)."""
    import torch
    if device:
        ins = [b.to_torch("cuda:0") for b in bs]
        rcs = [torch.empty(b.n_txn, dtype=torch.uint8, device="cuda:0") for b in bs]
        tns = [torch.empty(b.n_txn, dtype=torch.int64, device="cuda:0") if w else None
               for b, w in zip(bs, want)]
    else:
        ins = bs
        rcs = [np.zeros(b.n_txn, np.uint8) for b in bs]
        tns = [np.zeros(b.n_txn, np.uint64) if w else None for b, w in zip(bs, want)]
    ts = [eng.occ_submit_epoch(x, r, t, append_history=a) for x, r, t, a in zip(ins, rcs, tns, app)]
    errs, where = [], []
    for t in ts:
        try:
            where.append(eng.occ_wait_epoch(t)["fin_where"])
            errs.append(None)
        except DccError as e:
            where.append(None)
            errs.append(e)
    rcs = [r.cpu().numpy() if device else r for r in rcs]
    tns = [None if t is None else (t.cpu().numpy().view(np.uint64) if device else t) for t in tns]
    return rcs, tns, errs, where


def check_mixed(eng, bs, want, app, rcs, tns, errs, where, skip=()):
    """Against the oracle's serial chain (a skipped epoch leaves no trace)."""
    tnc, hk, ht = 0, [np.zeros(0, np.uint64)], [np.zeros(0, np.uint64)]
    for i, b in enumerate(bs):
        if i in skip:
            assert errs[i] is not None, f"epoch {i} should fail"
            continue
        assert errs[i] is None, f"epoch {i}: {errs[i]}"
        rc, tn, tnc = orc.occ(b, tnc=tnc)
        assert np.array_equal(rcs[i], rc), f"epoch {i}: rc"
        if want[i]:
            assert np.array_equal(tns[i], tn), f"epoch {i}: tn"
        if app[i]:
            k, t = committed_pairs(b, tn)
            hk.append(k)
            ht.append(t)
    assert eng.tnc == tnc
    gk, gt = eng.history_export()
    wk, wt = sorted_pairs(np.concatenate(hk), np.concatenate(ht))
    assert np.array_equal(gk, wk) and np.array_equal(gt, wt)


@pytest.mark.parametrize("levels", [1, 2])
def test_chained_finish_falls_back_when_not_final(eng, levels):
    """One or two sweep levels per lane graph: the 1M-txn theta=0.9 epochs are
    not decided inside their graphs (more levels follow a host round trip), so
    every chained finish finds its epoch not final, or an epoch before it not
    finished, and the context finishes them in submit order; then a second
    pass at the default schedule numbers them on the device."""
    eng.set_option(OPT_PIPELINE, 3)
    eng.history_clear()
    try:
        bs = batches(1 << 20, 4, seed=0x3C1)
        want, app = [True] * 4, [True] * 4
        eng.set_option(OPT_SWEEP_LEVELS, levels)
        eng.tnc = 0
        out = run_mixed(eng, bs, want, app, True)
        check_mixed(eng, bs, want, app, *out)
        assert all(w == 2 for w in out[3]), out[3]  # every one finished by the host
        eng.set_option(OPT_SWEEP_LEVELS, 0)
        eng.history_clear()
        eng.tnc = 0
        out = run_mixed(eng, bs, want, app, True)
        check_mixed(eng, bs, want, app, *out)
        assert out[3].count(1) >= 3, out[3]  # numbered on the device (a lane's first may not be)
    finally:
        eng.set_option(OPT_SWEEP_LEVELS, 0)
        eng.history_clear()


@pytest.mark.parametrize("lanes", [2, 4])
def test_chained_finish_mixed_stream(eng, lanes):
    """Epochs with commit tn and the append, commit tn only, and neither, in
    one stream: the ones the host completes (no tn) move the device tnc past
    them for the chained finishes behind them."""
    eng.set_option(OPT_PIPELINE, lanes)
    eng.history_clear()
    try:
        bs = batches(50000, 9, seed=0x4D1)
        want = [True, False, True, True, False, False, True, True, True]
        app = [True, False, False, True, False, False, True, False, True]
        for rep in range(2):
            eng.history_clear()
            eng.tnc = 0
            out = run_mixed(eng, bs, want, app, rep == 0)
            check_mixed(eng, bs, want, app, *out)
            assert all((w == 0) == (not t) for w, t in zip(out[3], want)), out[3]
            assert 1 in out[3], out[3]
    finally:
        eng.history_clear()


def test_chained_finish_malformed_epoch_in_stream(eng):
    """A malformed epoch among chained ones: its error at its own wait, no
    trace in tnc or the history; the epochs behind it numbered as if it had
    not been submitted."""
    eng.set_option(OPT_PIPELINE, 3)
    eng.history_clear()
    try:
        bs = batches(20000, 6, seed=0x5E1)
        bad = d.EpochBatch(bs[2].offsets.copy(), bs[2].keys, bs[2].acctype)
        bad.offsets[100] = bad.offsets[101] + 1  # offsets decrease
        bs[2] = bad
        want, app = [True] * 6, [True] * 6
        eng.tnc = 0
        out = run_mixed(eng, bs, want, app, False)
        check_mixed(eng, bs, want, app, *out, skip=(2,))
        # and the stream goes on chained behind it
        eng.history_clear()
        eng.tnc = 0
        good = batches(20000, 6, seed=0x5E1)
        out = run_mixed(eng, good, want, app, False)
        check_mixed(eng, good, want, app, *out)
        assert 1 in out[3], out[3]
    finally:
        eng.history_clear()


def test_chained_finish_out_of_order_waits_and_lane_change(eng):
    """Chained epochs waited newest first, then the lane count changed with
    chained epochs in flight (they complete on their lanes first), then more
    chained epochs on the new lanes, CU-partitioned: one serial chain."""
    eng.set_option(OPT_PIPELINE, 3)
    eng.history_clear()
    try:
        bs = batches(30000, 8, seed=0x6A1)
        want, app = [True] * 8, [True, True, False, True, True, True, False, True]
        eng.tnc = 0
        rcs = [np.zeros(b.n_txn, np.uint8) for b in bs]
        tns = [np.zeros(b.n_txn, np.uint64) for b in bs]
        ts = [eng.occ_submit_epoch(bs[i], rcs[i], tns[i], append_history=app[i]) for i in range(4)]
        eng.set_option(OPT_PIPELINE, 4)
        eng.set_option(OPT_PIPE_PARTITION, 1)
        ts += [eng.occ_submit_epoch(bs[i], rcs[i], tns[i], append_history=app[i]) for i in range(4, 8)]
        where = {t: eng.occ_wait_epoch(t)["fin_where"] for t in reversed(ts)}
        check_mixed(eng, bs, want, app, rcs, tns, [None] * 8, [where[t] for t in ts])
        assert 1 in where.values(), where
    finally:
        eng.history_clear()
