"""GPU parity of the deferred central_finish (DCC_OCC_DEFER_FINISH +
dcc_occ_finish_epoch): a 2PC participant validates with its local RC
(OptCC::validate, occ.cpp:116-239), votes, and finishes with the GLOBAL RC
that RFIN brings back (worker_thread.cpp:286-297 -> OptCC::finish,
occ.cpp:248-294).  Only globally committed writers take a commit tn and join
the history; a txn that validated locally but aborted globally leaves no
trace, so a later epoch's history window never sees its writes."""
import numpy as np
import pytest

import _oracle as orc
import deneva_amd as d
from deneva_amd import RC_ABORT, RC_RCOK, WR
from deneva_amd._abi import DccError
from helpers import random_batch

pytestmark = pytest.mark.gpu


def has_write(b):
    off, at = np.asarray(b.offsets), np.asarray(b.acctype)
    w = np.zeros(b.n_txn, bool)
    for t in range(b.n_txn):
        w[t] = (at[off[t]:off[t + 1]] == WR).any()
    return w


def expected_finish(b, final, tnc):
    """central_finish over the global RC: tn and the (key, tn) history rows."""
    off, keys, at = np.asarray(b.offsets), np.asarray(b.keys), np.asarray(b.acctype)
    hw = has_write(b)
    tn = np.zeros(b.n_txn, np.uint64)
    hk, ht = [], []
    for t in range(b.n_txn):
        if final[t] == RC_RCOK and hw[t]:
            tnc += 1
            tn[t] = tnc
            for x in range(off[t], off[t + 1]):
                if at[x] == WR:
                    hk.append(keys[x])
                    ht.append(tnc)
    return tn, np.array(hk, np.uint64), np.array(ht, np.uint64), tnc


def global_rc(rc, rng, p_remote_abort):
    """The coordinator's decision: RCOK only where this node voted RCOK and
    no other participant voted abort."""
    g = np.asarray(rc).copy()
    remote = rng.random(g.shape[0]) < p_remote_abort
    g[remote] = RC_ABORT
    return g


@pytest.fixture
def eng(engine):
    engine.history_clear()
    engine.tnc = 0
    yield engine
    if engine.pending_finish is not None:  # never leave an epoch pending
        engine.occ_finish_epoch(np.full(engine.pending_finish, RC_ABORT, np.uint8), want_tn=False)
    engine.history_clear()
    engine.tnc = 0


@pytest.mark.parametrize("n", [1, 700, 40000])
def test_global_abort_keeps_writes_out_of_history(eng, n):
    rng = np.random.default_rng(n)
    b = random_batch(rng, n, 10, max(64, n // 8), p_write=0.4)
    eng.tnc = 100
    rc, tn, _ = eng.occ_validate_epoch(b, defer_finish=True)
    assert tn is None
    erc, _, _ = orc.occ(b, tnc=100)
    assert np.array_equal(np.asarray(rc), erc)
    assert eng.tnc == 100  # nothing committed until the global RC arrives
    g = global_rc(rc, rng, 0.3)
    got = eng.occ_finish_epoch(g)
    etn, hk, ht, etnc = expected_finish(b, g, 100)
    assert np.array_equal(np.asarray(got).astype(np.uint64), etn)
    assert eng.tnc == etnc
    k, t = eng.history_export()
    order = np.lexsort((ht, hk))
    assert np.array_equal(np.asarray(k), hk[order]) and np.array_equal(np.asarray(t), ht[order])

    # the next epoch's history window covers the whole finished epoch: its
    # readers abort exactly on the globally committed writes
    b2 = random_batch(rng, n, 8, max(64, n // 8), p_write=0.3)
    b2.start_tn = np.full(b2.n_txn, 100, np.uint64)
    b2.finish_tn = np.full(b2.n_txn, etnc, np.uint64)
    rc2, tn2, _ = eng.occ_validate_epoch(b2, want_tn=True)
    erc2, etn2, _ = orc.occ(b2, hist_keys=hk, hist_tn=ht, tnc=etnc)
    assert np.array_equal(np.asarray(rc2), erc2)
    assert np.array_equal(np.asarray(tn2).astype(np.uint64), etn2)


def test_remote_abort_of_only_writer_frees_the_key(eng):
    # txn 0 writes key 5 and validates locally; another participant aborts
    # it.  A reader of key 5 in the next epoch must commit.
    b = d.EpochBatch(np.array([0, 1], np.uint32), np.array([5], np.uint64),
                     np.array([WR], np.uint8))
    rc, _, _ = eng.occ_validate_epoch(b, defer_finish=True)
    assert list(np.asarray(rc)) == [RC_RCOK]
    tn = eng.occ_finish_epoch(np.array([RC_ABORT], np.uint8))
    assert list(np.asarray(tn)) == [0] and eng.tnc == 0 and eng.history_size == 0
    r = d.EpochBatch(np.array([0, 1], np.uint32), np.array([5], np.uint64),
                     np.array([0], np.uint8), start_tn=np.zeros(1, np.uint64),
                     finish_tn=np.ones(1, np.uint64))
    rc, _, _ = eng.occ_validate_epoch(r)
    assert list(np.asarray(rc)) == [RC_RCOK]
    # the same epoch committed globally: the reader aborts
    rc, _, _ = eng.occ_validate_epoch(b, defer_finish=True)
    eng.occ_finish_epoch(np.array([RC_RCOK], np.uint8))
    assert eng.tnc == 1
    rc, _, _ = eng.occ_validate_epoch(r)
    assert list(np.asarray(rc)) == [RC_ABORT]


def test_equal_votes_match_immediate_finish(eng):
    # global RC == local RC: the deferred pair equals one APPEND_HISTORY call
    rng = np.random.default_rng(9)
    b = random_batch(rng, 20000, 12, 3000, p_write=0.5)
    rc, _, _ = eng.occ_validate_epoch(b, defer_finish=True)
    tn_d = np.asarray(eng.occ_finish_epoch(np.asarray(rc).copy())).copy()
    hist_d = [np.asarray(a).copy() for a in eng.history_export()]
    tnc_d = eng.tnc
    eng.history_clear()
    eng.tnc = 0
    _, tn_i, _ = eng.occ_validate_epoch(b, want_tn=True, append_history=True)
    assert np.array_equal(tn_d, np.asarray(tn_i)) and eng.tnc == tnc_d
    hist_i = eng.history_export()
    assert all(np.array_equal(x, np.asarray(y)) for x, y in zip(hist_d, hist_i))


def test_device_pointers(eng):
    import torch
    rng = np.random.default_rng(4)
    b = random_batch(rng, 30000, 8, 2000, p_write=0.4)
    rc, _, _ = eng.occ_validate_epoch(b.to_torch("cuda:0"), defer_finish=True)
    g = global_rc(rc.cpu().numpy(), rng, 0.2)
    tn = eng.occ_finish_epoch(torch.from_numpy(g).to("cuda:0"))
    torch.cuda.synchronize()
    etn, _, _, etnc = expected_finish(b, g, 0)
    assert np.array_equal(tn.cpu().numpy().astype(np.uint64), etn) and eng.tnc == etnc


def test_errors(eng):
    rng = np.random.default_rng(2)
    b = random_batch(rng, 500, 6, 50, p_write=0.5)
    with pytest.raises(DccError):  # nothing pending
        eng.occ_finish_epoch(np.zeros(500, np.uint8))
    with pytest.raises(DccError):  # DEFER with APPEND_HISTORY
        eng.occ_validate_epoch(b, append_history=True, defer_finish=True)
    with pytest.raises(DccError):  # tn comes from the finish call
        eng.occ_validate_epoch(b, want_tn=True, defer_finish=True)
    rc, _, _ = eng.occ_validate_epoch(b, defer_finish=True)
    with pytest.raises(DccError):  # the pending epoch blocks the next one
        eng.occ_validate_epoch(b)
    rc = np.asarray(rc)
    assert (rc == RC_ABORT).any()
    with pytest.raises(ValueError):
        eng.occ_finish_epoch(rc[:10].copy())
    bad = np.zeros(500, np.uint8)  # global RCOK for a local abort
    with pytest.raises(DccError):
        eng.occ_finish_epoch(bad)
    # still pending after the rejected finish; a valid one goes through
    eng.occ_finish_epoch(rc.copy())
    assert eng.tnc == int(((rc == RC_RCOK) & has_write(b)).sum())


def test_sharded_context(eng):
    # key-sharded context: each shard appends its own keys' writes, the tn
    # numbering is the global one
    rng = np.random.default_rng(21)
    b = random_batch(rng, 20000, 10, 4000, p_write=0.4)
    with d.Engine(devices=[0, 0, 0]) as m:
        rc, _, _ = m.occ_validate_epoch(b, defer_finish=True)
        g = global_rc(rc, rng, 0.25)
        tn = m.occ_finish_epoch(g)
        etn, hk, ht, etnc = expected_finish(b, g, 0)
        assert np.array_equal(np.asarray(tn).astype(np.uint64), etn)
        b2 = random_batch(rng, 20000, 8, 4000, p_write=0.3)
        b2.start_tn = np.zeros(b2.n_txn, np.uint64)
        b2.finish_tn = np.full(b2.n_txn, etnc, np.uint64)
        rc2, _, _ = m.occ_validate_epoch(b2)
        erc2, _, _ = orc.occ(b2, hist_keys=hk, hist_tn=ht, tnc=etnc)
        assert np.array_equal(np.asarray(rc2), erc2)


def test_sharded_device_batch_calvin_between(eng):
    # a device batch on a key-sharded context: each rank's shard lives in the
    # context's own buffers, which the Calvin epoch run between the deferred
    # validate and the finish rewrites -- the finish must still append the
    # validated epoch's writes (the shard is kept aside), not the Calvin batch's
    import torch
    rng = np.random.default_rng(23)
    b = random_batch(rng, 20000, 10, 4000, p_write=0.4)
    c = d.gen_ycsb(n_txn=30000, zipf_theta=0.9, part_cnt=4, chunk_txns=4096, seed=77)
    with d.Engine(devices=[0, 0, 0]) as m:
        rc, _, _ = m.occ_validate_epoch(b.to_torch("cuda:0"), defer_finish=True)
        torch.cuda.synchronize()
        rc = rc.cpu().numpy()
        erc, _, _ = orc.occ(b)
        assert np.array_equal(rc, erc)
        g, crc, _, _ = m.calvin_order_epoch(c, want_group=True)
        eg, ecrc, _ = orc.calvin(c)
        assert np.array_equal(np.asarray(g).astype(np.uint32), eg)
        gl = global_rc(rc, rng, 0.25)
        tn = m.occ_finish_epoch(gl)
        etn, hk, ht, etnc = expected_finish(b, gl, 0)
        assert np.array_equal(np.asarray(tn).astype(np.uint64), etn)
        # the history holds b's committed writes: a later epoch's window sees them
        b2 = random_batch(rng, 20000, 8, 4000, p_write=0.3)
        b2.start_tn = np.zeros(b2.n_txn, np.uint64)
        b2.finish_tn = np.full(b2.n_txn, etnc, np.uint64)
        rc2, _, _ = m.occ_validate_epoch(b2)
        erc2, _, _ = orc.occ(b2, hist_keys=hk, hist_tn=ht, tnc=etnc)
        assert np.array_equal(np.asarray(rc2), erc2)


def test_compact_device_batch_calvin_between(eng):
    # a DEVICE batch in the compact form (u32 keys, 2-bit types): its widened
    # keys / types live in the context's staging buffers, which a Calvin
    # epoch between the deferred validate and the finish rewrites -- the
    # finish must append the validated epoch's writes (kept aside), not the
    # Calvin batch's
    import torch
    from deneva_amd.engine import pack_acctype
    rng = np.random.default_rng(31)
    b = d.gen_ycsb(n_txn=30000, zipf_theta=0.9, table_size=1 << 16, seed=31)
    keys = torch.from_numpy(np.asarray(b.keys, np.uint32).view(np.int32)).cuda()
    at = torch.from_numpy(pack_acctype(b.acctype)).cuda()
    off = torch.from_numpy(np.asarray(b.offsets, np.uint32).view(np.int32)).cuda()
    db = d.EpochBatch(off, keys, at, meta={"acctype_2bit": True})
    rc, _, _ = eng.occ_validate_epoch(db, defer_finish=True)
    torch.cuda.synchronize()
    rc = rc.cpu().numpy()
    assert np.array_equal(rc, orc.occ(b)[0])
    c = d.gen_ycsb(n_txn=40000, zipf_theta=0.9, part_cnt=4, chunk_txns=4096, seed=78)
    g, _, _, _ = eng.calvin_order_epoch(c, want_group=True)  # host batch: the same staging buffers
    assert np.array_equal(np.asarray(g).astype(np.uint32), orc.calvin(c)[0])
    gl = global_rc(rc, rng, 0.2)
    tn = eng.occ_finish_epoch(gl)
    etn, hk, ht, etnc = expected_finish(b, gl, 0)
    assert np.array_equal(np.asarray(tn).astype(np.uint64), etn) and eng.tnc == etnc
    k, t = eng.history_export()
    order = np.lexsort((ht, hk))
    assert np.array_equal(np.asarray(k), hk[order]) and np.array_equal(np.asarray(t), ht[order])
