"""GPU parity of the sweep's read-only split (DCC_OPT_RO_SPLIT):
read-only txns that survive the level-0 filter leave the level lists and are
decided at the end against the epoch's committed-writer table (k_sw_wall
builds it from the committed writers the serial passes list, k_sw_ro decides).
Read-only txns never enter `active` (occ.cpp:151-154), so they neither kill
nor block, and each one's decision only needs the writers before it.

Cases: the split on and off on the same batches, the writer table overflowing
(the host rebuilds it sized for every write of the epoch), a later level
handing its write-only list to the round solver while read-only txns wait
(the table is then built from every committed txn of the decided epoch), the
serial-only last level resumed by the host, history windows, and the
decisions against the oracle's serial replay bit for bit."""
import numpy as np
import pytest

import _oracle as orc
import deneva_amd as d
from deneva_amd import RD, WR, EpochBatch
from deneva_amd._abi import OPT_RO_SPLIT, OPT_SOLVER, OPT_SWEEP_LEVELS

pytestmark = pytest.mark.gpu


@pytest.fixture
def eng(engine):
    engine.set_option(OPT_SOLVER, 0)
    yield engine
    engine.set_option(OPT_RO_SPLIT, 1)
    engine.set_option(OPT_SWEEP_LEVELS, 0)


def check(engine, b, hist=None, tnc=0):
    engine.tnc = tnc
    rc, tn, st = engine.occ_validate_epoch(b, want_tn=True)
    hk, ht = (None, None) if hist is None else hist
    erc, etn, etnc = orc.occ(b, hist_keys=hk, hist_tn=ht, tnc=tnc)
    rc = np.asarray(rc)
    bad = np.nonzero(rc != erc)[0]
    assert bad.size == 0, f"rc mismatch at {bad[:10]} (gpu {rc[bad[:10]]} oracle {erc[bad[:10]]})"
    assert np.array_equal(np.asarray(tn).astype(np.uint64), etn), "commit tn mismatch"
    assert engine.tnc == etnc
    return st


@pytest.mark.parametrize("split", [0, 1])
@pytest.mark.parametrize("theta,n", [(0.9, 1 << 20), (0.99, 1 << 20), (0.9, 65536), (0.6, 200000),
                                     (0.9, 3000)])
def test_split_on_off(eng, split, theta, n):
    eng.set_option(OPT_RO_SPLIT, split)
    b = d.gen_ycsb(n_txn=n, zipf_theta=theta, seed=0xA11CE + n)
    check(eng, b)


@pytest.mark.parametrize("bits", [4, 8, 12])
def test_writer_table_overflow(eng, bits):
    # a 2^bits-slot table overflows at once: the fallback table built from the
    # decided epoch decides the RO list; the next epoch runs with a larger
    # table (or overflows again) -- decisions identical every time
    b = d.gen_ycsb(n_txn=1 << 20, zipf_theta=0.9)
    eng.set_option(OPT_RO_SPLIT, bits)
    for _ in range(3):
        check(eng, b)


def handoff_batch(n=1 << 19, seed=7):
    """Level 0 kills ~76 % (a hot key written by txn 0); the rest are
    independent write txns (18 %, unique keys, so the level-1 filter kills
    none and the level-1 list goes to the round solver) and read-only txns
    (6 %, some reading keys an independent writer before them wrote)."""
    rng = np.random.default_rng(seed)
    hot = np.uint64(1)
    kind = rng.choice(3, size=n, p=[0.76, 0.18, 0.06])
    kind[0] = 0
    txns = []
    writers = []  # (txn, key) of independent write txns
    fresh = 10_000_000
    for i in range(n):
        if i == 0 or kind[i] == 0:
            txns.append([(int(hot), WR if i == 0 else RD)] + [(fresh + 4 * i + q, RD) for q in range(3)])
        elif kind[i] == 1:
            ks = [fresh + 4 * i + q for q in range(4)]
            txns.append([(k, WR if q % 2 == 0 else RD) for q, k in enumerate(ks)])
            writers.append((i, ks[0]))
        else:
            acc = [(fresh + 4 * i + q, RD) for q in range(3)]
            if writers and rng.random() < 0.5:  # a key an earlier independent writer wrote
                acc.append((writers[rng.integers(len(writers))][1], RD))
            else:
                acc.append((fresh + 4 * i + 3, RD))
            txns.append(acc)
    off = np.zeros(n + 1, np.uint32)
    off[1:] = np.cumsum([len(t) for t in txns])
    keys = np.array([k for t in txns for k, _ in t], np.uint64)
    at = np.array([a for t in txns for _, a in t], np.uint8)
    return EpochBatch(off, keys, at)


def test_handoff_after_split(eng):
    b = handoff_batch()
    st = check(eng, b)
    assert st["fallback"] >= 1, "the level-1 list was expected to go to the round solver"


@pytest.mark.parametrize("levels", [1, 2, 7])
def test_split_levels_per_sync(eng, levels):
    # host continuations (the RO list decided again after every resumed level)
    eng.set_option(OPT_SWEEP_LEVELS, levels)
    check(eng, d.gen_ycsb(n_txn=300000, zipf_theta=0.9, seed=0x5EED))


def test_split_history_window(eng):
    n = 1 << 18
    rng = np.random.default_rng(11)
    b = d.gen_ycsb(n_txn=n, zipf_theta=0.9, seed=0xB0B)
    hk = b.keys[rng.integers(0, b.nnz, size=5000)].astype(np.uint64)
    ht = rng.integers(1, 400, size=5000).astype(np.uint64)
    b.start_tn = rng.integers(0, 300, size=n).astype(np.uint64)
    b.finish_tn = (b.start_tn + rng.integers(0, 200, size=n)).astype(np.uint64)
    eng.history_clear()
    eng.history_append(hk, ht)
    try:
        check(eng, b, hist=(hk, ht), tnc=400)
    finally:
        eng.history_clear()
        eng.tnc = 0


def test_split_device_pointers_graph(eng):
    # the captured graph replays the split (k_sw_ro inside it) bit-exactly
    import torch
    b = d.gen_ycsb(n_txn=1 << 20, zipf_theta=0.9)
    db = b.to_torch("cuda:0")
    rc = torch.empty(b.n_txn, dtype=torch.uint8, device="cuda:0")
    erc, _, _ = orc.occ(b)
    for _ in range(3):
        rc.fill_(7)
        eng.occ_validate_epoch(db, out_rc=rc)
        torch.cuda.synchronize()
        assert np.array_equal(rc.cpu().numpy(), erc)
