"""Batch construction helpers shared by the CPU and GPU tests."""
from __future__ import annotations

import numpy as np

from deneva_amd import EpochBatch, RD, WR


def make_batch(txns, start_tn=None, finish_tn=None, order=None) -> EpochBatch:
    """txns: list of lists of (key, acctype)."""
    off = np.zeros(len(txns) + 1, np.uint32)
    keys, at = [], []
    for i, t in enumerate(txns):
        for k, a in t:
            keys.append(k)
            at.append(a)
        off[i + 1] = len(keys)
    st = None if start_tn is None else np.asarray(start_tn, np.uint64)
    ft = None if finish_tn is None else np.asarray(finish_tn, np.uint64)
    od = None if order is None else np.asarray(order, np.uint64)
    return EpochBatch(off, np.asarray(keys, np.uint64).reshape(-1),
                      np.asarray(at, np.uint8).reshape(-1), st, ft, od)


def random_batch(rng: np.random.Generator, n: int, max_len: int, n_keys: int,
                 p_write: float = 0.3, types=(RD, WR), unique=True) -> EpochBatch:
    """Ragged random batch: lengths in [0, max_len], keys uniform in [0, n_keys)."""
    lens = rng.integers(0, max_len + 1, size=n)
    txns = []
    for L in lens:
        if unique:
            L = min(int(L), n_keys)
            ks = rng.choice(n_keys, size=L, replace=False)
        else:
            ks = rng.integers(0, n_keys, size=int(L))
        ts = []
        for k in ks:
            if len(types) == 2:
                ts.append((int(k), WR if rng.random() < p_write else RD))
            else:
                ts.append((int(k), int(rng.choice(types))))
        txns.append(ts)
    return make_batch(txns)


def chain_batch(n: int) -> EpochBatch:
    """Txn i writes key i and reads key i-1: decisions alternate and the fixed
    point needs ~n rounds (exercises the round-tag wrap)."""
    txns = [[(0, WR)]] + [[(i - 1, RD), (i, WR)] for i in range(1, n)]
    return make_batch(txns)


def c4_batch(n_txn: int = 1 << 20, seed=None):
    """BASELINE config C4: YCSB theta 0.9, 16 partitions (keys row*16+part),
    65,536-txn generator chunks, each txn's home partition its origin node and
    the sequencer order (origin, FIFO within the origin) -- sched_dequeue's
    (epoch, origin, FIFO) order (work_queue.cpp:105-151)."""
    import deneva_amd as d
    kw = {} if seed is None else {"seed": seed}
    b = d.gen_ycsb(n_txn=n_txn, zipf_theta=0.9, part_cnt=16, chunk_txns=65536, want_home=True,
                   **kw)
    home = b.meta["home"].astype(np.uint64)
    seq = np.zeros(b.n_txn, np.uint64)
    for h in np.unique(home):
        idx = np.nonzero(home == h)[0]
        seq[idx] = np.arange(idx.size, dtype=np.uint64)
    b.order = (home << np.uint64(32)) | seq
    return b
