#!/usr/bin/env python3
"""Writes the committed .dccb golden fixtures (batch + the oracle's decisions).

The reference has no tests or golden vectors for this path and cannot be built
here; these fixtures freeze the oracle's literal replays
(oracle/occ_ref.c: OptCC central_validate/central_finish epoch replay,
oracle/calvin_ref.c: Row_lock CALVIN grant/release simulation) on seeded
batches in the configs' shapes, so that the CPU suite pins the oracle and the
GPU suite checks the engine against stored vectors as well as live replays.

    python tests/golden/make_fixtures.py        # rewrites tests/golden/*.dccb
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))

import _oracle as orc  # noqa: E402
import deneva_amd as d  # noqa: E402
from deneva_amd._abi import FILE_CALVIN, FILE_OCC  # noqa: E402


def occ_fixture(name, b, seed, tnc=0):
    rc, tn, _ = orc.occ(b, tnc=tnc, literal=True)
    d.write_batch_file(os.path.join(HERE, name), b, kind=FILE_OCC, rc=rc, commit_tn=tn, seed=seed,
                       tnc_before=tnc)


def calvin_fixture(name, b, seed):
    g, rc, w = orc.calvin(b, literal=True)
    d.write_batch_file(os.path.join(HERE, name), b, kind=FILE_CALVIN, rc=rc, group=g, wave=w,
                       seed=seed)


def history_of(b, tn):
    """(key, tn) of every write of a committed txn (central_finish, occ.cpp:277-286)."""
    off = b.offsets.astype(np.int64)
    txn = np.repeat(np.arange(b.n_txn), np.diff(off))
    sel = (b.acctype == 1) & (tn[txn] > 0)
    return b.keys[sel].copy(), tn[txn][sel].astype(np.uint64)


def main():
    # C1 shape: REQ_PER_QUERY=10, theta 0.6, 64K-row table (config.h:169-177)
    occ_fixture("c1_ycsb_theta06_seed7.dccb",
                d.gen_ycsb(n_txn=4000, zipf_theta=0.6, req_per_query=10, table_size=65536, seed=7),
                seed=7)
    # C2 shape, small: 16 keys, theta 0.9, 16M-row table
    occ_fixture("c2_ycsb_theta09_3000.dccb",
                d.gen_ycsb(n_txn=3000, zipf_theta=0.9, seed=0xD3E7A001), seed=0xD3E7A001)
    # C3 shape, small: TPC-C NewOrder + Payment, 4 warehouses
    occ_fixture("c3_tpcc_4wh_2048.dccb", d.gen_tpcc(n_txn=2048, num_wh=4, seed=0xD3E7A003),
                seed=0xD3E7A003)
    # two epochs with the history window live (TS_CAS-style timestamps): the
    # committed write sets of epoch 0 (tn numbered from tnc_before + 1) form the
    # history epoch 1's windows (start_tn, finish_tn] are checked against
    rng = np.random.default_rng(0xD3E7A004)
    e0 = d.gen_ycsb(n_txn=800, zipf_theta=0.6, table_size=1 << 14, seed=0xD3E7A004)
    rc0, tn0, tnc1 = orc.occ(e0, tnc=100, literal=True)
    d.write_batch_file(os.path.join(HERE, "occ_hist_epoch0.dccb"), e0, kind=FILE_OCC, rc=rc0,
                       commit_tn=tn0, seed=0xD3E7A004, epoch=0, tnc_before=100)
    hk, ht = history_of(e0, tn0)
    e1 = d.gen_ycsb(n_txn=1500, zipf_theta=0.6, table_size=1 << 14, seed=0xD3E7A014)
    e1.start_tn = rng.integers(90, tnc1 + 5, size=e1.n_txn).astype(np.uint64)
    e1.finish_tn = (e1.start_tn + rng.integers(0, 40, size=e1.n_txn)).astype(np.uint64)
    rc1, tn1, _ = orc.occ(e1, hist_keys=hk, hist_tn=ht, tnc=tnc1, literal=True)
    d.write_batch_file(os.path.join(HERE, "occ_hist_epoch1.dccb"), e1, kind=FILE_OCC, rc=rc1,
                       commit_tn=tn1, seed=0xD3E7A014, epoch=1, tnc_before=tnc1)
    # C4 shape, small: Calvin, 16 partitions, sequencer (origin, FIFO) order
    b = d.gen_ycsb(n_txn=2000, zipf_theta=0.9, part_cnt=16, chunk_txns=125, table_size=1 << 14,
                   want_home=True, seed=0xD3E7A005)
    home = b.meta["home"].astype(np.uint64)
    seq = np.zeros(b.n_txn, np.uint64)
    for h in np.unique(home):
        idx = np.nonzero(home == h)[0]
        seq[idx] = np.arange(idx.size, dtype=np.uint64)
    b.order = (home << np.uint64(32)) | seq
    calvin_fixture("c4_calvin_16p_2000.dccb", b, seed=0xD3E7A005)


if __name__ == "__main__":
    main()
