#!/usr/bin/env python3
"""CPU model of a data-parallel Calvin wave computation.

wave(t) = 1 + max over t's rows of the largest wave in the group before t's
group on that row (0 with no such group) -- oracle_calvin_formula's rule
(row_lock.cpp:317-357 released in waves).  The model iterates, from wave = 0:

  1. per (row, group) node G: W(G) = max wave of its members;
  2. per row, along its groups: M(g) = max(W(g), M(g-1) + 1) -- a max-plus
     scan, so a row's chain is propagated whole in one iteration;
  3. per txn: wave(t) = max over its rows of M(g_r(t) - 1) + 1.

Every step keeps each value a lower bound of the true waves, and a fixed point
is the true waves, so the iteration count is the longest run of row changes on
a critical path.  Prints the count per batch and checks the result against
the oracle's waves.
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def model(b, verbose=True):
    import _oracle as orc
    g, rc, wv = orc.calvin(b)
    n = b.n_txn
    off = np.asarray(b.offsets, np.int64)
    keys = np.asarray(b.keys, np.uint64)
    at = np.asarray(b.acctype, np.uint8)
    txn = np.repeat(np.arange(n, dtype=np.int64), np.diff(off))
    live = g != np.uint32(0xFFFFFFFF)
    k, gg, tt = keys[live], g[live].astype(np.int64), txn[live]
    o = np.lexsort((gg, k))
    k, gg, tt = k[o], gg[o], tt[o]
    # node = (row, group) runs
    newnode = np.ones(k.size, bool)
    newnode[1:] = (k[1:] != k[:-1]) | (gg[1:] != gg[:-1])
    node = np.cumsum(newnode) - 1
    nn = int(node[-1]) + 1
    nrow = k[newnode]
    ngrp = gg[newnode]
    rowstart = np.ones(nn, bool)
    rowstart[1:] = nrow[1:] != nrow[:-1]
    # predecessor node of each request's node (or -1)
    pred = node - 1
    pred[rowstart[node]] = -1
    wave = np.zeros(n, np.int64)
    it = 0
    seg_id = np.cumsum(rowstart) - 1
    t0 = time.time()
    while True:
        it += 1
        W = np.full(nn, -1, np.int64)
        np.maximum.at(W, node, wave[tt])
        # max-plus scan along each row: M(g) = max(W(g), M(g-1)+1)
        # = max over g' <= g in the row of W(g') + (g - g'); with idx = node
        # position: M = max_{g'} (W(g') - idx') + idx, a segmented running max
        idx = np.arange(nn, dtype=np.int64)
        v = W - idx
        # segmented cumulative max: offset each segment so segments don't mix
        big = np.int64(1) << 40
        vv = v + seg_id * big
        M = np.maximum.accumulate(vv) - seg_id * big + idx
        cand = np.where(pred >= 0, M[np.maximum(pred, 0)] + 1, 0)
        nw = np.zeros(n, np.int64)
        np.maximum.at(nw, tt, cand)
        if np.array_equal(nw, wave):
            break
        wave = nw
    ok = np.array_equal(wave.astype(np.uint32), wv)
    if verbose:
        print(f"n={n} nodes={nn} max_wave={int(wv.max())} iterations={it} "
              f"matches_oracle={ok} ({time.time() - t0:.1f} s)")
    return it, ok


if __name__ == "__main__":
    from helpers import c4_batch
    import deneva_amd as d
    for nt in (1 << 16, 1 << 18):
        model(c4_batch(nt))
    model(c4_batch())
