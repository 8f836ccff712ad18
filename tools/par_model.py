#!/usr/bin/env python3
"""CPU model: how deep is the rounds fixed point on the sweep's
later level lists?  For the headline batch, after the level-0 serial range
(p0 txns) and its filter, take the surviving write txns (the level-1 list)
and count (a) its live accesses (an earlier list txn writes the key),
(b) the rounds the fixed point needs when it starts on the whole list, and
(c) how many txns are still undecided after each round.  Uses the oracle's
decisions as the check (checker code)."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def rounds(owner_pos, kid, isw, m):
    """owner_pos: list position of each access; kid: dense key id; isw: write.
    Returns (status per list txn, undecided count after each round)."""
    nk = int(kid.max()) + 1 if kid.size else 0
    st = np.zeros(m, np.int8)  # 0 undecided, 1 commit, 2 abort
    hist = []
    BIG = np.iinfo(np.int64).max
    while (st == 0).any():
        alive_w = isw & (st[owner_pos] != 2)
        o = np.full(nk, BIG, np.int64)
        np.minimum.at(o, kid[alive_w], owner_pos[alive_w])
        ok = o[kid]
        earlier = ok < owner_pos
        com = earlier & (st[np.minimum(ok, m - 1)] == 1)
        blk = earlier & (st[np.minimum(ok, m - 1)] == 0)
        kill = np.zeros(m, bool)
        kill[owner_pos[com]] = True
        block = np.zeros(m, bool)
        block[owner_pos[blk]] = True
        und = st == 0
        st[und & kill] = 2
        st[und & ~kill & ~block] = 1
        hist.append(int((st == 0).sum()))
        if len(hist) > 500:
            break
    return st, hist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--txns", type=int, default=1 << 20)
    ap.add_argument("--theta", type=float, default=0.9)
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0xD3E7A001)
    ap.add_argument("--p0", type=int, default=1024)
    a = ap.parse_args()
    import deneva_amd as d
    import _oracle as orc
    b = d.gen_ycsb(n_txn=a.txns, zipf_theta=a.theta, seed=a.seed)
    rc, _, _ = orc.occ(b)
    n = b.n_txn
    off = np.asarray(b.offsets, np.int64)
    keys = np.asarray(b.keys, np.uint64)
    at = np.asarray(b.acctype)
    owner = np.repeat(np.arange(n), np.diff(off))
    isw = at == d.WR
    hasw = np.zeros(n, bool)
    hasw[owner[isw]] = True
    commit = rc == 0
    ser = np.arange(min(a.p0, n))
    cm = ser[commit[ser] & hasw[ser]]
    cset = np.unique(keys[np.isin(owner, cm) & isw])
    hit = np.zeros(n, bool)
    sel = (owner >= a.p0) & np.isin(keys, cset)
    hit[owner[sel]] = True
    surv = np.arange(a.p0, n)[~hit[a.p0:]]
    lst = surv[hasw[surv]]
    m = lst.size
    pos = np.full(n, -1, np.int64)
    pos[lst] = np.arange(m)
    am = pos[owner] >= 0
    op = pos[owner[am]]
    k = keys[am]
    w = isw[am]
    _, kid = np.unique(k, return_inverse=True)
    # live accesses: an earlier list txn writes the key
    nk = int(kid.max()) + 1
    fw = np.full(nk, np.iinfo(np.int64).max, np.int64)
    np.minimum.at(fw, kid[w], op[w])
    live = fw[kid] < op
    ntx_live = np.unique(op[live]).size
    print(f"level-1 list: {m} write txns, {op.size} accesses, {nk} keys, "
          f"live accesses {int(live.sum())}, txns with a live access {ntx_live}")
    st, hist = rounds(op, kid, w, m)
    ok = np.array_equal(st == 1, commit[lst])
    print(f"rounds {len(hist)}, parity vs oracle {ok}")
    print("undecided after each round:", hist[:60])


if __name__ == "__main__":
    main()
