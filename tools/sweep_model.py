#!/usr/bin/env python3
"""CPU model of the sweep's level structure for a batch: per
level the list length, the serially decided txns, commits and survivors.

    python tools/sweep_model.py [--txns N] [--theta T] [--split-ro] [--pmax 1024,2048,...]

--split-ro models read-only txns kept out of the level lists after the
level-0 filter (they are decided at the end against the first committed
writer of each key).  Uses the oracle's decisions (checker code), so the
model is exact about which txns commit."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--txns", type=int, default=1 << 20)
    ap.add_argument("--theta", type=float, default=0.9)
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0xD3E7A001)
    ap.add_argument("--split-ro", action="store_true")
    ap.add_argument("--mixed-l0", action="store_true",
                    help="with --split-ro: level 0's serial range is its first p positions "
                         "(read-only txns included), later levels hold write txns only")
    ap.add_argument("--pmax", default="1024,2048,4096,8192,16384,32768")
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
    pm = [int(x) for x in a.pmax.split(",")]
    lst = np.arange(n)
    lvl = 0
    ro_def = 0
    tot_serial = 0
    while lst.size:
        p = pm[min(lvl, len(pm) - 1)]
        if a.split_ro and lvl > 0:
            cand = lst
        else:
            cand = lst
        if a.split_ro and not (a.mixed_l0 and lvl == 0):
            wpos = np.nonzero(hasw[cand])[0]
            if wpos.size <= p:
                ser_end = cand.size
            else:
                ser_end = wpos[p - 1] + 1
            ser = cand[:ser_end]
            nser_w = int(hasw[ser].sum())
        else:
            ser_end = min(p, cand.size)
            ser = cand[:ser_end]
            nser_w = int(hasw[ser].sum())
        cm = ser[commit[ser] & hasw[ser]]
        cset = np.unique(keys[np.isin(owner, cm) & isw])
        rest = cand[ser_end:]
        if rest.size:
            m = np.isin(owner, rest)
            hit = np.zeros(n, bool)
            sel = m & np.isin(keys, cset)
            hit[owner[sel]] = True
            surv = rest[~hit[rest]]
        else:
            surv = rest
        if a.split_ro:
            ro = surv[~hasw[surv]]
            ro_def += ro.size
            surv = surv[hasw[surv]]
        tot_serial += nser_w if (a.split_ro and not (a.mixed_l0 and lvl == 0)) else ser.size
        print(f"level {lvl}: list {cand.size:8d}  serial {ser.size:6d} (write txns {nser_w:6d}, "
              f"commits {int(commit[ser].sum()):5d})  |C| {cset.size:6d}  survivors {surv.size:7d}"
              + (f"  RO deferred so far {ro_def}" if a.split_ro else ""))
        lst = surv
        lvl += 1
    print(f"levels {lvl}, serially decided {tot_serial}, commits {int(commit.sum())}, "
          f"write-txn commits {int((commit & hasw).sum())}")


if __name__ == "__main__":
    main()
