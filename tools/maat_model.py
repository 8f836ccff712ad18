#!/usr/bin/env python3
"""CPU model of the MaaT round solver: rounds to convergence
with the current blocking rule (any undecided earlier writer of a row the txn
touches, or undecided earlier reader of a row it writes, blocks it) and with
a refined rule that ignores undecided predecessors whose commit could not
change the decision:

  an undecided writer j (cts_j >= Llo_j) lowers U_i only to cts_j - 1 >= Llo_j - 1,
  so it matters only if Llo_j <= L_i + 1;
  an undecided reader j (cts_j < U_j) raises L_i only if cts_j + 1 > L_i,
  so it matters only if U_j > L_i.

Both rules are exact (decisions equal the serial formula, checked against
the oracle); the model counts rounds.  Empty row table (base = 1).

    python tools/maat_model.py [--txns N]"""
import argparse
import os
import sys

import numpy as np
import pandas as pd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

INF = 1 << 50  # exact in float64 (pandas shift goes through NaN)


def run(g_row, g_txn, g_r, g_w, n, refined):
    st = np.zeros(n, np.int8)  # 0 und, 1 com, 2 abo
    cts = np.zeros(n, np.int64)
    llo = np.ones(n, np.int64)       # known lower bound (base = 1)
    uhi = np.full(n, INF, np.int64)  # known upper bound
    rounds = []
    first = np.r_[True, g_row[1:] != g_row[:-1]]
    seg = np.cumsum(first) - 1
    while (st == 0).any():
        s = st[g_txn]
        com, und = s == 1, s == 0
        rmax = np.where(com & g_r, cts[g_txn], 0)
        wmin = np.where(com & g_w, cts[g_txn], INF)
        wlo = np.where(und & g_w, llo[g_txn], INF)
        rhi = np.where(und & g_r, uhi[g_txn], -1)
        df = pd.DataFrame({"s": seg, "rmax": rmax, "wmin": wmin, "wlo": wlo, "rhi": rhi})
        gb = df.groupby("s", sort=False)
        ex = pd.DataFrame({"rmax": gb["rmax"].cummax(), "wmin": gb["wmin"].cummin(),
                           "wlo": gb["wlo"].cummin(), "rhi": gb["rhi"].cummax()})
        ex = ex.groupby(seg, sort=False).shift(1)  # exclusive within the row
        e_rmax = ex["rmax"].fillna(0).to_numpy(np.int64)
        e_wmin = ex["wmin"].fillna(INF).to_numpy(np.int64)
        e_wlo = ex["wlo"].fillna(INF).to_numpy(np.int64)
        e_rhi = ex["rhi"].fillna(-1).to_numpy(np.int64)
        lacc = np.ones(n, np.int64)
        np.maximum.at(lacc, g_txn[g_w], np.where(e_rmax[g_w] > 0, e_rmax[g_w] + 1, 0))
        uacc = np.full(n, INF, np.int64)
        v = np.where(e_wmin < INF, e_wmin - 1, INF)
        np.minimum.at(uacc, g_txn, v)
        minw = np.full(n, INF, np.int64)
        np.minimum.at(minw, g_txn, e_wlo)
        maxr = np.full(n, -1, np.int64)
        np.maximum.at(maxr, g_txn[g_w], e_rhi[g_w])
        L, U = lacc, uacc
        if refined:
            blocked = (minw <= L + 1) | (maxr > L)
        else:
            blocked = (minw < INF) | (maxr >= 0)
        u = st == 0
        ab = u & (L >= U)
        cm = u & ~ab & ~blocked
        st[ab] = 2
        st[cm] = 1
        cts[cm] = L[cm]
        llo = np.where(u, np.maximum(llo, L), llo)
        uhi = np.where(u, np.minimum(uhi, U), uhi)
        rounds.append(int((st == 0).sum()))
        if len(rounds) > 400:
            break
    return st, cts, rounds


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--txns", type=int, default=65536)
    a = ap.parse_args()
    import deneva_amd as d
    import _oracle as orc
    b = d.gen_ycsb(n_txn=a.txns, zipf_theta=0.9)
    erc, ects, _ = orc.maat(b)
    n = b.n_txn
    off = np.asarray(b.offsets, np.int64)
    keys = np.asarray(b.keys, np.uint64)
    at = np.asarray(b.acctype)
    owner = np.repeat(np.arange(n), np.diff(off))
    # (row, txn) groups with their R / W bits, sorted by row then txn
    df = pd.DataFrame({"k": keys, "t": owner, "r": at == d.RD, "w": at == d.WR})
    g = df.groupby(["k", "t"], sort=True).agg(r=("r", "any"), w=("w", "any")).reset_index()
    g_row = pd.factorize(g["k"])[0]
    g_txn = g["t"].to_numpy(np.int64)
    g_r = g["r"].to_numpy()
    g_w = g["w"].to_numpy()
    for refined in (False, True):
        st, cts, rounds = run(g_row, g_txn, g_r, g_w, n, refined)
        ok = np.array_equal(st == 1, erc == 0) and np.array_equal(np.where(st == 1, cts, 0),
                                                                  np.asarray(ects, np.int64))
        print(f"{'refined' if refined else 'current'}: rounds {len(rounds)}, parity {ok}, "
              f"undecided per round {rounds[:50]}")


if __name__ == "__main__":
    main()
