#!/usr/bin/env python3
"""Summarise tools/gpu_pmc_r05.sh's passes into the JSON bench.py reads
(profiles/r05/pmc.json).  Per workload: the HBM-side traffic of one epoch
(FETCH_SIZE x2 -- gfx950 counts 128-B requests at 64 B, MI355X_MICROARCH.md
HBM section -- plus WRITE_SIZE), the epoch's L2 hit rate (TCC_HIT_sum /
(TCC_HIT_sum + TCC_MISS_sum)) and per kernel the same, median over the
measured epochs (the first epoch of each workload, a warm-up / graph
capture, is dropped).

An epoch is the dispatches from a start kernel up to its workload's last
kernel (the last end kernel before the next start): a workload's epoch never
absorbs the next workload's first launches (round 4 split at the next start
kernel, so the last C5 epoch took in MaaT's row-table clear).  The passes of
`--only C2,C3,C5,MAAT_1M` run the workloads back to back, W + S epochs each
(bench.py's warm-up + steps), so consecutive OCC epochs are split by count.
    pmc_r04.py <pass dir root> <out json>"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

PER = 3  # epochs per workload in the passes (--warmup 1 --steps 2)


def dispatches(root, name):
    per = defaultdict(lambda: defaultdict(float))
    kname = {}
    for f in glob.glob(os.path.join(root, name, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            d = int(r["Dispatch_Id"])
            per[d][r["Counter_Name"]] += float(r["Counter_Value"])
            kname[d] = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    return [(kname[d], per[d]) for d in sorted(per)]


def split(disp, starts, ends):
    """Epochs: [(start kernel, [(kernel, counters)])], each from a dispatch
    whose name holds one of `starts` through the last dispatch before the next
    start whose name holds one of `ends` (dispatches after it are dropped)."""
    out = []
    for k, c in disp:
        s = next((x for x in starts if x in k), None)
        if s:
            out.append([s, [], 0])
        if out:
            out[-1][1].append((k, c))
            if any(e in k for e in ends):
                out[-1][2] = len(out[-1][1])
    return [(s, ks[:last]) for s, ks, last in out if last]


def summarise(fe, wr, l2):
    """fe / wr / l2: lists of epochs (each [(kernel, counters)]), the
    warm-up epoch already dropped."""
    f = [2 * 1024 * sum(c.get("FETCH_SIZE", 0.0) for _, c in e) for e in fe]
    w = [1024 * sum(c.get("WRITE_SIZE", 0.0) for _, c in e) for e in wr]
    n = min(len(f), len(w))

    def hit(pairs):
        h = sum(a for a, _ in pairs)
        m = sum(b for _, b in pairs)
        return h / (h + m) if h + m else None

    kern = defaultdict(lambda: {"fetch": [], "write": [], "l2": []})
    for e in fe:
        acc = defaultdict(float)
        for k, c in e:
            acc[k] += 2 * 1024 * c.get("FETCH_SIZE", 0.0)
        for k, v in acc.items():
            kern[k]["fetch"].append(v)
    for e in wr:
        acc = defaultdict(float)
        for k, c in e:
            acc[k] += 1024 * c.get("WRITE_SIZE", 0.0)
        for k, v in acc.items():
            kern[k]["write"].append(v)
    for e in l2:
        for k, c in e:
            kern[k]["l2"].append((c.get("TCC_HIT_sum", 0.0), c.get("TCC_MISS_sum", 0.0)))
    med = lambda v: statistics.median(v) if v else 0.0
    ep_l2 = [hit([(c.get("TCC_HIT_sum", 0.0), c.get("TCC_MISS_sum", 0.0)) for _, c in e]) for e in l2]
    ep_l2 = [x for x in ep_l2 if x is not None]
    return {
        "epoch_bytes": statistics.median([f[i] + w[i] for i in range(n)]) if n else None,
        "epoch_fetch_bytes": med(f) if f else None,
        "epoch_write_bytes": med(w) if w else None,
        "epoch_l2_hit": statistics.median(ep_l2) if ep_l2 else None,
        "epochs": n,
        "kernels": {k: {"fetch_bytes": med(v["fetch"]), "write_bytes": med(v["write"]),
                        "l2_hit": hit(v["l2"])} for k, v in kern.items()},
    }


def workloads(root, prefix, plan, ends):
    """plan: [(name, start kernel)] in run order, PER epochs each; ends: the
    workloads' last kernels."""
    passes = {}
    for p in ("fetch", "write", "l2"):
        eps = split(dispatches(root, f"{prefix}_{p}"), sorted({s for _, s in plan}), ends)
        passes[p] = eps
    out = {}
    cur = {p: 0 for p in passes}
    for name, start in plan:
        got = {}
        for p, eps in passes.items():
            mine = []
            i = cur[p]
            while i < len(eps) and len(mine) < PER:
                if eps[i][0] == start:
                    mine.append(eps[i][1])
                i += 1
            cur[p] = i
            got[p] = mine[1:] if len(mine) > 1 else mine
        out[name] = summarise(got["fetch"], got["write"], got["l2"])
    return out


def main():
    root, dst = sys.argv[1], sys.argv[2]
    res = {"source": "rocprofv3 --kernel-trace --pmc, one pass per counter set (tools/gpu_pmc_r05.sh)",
           "correction": "FETCH_SIZE x2 (gfx950: 128-B requests counted at 64 B); "
                         "l2_hit = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum); an epoch ends at its "
                         "workload's last kernel"}
    occ_end = ("k_final", "k_fin_apply")
    res.update(workloads(root, "h", [("headline", "k_fill")], occ_end))
    res.update(workloads(root, "c4", [("C4", "k_cv_prep")], ("k_cb_put", "k_cv_ready")))
    res.update(workloads(root, "s", [("C2", "k_fill"), ("C3", "k_fill"), ("C5", "k_fill"),
                                     ("MAAT_1M", "k_mt_check")], occ_end + ("k_mt_finish",)))
    os.makedirs(os.path.dirname(os.path.abspath(dst)), exist_ok=True)
    json.dump(res, open(dst, "w"), indent=1)
    for k in ("headline", "C2", "C3", "C4", "C5", "MAAT_1M"):
        v = res.get(k) or {}
        eb = v.get("epoch_bytes")
        print(f"{k:9s} epoch traffic {eb / 1e6 if eb else float('nan'):9.1f} MB  l2 hit {v.get('epoch_l2_hit')}  "
              f"epochs {v.get('epochs')}")


if __name__ == "__main__":
    main()
