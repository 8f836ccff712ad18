#!/usr/bin/env python3
"""HBM traffic of one whole OCC epoch from rocprofv3 --pmc passes
(tools/gpu_pmc_epoch.sh): FETCH_SIZE and WRITE_SIZE (kB, one pass each)
summed over every dispatch of an epoch (an epoch = the dispatches from one
k_fill (k_fill_prep / k_prep in older builds) to the next), median over the run's epochs.  gfx950 correction
(MI355X_MICROARCH.md, HBM / rocprofv3 section): FETCH_SIZE counts 128-B
requests at 64 B, so it is doubled.  Also reports the level-0 filter alone.
Writes <out json>[key] = {"bytes_per_epoch", "source", ...} for bench.py.
Usage: epoch_traffic.py <pmc dir> <key> <out json> <source label>"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict


def load(root, pas):
    rows = []
    for f in glob.glob(os.path.join(root, pas, "**", "*counter_collection.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    per = defaultdict(lambda: {"name": "", "v": 0.0})
    for r in rows:
        d = per[int(r["Dispatch_Id"])]
        d["name"] = r["Kernel_Name"]
        d["v"] += float(r["Counter_Value"])
    return [per[k] for k in sorted(per)]


def epochs(disp):
    out, cur = [], None
    for d in disp:
        if "k_prep" in d["name"] or "k_fill" in d["name"]:
            if cur:
                out.append(cur)
            cur = []
        if cur is not None:
            cur.append(d)
    if cur:
        out.append(cur)
    return out


def main():
    root, key, out, src = sys.argv[1:5]
    fe = epochs(load(root, "fetch"))
    wr = epochs(load(root, "write"))
    n = min(len(fe), len(wr))
    if n == 0:
        raise SystemExit("no epochs found")
    tot = [2.0 * sum(d["v"] for d in fe[i]) * 1024 + sum(d["v"] for d in wr[i]) * 1024 for i in range(n)]
    filt = []
    for i in range(n):
        # the epoch's first filter dispatch is level 0's
        f = [d["v"] for d in fe[i] if "k_sw_filter" in d["name"]]
        w = [d["v"] for d in wr[i] if "k_sw_filter" in d["name"]]
        if f and w:
            filt.append(2.0 * f[0] * 1024 + w[0] * 1024)
    res = {"bytes_per_epoch": statistics.median(tot), "epochs": n,
           "filter_bytes_per_launch": statistics.median(filt) if filt else None,
           "source": src, "correction": "FETCH_SIZE x2 (gfx950 128-B requests counted at 64 B)"}
    tj = json.load(open(out)) if os.path.exists(out) else {}
    tj[key] = res
    os.makedirs(os.path.dirname(out), exist_ok=True)
    json.dump(tj, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
