#!/usr/bin/env python3
"""Per-dispatch PMC table from rocprofv3 --pmc passes (one directory per pass,
same program each pass): one row per dispatch of the matching kernels, in
dispatch order, all counters side by side.  Usage:
pmc_dispatch.py <pmc dir> <kernel substring> [last_n]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    root, want = sys.argv[1], sys.argv[2]
    last = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    cols, table = [], defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True)):
        per, names = defaultdict(float), {}
        for r in csv.DictReader(open(f)):
            per[(int(r["Dispatch_Id"]), r["Counter_Name"])] += float(r["Counter_Value"])
            names[int(r["Dispatch_Id"])] = r["Kernel_Name"].split("(")[0]
        seq = [d for d in sorted(names) if want in names[d]]
        for i, d in enumerate(seq):
            for (dd, cn), v in per.items():
                if dd == d:
                    table[i][cn] = v
                    table[i]["_k"] = names[d]
                    if cn not in cols:
                        cols.append(cn)
    rows = sorted(table)[-last:]
    print("idx kernel " + " ".join(f"{c[:14]:>14s}" for c in cols))
    for i in rows:
        print(f"{i:3d} {table[i]['_k'][-14:]:14s} " +
              " ".join(f"{table[i].get(c, 0):14.0f}" for c in cols))


if __name__ == "__main__":
    main()
