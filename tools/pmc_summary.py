#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools/gpu_pmc.sh output): per kernel,
the mean of every collected counter per dispatch.  Usage:
pmc_summary.py <pmc dir> [kernel substring ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    want = sys.argv[2:]
    acc = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        rows = list(csv.DictReader(open(f)))
        per = defaultdict(float)
        names = {}
        for r in rows:
            k = (r["Dispatch_Id"], r["Counter_Name"])
            per[k] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
        for (disp, cn), v in per.items():
            kn = names[disp].replace("(anonymous namespace)::", "").split("(")[0]
            acc[kn][cn].append(v)
    for kn in sorted(acc):
        if want and not any(w in kn for w in want):
            continue
        print(kn)
        for cn in sorted(acc[kn]):
            vals = acc[kn][cn]
            print(f"    {cn:28s} mean {sum(vals) / len(vals):16.1f}   n {len(vals)}")


if __name__ == "__main__":
    main()
