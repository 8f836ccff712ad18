#!/usr/bin/env python3
"""Per-kernel PMC summary of tools/gpu_df_diag.sh's passes: median per
dispatch of FETCH_SIZE x2 (gfx950 tallies 128-B requests at 64 B,
MI355X_MICROARCH.md HBM section), WRITE_SIZE (KB) and the L2 hit rate.
    pmc_kernels.py <pass dir root>"""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def per_kernel(root, name):
    per = defaultdict(lambda: defaultdict(float))
    kname = {}
    for f in glob.glob(os.path.join(root, name, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            d = int(r["Dispatch_Id"])
            per[d][r["Counter_Name"]] += float(r["Counter_Value"])
            kname[d] = r["Kernel_Name"].split("(")[0].replace("void ", "")
    out = defaultdict(list)
    for d in per:
        out[kname[d]].append(per[d])
    return out


def main():
    root = sys.argv[1]
    fe, wr, l2 = per_kernel(root, "fetch"), per_kernel(root, "write"), per_kernel(root, "l2")
    print(f"{'kernel':32s} {'fetch MB':>9s} {'write MB':>9s} {'L2 hit':>7s}")
    for k in sorted(fe, key=lambda k: -statistics.median(x.get("FETCH_SIZE", 0) for x in fe[k])):
        f = statistics.median(x.get("FETCH_SIZE", 0) for x in fe[k]) * 2 / 1024
        w = statistics.median(x.get("WRITE_SIZE", 0) for x in wr.get(k, [{}])) / 1024
        h = [x.get("TCC_HIT_sum", 0) for x in l2.get(k, [])]
        m = [x.get("TCC_MISS_sum", 0) for x in l2.get(k, [])]
        hr = statistics.median(a / (a + b) if a + b else 0 for a, b in zip(h, m)) if h else 0
        print(f"{k[:32]:32s} {f:9.1f} {w:9.1f} {hr:7.3f}")


if __name__ == "__main__":
    main()
