#!/usr/bin/env python3
"""Compact table of a rocprofv3 kernel_stats.csv: name, calls, avg / max us.
    kstats.py <dir or csv> [top]"""
import csv
import glob
import os
import sys

p = sys.argv[1]
if os.path.isdir(p):
    p = glob.glob(os.path.join(p, "**", "*kernel_stats.csv"), recursive=True)[0]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
for r in list(csv.DictReader(open(p)))[:top]:
    name = r["Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    print(f"{name[-44:]:44s} {r['Calls']:>5s} avg {float(r['AverageNs']) / 1e3:8.1f} us"
          f"  max {float(r['MaxNs']) / 1e3:8.1f}  total {float(r['TotalDurationNs']) / 1e3:9.1f}")
