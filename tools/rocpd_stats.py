#!/usr/bin/env python3
"""Per-kernel duration summary (the --stats table) from a rocprofv3 rocpd
database: name, calls, total / average / min / max ns, percentage.
Usage: rocpd_stats.py <results.db> [out.csv]"""
import csv
import sqlite3
import sys
from collections import defaultdict


def main():
    c = sqlite3.connect(sys.argv[1])
    d = defaultdict(list)
    for name, dur in c.execute("select name, duration from kernels"):
        d[name].append(int(dur))
    tot = sum(sum(v) for v in d.values()) or 1
    rows = sorted(d.items(), key=lambda kv: -sum(kv[1]))
    out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.writer(out)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, v in rows:
        w.writerow([name, len(v), sum(v), f"{sum(v) / len(v):.1f}", f"{100 * sum(v) / tot:.2f}", min(v), max(v)])


if __name__ == "__main__":
    main()
