#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace of the pipelined headline
(bench.py --pipeline L): per queue the kernels it ran, the busy time against
the sum of the kernels' durations (> 1 means kernels of different lanes ran
at the same time), and the time with 1, 2, 3... kernels in flight -- over
the whole trace and over the lanes' queues alone (the queues that ran more
than one epoch's k_fill besides the main stream's).
Usage: trace_overlap.py <kernel_trace.csv> [name-filter]"""
import csv
import sys
from collections import Counter


def summary(ev, title):
    if not ev:
        print(title, "no kernels")
        return
    ev.sort()
    # the pipelined section: the longest stretch in which more than one queue ran
    qs = Counter(q for _, _, q, _ in ev)
    t0, t1 = ev[0][0], max(e for _, e, _, _ in ev)
    pts = sorted([(s, 1) for s, _, _, _ in ev] + [(e, -1) for _, e, _, _ in ev])
    depth, last, hist = 0, t0, Counter()
    for t, d in pts:
        if t > last:
            hist[depth] += t - last
        depth += d
        last = t
    busy = sum(v for k, v in hist.items() if k > 0)
    work = sum(e - s for s, e, _, _ in ev)
    print(f"{title}: kernels {len(ev)} on {len(qs)} queues: " + ", ".join(f"q{q}:{n}" for q, n in sorted(qs.items())))
    print(f"span {(t1 - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us, kernel time {work / 1e3:.1f} us, "
          f"overlap factor {work / max(busy, 1):.2f}")
    for k in sorted(hist):
        if k:
            print(f"  {k} kernels in flight: {hist[k] / 1e3:9.1f} us ({hist[k] / max(busy, 1):.0%} of busy)")


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    flt = sys.argv[2] if len(sys.argv) > 2 else "dcc::"
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"])
          for r in rows if flt in r["Kernel_Name"]]
    summary(ev, "whole trace")
    fills = Counter(q for _, _, q, n in ev if "k_fill" in n)
    main_q = Counter(q for _, _, q, _ in ev).most_common(1)[0][0] if ev else None
    lanes = {q for q, k in fills.items() if k > 1 and q != main_q}
    summary([x for x in ev if x[2] in lanes], f"pipeline lanes {sorted(lanes)}")


if __name__ == "__main__":
    main()
