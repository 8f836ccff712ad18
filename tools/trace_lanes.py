#!/usr/bin/env python3
"""Per-lane timeline of a pipelined headline trace (rocprofv3 kernel trace
CSV of bench.py --pipeline L): for each lane queue, epochs cut at k_fill;
per kernel name the mean duration and the mean gap between the end of the
previous kernel of the same queue and this kernel's start (dispatch +
dependency latency), against the same figures of the single-epoch queue.
Usage: trace_lanes.py <kernel_trace.csv>"""
import csv
import sys
from collections import Counter, defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"].split("(")[0])
          for r in rows if "dcc::" in r["Kernel_Name"]]
    ev.sort()
    byq = defaultdict(list)
    for e in ev:
        byq[e[2]].append(e)
    fills = Counter(q for _, _, q, n in ev if "k_fill" in n)
    for q, es in sorted(byq.items()):
        if fills[q] < 2:
            continue
        dur, gap, cnt = defaultdict(float), defaultdict(float), Counter()
        spans = []
        t_ep = None
        prev_end = None
        for s, e, _, n in es:
            if "k_fill" in n:
                if t_ep is not None:
                    spans.append(prev_end - t_ep)
                t_ep = s
            else:
                if prev_end is not None:
                    gap[n] += s - prev_end
            dur[n] += e - s
            cnt[n] += 1
            prev_end = e
        tot_d = sum(dur.values()) / max(1, fills[q])
        tot_g = sum(gap.values()) / max(1, fills[q])
        print(f"queue {q}: {fills[q]} epochs, per epoch kernels {tot_d / 1e3:.1f} us, gaps {tot_g / 1e3:.1f} us, "
              f"mean span {sum(spans) / max(1, len(spans)) / 1e3:.1f} us")
        for n in sorted(dur, key=lambda n: -dur[n]):
            print(f"   {n[:28]:28s} x{cnt[n] / fills[q]:.1f}  dur {dur[n] / cnt[n] / 1e3:7.2f} us  "
                  f"gap before {gap[n] / cnt[n] / 1e3:6.2f} us")


if __name__ == "__main__":
    main()
