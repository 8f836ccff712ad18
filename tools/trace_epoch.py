#!/usr/bin/env python3
"""Print the kernel timeline of one OCC epoch from a rocprofv3 kernel trace
(csv): every dispatch of the epoch, with its duration and the idle gap before
it.  An epoch ends with the k_stage_final dispatch (stage solver) or starts
with k_fill (k_fill_prep / k_prep in older builds).

    trace_epoch.py <kernel_trace.csv> [epoch_index]   (default: the second to last)
"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "k_stage_final" in r["Kernel_Name"]]
    if ends:
        bounds = [(ends[i - 1] + 1 if i else 0, ends[i] + 1) for i in range(len(ends))]
    else:
        starts = [i for i, r in enumerate(rows) if any(k in r["Kernel_Name"] for k in ("k_prep", "k_fill", "k_cv_prep"))]
        bounds = [(s, starts[i + 1] if i + 1 < len(starts) else len(rows)) for i, s in enumerate(starts)]
    e = int(sys.argv[2]) if len(sys.argv) > 2 else max(0, len(bounds) - 2)
    a, b = bounds[e]
    t0 = int(rows[a]["Start_Timestamp"])
    prev_end = t0
    busy = 0
    for r in rows[a:b]:
        s, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0][:60]
        print(f"{(s - t0) / 1e3:9.1f} us  gap {(s - prev_end) / 1e3:7.1f}  dur {(en - s) / 1e3:8.1f}  "
              f"grid {r.get('Grid_Size_X', r.get('Grid_Size', '?')):>8}  {name}")
        busy += en - s
        prev_end = en
    print(f"epoch span {(prev_end - t0) / 1e3:.1f} us, kernels busy {busy / 1e3:.1f} us")


if __name__ == "__main__":
    main()
