#!/usr/bin/env python3
"""HBM traffic per launch of the roofline kernel from rocprofv3 --pmc passes
(tools/gpu_pmc.sh): FETCH_SIZE and WRITE_SIZE (kilobytes, one pass each),
mean over the kernel's level-0 dispatches (the largest grid).  gfx950
correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts 128-B
requests at 64 B, so it is doubled.  Writes profiles/traffic.json for
bench.py (key "<txns>:<theta>:<keys>:<kernel>") and prints the summary.
Usage: traffic.py <pmc dir> <kernel substring> <key> [traffic.json]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def per_dispatch(root, want):
    out = defaultdict(dict)  # (pass, dispatch) -> counters
    for f in sorted(glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"),
                              recursive=True)):
        pas = f.split(os.sep)[len(root.rstrip(os.sep).split(os.sep))]
        for r in csv.DictReader(open(f)):
            if want not in r["Kernel_Name"]:
                continue
            d = out[(pas, int(r["Dispatch_Id"]))]
            d["grid"] = int(r.get("Grid_Size", 0) or 0)
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def main():
    root, want, key = sys.argv[1], sys.argv[2], sys.argv[3]
    rows = per_dispatch(root, want)
    vals = defaultdict(list)
    gmax = max((d["grid"] for d in rows.values()), default=0)
    for (_, _), d in rows.items():
        if d["grid"] != gmax:
            continue
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            if c in d:
                vals[c].append(d[c])
    if not vals.get("FETCH_SIZE") or not vals.get("WRITE_SIZE"):
        raise SystemExit("no FETCH_SIZE / WRITE_SIZE for " + want)
    fetch_kb = sum(vals["FETCH_SIZE"]) / len(vals["FETCH_SIZE"])
    write_kb = sum(vals["WRITE_SIZE"]) / len(vals["WRITE_SIZE"])
    fetch = 2.0 * fetch_kb * 1024.0  # gfx950: FETCH_SIZE is half the bytes read
    write = write_kb * 1024.0
    summary = {"kernel": want, "grid": gmax, "dispatches": len(vals["FETCH_SIZE"]),
               "FETCH_SIZE_kB": fetch_kb, "WRITE_SIZE_kB": write_kb,
               "read_bytes_corrected": fetch, "write_bytes": write,
               "traffic_bytes": fetch + write}
    print(json.dumps(summary, indent=1))
    tf = sys.argv[4] if len(sys.argv) > 4 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "traffic.json")
    tj = json.load(open(tf)) if os.path.exists(tf) else {}
    tj[key] = fetch + write
    tj[key + ":detail"] = summary
    json.dump(tj, open(tf, "w"), indent=1)


if __name__ == "__main__":
    main()
