#!/usr/bin/env python3
"""Per-round undecided counts and scan lengths of a MaaT epoch (DCC_MT_DEBUG=1)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import deneva_amd as d  # noqa: E402
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
b = d.gen_ycsb(n_txn=n, zipf_theta=0.9)
with d.Engine(0) as eng:
    eng.maat_rows_clear()
    _, _, st = eng.maat_validate_epoch(b, want_cts=False)
    print(f"{st['device_ms']:.3f} ms, {st['rounds']} rounds, {st['n_commit']} commits", file=sys.stderr)
