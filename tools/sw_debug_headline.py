#!/usr/bin/env python3
"""Serial-pass / filter / pre-pass stamps of the headline epoch (DCC_SW_DEBUG:
the driver prints per-level loop cycles per tile, candidates and fixed-point
rounds per tile, waits, pre-pass phases).  Run on the GPU box:
    DCC_SW_DEBUG=1 python tools/sw_debug_headline.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import deneva_amd as d  # noqa: E402

b = d.gen_ycsb(n_txn=1 << 20, zipf_theta=0.9)
db = b.to_torch("cuda:0")
with d.Engine(0) as eng:
    for i in range(3):
        _, _, st = eng.occ_validate_epoch(db)
        print(f"epoch {i}: {st['device_ms']:.4f} ms, commits {st['n_commit']}", file=sys.stderr, flush=True)
