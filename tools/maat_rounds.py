#!/usr/bin/env python3
"""MaaT 1M epoch with DCC_MT_DEBUG=1: undecided txns and scan length per round
(stderr), device ms per epoch.  Run on the GPU box."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import deneva_amd as d  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
b = d.gen_ycsb(n_txn=n, zipf_theta=0.9)
db = b.to_torch("cuda:0")
rc = torch.empty(n, dtype=torch.uint8, device="cuda:0")
EP = int(os.environ.get("EPOCHS", "2"))
dev = []
with d.Engine(0) as eng:
    for i in range(EP):
        eng.maat_rows_clear()
        st = eng.maat_validate_epoch(db, want_cts=False, out_rc=rc)[2]
        print(f"epoch {i}: device {st['device_ms']:.3f} ms, rounds {st['rounds']}, commits {st['n_commit']}",
              file=sys.stderr, flush=True)
        dev.append(st['device_ms'])
if EP > 2:
    import statistics
    print(f"median of epochs 1..: {statistics.median(dev[1:]):.3f} ms", file=sys.stderr, flush=True)
