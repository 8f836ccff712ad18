"""Sweep epochs of the headline batch (1M YCSB theta=0.9 txns): driver for
DCC_SW_DEBUG clock stamps and per-dispatch PMC passes (tools/gpu_pmc_sweep.sh);
the last line is the median device ms over the repeats and the level count."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import deneva_amd as d  # noqa: E402

b = d.gen_ycsb(n_txn=1 << 20, zipf_theta=0.9)
db = b.to_torch("cuda:0")
reps = 2 if os.environ.get("DCC_SW_DEBUG") else 12
with d.Engine(0) as e:
    ms = []
    for _ in range(reps):
        rc, _, st = e.occ_validate_epoch(db)
        ms.append(st["device_ms"])
    ms.sort()
    print(ms[len(ms) // 2], st["rounds"])
