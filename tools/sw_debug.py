"""Two sweep epochs of the headline batch (1M YCSB theta=0.9 txns): driver for
DCC_SW_DEBUG clock stamps and per-dispatch PMC passes (tools/gpu_pmc_sweep.sh)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import deneva_amd as d  # noqa: E402

b = d.gen_ycsb(n_txn=1 << 20, zipf_theta=0.9)
db = b.to_torch("cuda:0")
with d.Engine(0) as e:
    for _ in range(2):
        rc, _, st = e.occ_validate_epoch(db)
    print(st["device_ms"], st["rounds"])
