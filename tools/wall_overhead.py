#!/usr/bin/env python3
"""Host overhead per headline epoch: wall per call against the device time
(HIP events) and the C-side wall (stats total_ms).  Run on the GPU box:
    DCC_SPIN_WAIT=0|1 python tools/wall_overhead.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import deneva_amd as d  # noqa: E402
import torch  # noqa: E402

b = d.gen_ycsb(n_txn=1 << 20, zipf_theta=0.9, seed=0xD3E7A001)
db = b.to_torch("cuda:0")
rc = torch.empty(b.n_txn, dtype=torch.uint8, device="cuda:0")
with d.Engine(0) as eng:
    for _ in range(5):
        eng.occ_validate_epoch(db, out_rc=rc)
    torch.cuda.synchronize()
    walls, devs, tots = [], [], []
    t_all = time.perf_counter()
    for _ in range(100):
        t0 = time.perf_counter()
        st = eng.occ_validate_epoch(db, out_rc=rc)[2]
        walls.append(time.perf_counter() - t0)
        devs.append(st["device_ms"])
        tots.append(st["total_ms"])
    t_all = (time.perf_counter() - t_all) / 100
print(f"spin={os.environ.get('DCC_SPIN_WAIT', 'default')}: wall/call {np.mean(walls) * 1e3:.4f} ms "
      f"(loop {t_all * 1e3:.4f}), C-side {np.mean(tots):.4f} ms, device {np.mean(devs):.4f} ms")
