#!/usr/bin/env python3
"""C4 epochs only (no oracle, no CPU leg): for kernel timing runs."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
import deneva_amd as d  # noqa: E402
from helpers import c4_batch  # noqa: E402

b = c4_batch()
db = b.to_torch("cuda:0")
eng = d.Engine(0)
g = torch.empty(b.nnz, dtype=torch.int32, device="cuda:0")
rc = torch.empty(b.n_txn, dtype=torch.uint8, device="cuda:0")
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6):
    eng.calvin_order_epoch(db, want_group=True, out_group=g, out_rc=rc)
torch.cuda.synchronize()
print("ok")
