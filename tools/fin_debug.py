#!/usr/bin/env python3
"""Debug aid for the one-launch central_finish (k_fin): a 65,536-txn epoch
with commit tn into device outputs; per 1,024-txn block, how the device's
numbering differs from the oracle's."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import _oracle as orc  # noqa: E402
import deneva_amd as d  # noqa: E402


def main():
    import torch
    eng = d.Engine(0)
    for n, theta in [(65536, 0.0), (65536, 0.9), (5000, 0.0)]:
        b = d.gen_ycsb(n_txn=n, zipf_theta=theta)
        erc, etn, _ = orc.occ(b)
        db = b.to_torch("cuda:0")
        rc = torch.empty(n, dtype=torch.uint8, device="cuda:0")
        tn = torch.zeros(n, dtype=torch.int64, device="cuda:0")
        for rep in range(3):
            eng.tnc = 0
            try:
                eng.occ_validate_epoch(db, want_tn=True, out_rc=rc, out_tn=tn)
                err = ""
            except Exception as e:  # noqa: BLE001
                err = str(e)
            torch.cuda.synchronize()
            g = tn.cpu().numpy().astype(np.uint64)
            bad = np.nonzero(g != etn)[0]
            print(n, theta, rep, "err:", err[:90], "bad:", bad.size, "first:", bad[:5],
                  "blocks:", np.unique(bad // 1024)[:10], flush=True)
            if bad.size:
                i = bad[0]
                print("   gpu", g[i:i + 3], "oracle", etn[i:i + 3])
    eng.close()


if __name__ == "__main__":
    main()
