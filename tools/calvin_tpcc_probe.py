"""TPC-C Calvin epoch (262,144 txns, 128 warehouses) device time on the sort
path (DCC_OPT_CALVIN_PATH 1) and the bucket path with the hashed carry table
(2) -- measurement aid."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import deneva_amd as d  # noqa: E402


def main():
    eng = d.Engine(0)
    b = d.gen_tpcc(n_txn=262144, num_wh=128)
    db = b.to_torch("cuda:0")
    g = torch.empty(b.nnz, dtype=torch.int32, device="cuda:0")
    rc = torch.empty(b.n_txn, dtype=torch.uint8, device="cuda:0")
    out = {}
    for path in (1, 2, 0):
        eng.set_option(d._abi.OPT_CALVIN_PATH, path)
        ms = []
        for i in range(12):
            st = eng.calvin_order_epoch(db, want_group=True, out_group=g, out_rc=rc)[3]
            if i >= 2:
                ms.append(st["device_ms"])
        out[path] = (float(np.median(ms)), st["fallback"])
    print("TPC-C Calvin 262144 x 128 WH: sort path %.4f ms | bucket (hashed) %.4f ms (bucket=%d) | auto %.4f ms (bucket=%d)"
          % (out[1][0], out[2][0], out[2][1], out[0][0], out[0][1]), flush=True)


if __name__ == "__main__":
    main()
