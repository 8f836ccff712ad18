#!/usr/bin/env python3
"""How much of the GPU does one headline OCC epoch leave idle?  K epochs on
one context, then the same K epochs split over two contexts driven by two
host threads (each epoch is the latency-bound sweep chain; two independent
epochs can share the chip).  Parity is checked on every epoch."""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import _oracle as orc  # noqa: E402
import deneva_amd as d  # noqa: E402


def main():
    import torch
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    b = d.gen_ycsb(n_txn=1 << 20, zipf_theta=0.9, seed=0xD3E7A001)
    erc, _, _ = orc.occ(b)
    db = b.to_torch("cuda:0")
    engs = [d.Engine(0), d.Engine(0)]
    outs = [torch.empty(b.n_txn, dtype=torch.uint8, device="cuda:0") for _ in engs]
    for e, o in zip(engs, outs):
        for _ in range(3):
            e.occ_validate_epoch(db, out_rc=o)
    torch.cuda.synchronize()

    def run(e, o, n, bad):
        for _ in range(n):
            e.occ_validate_epoch(db, out_rc=o)

    for trial in range(2):
        t0 = time.perf_counter()
        run(engs[0], outs[0], K, None)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        th = [threading.Thread(target=run, args=(engs[i], outs[i], K // 2, None)) for i in range(2)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        ok = all(np.array_equal(o.cpu().numpy(), erc) for o in outs)
        one, two = (t1 - t0) / K * 1e3, (t2 - t1) / K * 1e3
        print(f"trial {trial}: one context {one:.4f} ms/epoch, two contexts {two:.4f} ms/epoch "
              f"(x{one / two:.2f}), parity {ok}", flush=True)


if __name__ == "__main__":
    main()
