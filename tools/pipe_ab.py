#!/usr/bin/env python3
"""A/B of the pipelined headline (dcc_occ_submit_epoch): for each (lanes,
reserve) in argv ("L:R" pairs), K pipelined 1M-txn theta=0.9 epochs over L
distinct resident batches; ms per epoch (best of 3 timed runs) and parity of
every lane's last decisions against the oracle."""
import os
import sys
import time
from collections import deque

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import _oracle as orc  # noqa: E402
import deneva_amd as d  # noqa: E402


def main():
    import torch
    K = int(os.environ.get("K", "60"))
    cfgs = [tuple(int(x) for x in a.split(":")) for a in sys.argv[1:]] or [(2, 0)]
    L_max = max(c[0] for c in cfgs)
    bs = [d.gen_ycsb(n_txn=1 << 20, zipf_theta=0.9, seed=0xD3E7A001 + i) for i in range(L_max)]
    exp = [orc.occ(b)[0] for b in bs]
    dbs = [b.to_torch("cuda:0") for b in bs]
    outs = [torch.empty(b.n_txn, dtype=torch.uint8, device="cuda:0") for b in bs]
    eng = d.Engine(0)
    for L, R in cfgs:
        eng.set_option(d._abi.OPT_PIPELINE, L)

        def run(k):
            q = deque()
            for i in range(k):
                q.append(eng.occ_submit_epoch(dbs[i % L], outs[i % L]))
                if len(q) >= L:
                    eng.occ_wait_epoch(q.popleft())
            while q:
                eng.occ_wait_epoch(q.popleft())
        run(3 * L)
        best = 1e9
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run(K)
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t0) / K * 1e3)
        par = all(np.array_equal(outs[i].cpu().numpy(), exp[i]) for i in range(L))
        print(f"lanes {L} reserve {R}: {best:.4f} ms/epoch, parity {par}", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
