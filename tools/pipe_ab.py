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
    cfgs = [tuple(int(x) for x in a.split(":")) for a in sys.argv[1:]] or [(3,)]
    L_max = max(c[0] for c in cfgs)
    like = os.environ.get("LIKE", "")  # bench-like setup steps (bisecting a bench/probe gap)
    if "s" in like:
        import torch.distributed  # noqa: F401
        torch.cuda.set_device(0)
    bs = [d.gen_ycsb(n_txn=1 << 20, zipf_theta=0.9, seed=0xD3E7A001 + i) for i in range(L_max)]
    exp = [orc.occ(b)[0] for b in bs]
    if "e" in like:
        eng = d.Engine(0)
    if "x" in like:
        extra = bs[0].to_torch("cuda:0")  # noqa: F841  (the bench's latency batch)
        extra_out = torch.empty(bs[0].n_txn, dtype=torch.uint8, device="cuda:0")  # noqa: F841
    dbs = [b.to_torch("cuda:0") for b in bs]
    outs = [torch.empty(b.n_txn, dtype=torch.uint8, device="cuda:0") for b in bs]
    if "e" not in like:
        eng = d.Engine(0)
    if os.environ.get("PRE"):  # the bench's order: single epochs on the parent context first
        for _ in range(int(os.environ["PRE"])):
            eng.occ_validate_epoch(dbs[0], out_rc=outs[0])
        torch.cuda.synchronize()
    serial = bool(os.environ.get("SERIAL"))  # one epoch in flight: latency over L rotating batches
    for L, *_ in cfgs:
        eng.set_option(d._abi.OPT_PIPELINE, L)

        host = [0.0, 0.0]

        def run(k):
            q = deque()
            for i in range(k):
                t0 = time.perf_counter()
                q.append(eng.occ_submit_epoch(dbs[i % L], outs[i % L]))
                t1 = time.perf_counter()
                host[0] += t1 - t0
                if len(q) >= (1 if serial else L):
                    eng.occ_wait_epoch(q.popleft())
                    host[1] += time.perf_counter() - t1
            while q:
                eng.occ_wait_epoch(q.popleft())
        run(3 * L)
        runs = []
        for _ in range(3):
            host[0] = host[1] = 0.0
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run(K)
            torch.cuda.synchronize()
            runs.append((time.perf_counter() - t0) / K * 1e3)
        par = all(np.array_equal(outs[i].cpu().numpy(), exp[i]) for i in range(L))
        print(f"lanes {L}: {min(runs):.4f} ms/epoch (runs {' '.join(f'{x:.4f}' for x in runs)}; last run "
              f"host in submit {host[0] / K * 1e6:.1f} us, in wait {host[1] / K * 1e6:.1f} us per epoch), "
              f"parity {par}", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
