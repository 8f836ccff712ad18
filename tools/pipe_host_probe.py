"""Host cost of the pipeline calls (measurement aid): submit L epochs, let
the GPU finish them (sleep), then time each wait -- the host work of
dcc_occ_wait_epoch when nothing is left to wait for -- and each submit.
Then the steady loop of bench.py at L lanes with per-call host times."""
import os
import sys
import time

os.environ.setdefault("GPU_MAX_HW_QUEUES", "12")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import deneva_amd as d  # noqa: E402


def main():
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    eng = d.Engine(0)
    eng.set_option(d._abi.OPT_PIPELINE, L)
    bs = [d.gen_ycsb(n_txn=1 << 20, zipf_theta=0.9, seed=0xD3E7A001 + i).to_torch("cuda:0") for i in range(L)]
    outs = [torch.empty(1 << 20, dtype=torch.uint8, device="cuda:0") for _ in range(L)]
    torch.cuda.synchronize()
    for _ in range(3):
        ts = [eng.occ_submit_epoch(bs[i], outs[i]) for i in range(L)]
        for t in ts:
            eng.occ_wait_epoch(t)
    sub, wt = [], []
    for _ in range(20):
        ts = []
        for i in range(L):
            t0 = time.perf_counter()
            ts.append(eng.occ_submit_epoch(bs[i], outs[i]))
            sub.append(time.perf_counter() - t0)
        time.sleep(0.01)
        for t in ts:
            t0 = time.perf_counter()
            eng.occ_wait_epoch(t)
            wt.append(time.perf_counter() - t0)
    print(f"L={L} idle-GPU host cost: submit {np.median(sub) * 1e6:.1f} us (p90 {np.percentile(sub, 90) * 1e6:.1f}), "
          f"wait {np.median(wt) * 1e6:.1f} us (p90 {np.percentile(wt, 90) * 1e6:.1f})")
    # steady loop
    from collections import deque
    K = 400
    inflight = deque()
    tsub = twait = 0.0
    torch.cuda.synchronize()
    t_all = time.perf_counter()
    for k in range(K):
        t0 = time.perf_counter()
        inflight.append(eng.occ_submit_epoch(bs[k % L], outs[k % L]))
        t1 = time.perf_counter()
        tsub += t1 - t0
        if len(inflight) >= L:
            eng.occ_wait_epoch(inflight.popleft())
            twait += time.perf_counter() - t1
    while inflight:
        eng.occ_wait_epoch(inflight.popleft())
    torch.cuda.synchronize()
    dt = time.perf_counter() - t_all
    print(f"L={L} steady: {dt / K * 1e3:.4f} ms/epoch, submit {tsub / K * 1e6:.1f} us, wait {twait / K * 1e6:.1f} us")


if __name__ == "__main__":
    main()
