"""Where the pipelined central_finish's time goes (measurement aid): the
same 4-lane stream of 1M-txn epochs with (a) no commit tn, (b) commit tn,
(c) commit tn + history append, (d) (c) with the history trimmed every
epoch (no base growth).  ms per epoch and host split per call."""
import os
import sys
import time

os.environ.setdefault("GPU_MAX_HW_QUEUES", "12")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from collections import deque  # noqa: E402

import torch  # noqa: E402

import deneva_amd as d  # noqa: E402


def main():
    L, K = 4, 40
    eng = d.Engine(0)
    eng.set_option(d._abi.OPT_PIPELINE, L)
    bs = [d.gen_ycsb(n_txn=1 << 20, zipf_theta=0.9, seed=0xD3E7A001 + i).to_torch("cuda:0") for i in range(L)]
    rcs = [torch.empty(1 << 20, dtype=torch.uint8, device="cuda:0") for _ in range(L)]
    tns = [torch.empty(1 << 20, dtype=torch.int64, device="cuda:0") for _ in range(L)]
    for mode in ("none", "tn", "tn+app", "tn+app+trim"):
        for rep in range(2):
            eng.history_clear()
            eng.tnc = 0
            torch.cuda.synchronize()
            fl = deque()
            ts = tw = 0.0
            t_all = time.perf_counter()
            for k in range(K):
                t0 = time.perf_counter()
                fl.append(eng.occ_submit_epoch(bs[k % L], rcs[k % L], None if mode == "none" else tns[k % L],
                                               append_history=mode.startswith("tn+app")))
                t1 = time.perf_counter()
                ts += t1 - t0
                if len(fl) >= L:
                    eng.occ_wait_epoch(fl.popleft())
                    tw += time.perf_counter() - t1
                    if mode == "tn+app+trim" and k % 4 == 3:
                        eng.history_trim(max(0, eng.tnc - 1))
            while fl:
                eng.occ_wait_epoch(fl.popleft())
            torch.cuda.synchronize()
            dt = time.perf_counter() - t_all
        print(f"{mode:12s} {dt / K * 1e3:.4f} ms/epoch  submit {ts / K * 1e6:.1f} us  wait {tw / K * 1e6:.1f} us "
              f"history {eng.history_size}", flush=True)


if __name__ == "__main__":
    main()
