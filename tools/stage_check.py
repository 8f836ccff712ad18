#!/usr/bin/env python3
"""GPU quick check of the OCC stage solver: decisions vs the oracle on a few
shapes, then the headline epoch timing.  Prints one line per case.

    python tools/stage_check.py [--quick] [--time N]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import _oracle as orc  # noqa: E402
import deneva_amd as d  # noqa: E402
from helpers import chain_batch, random_batch  # noqa: E402


def cases(quick):
    rng = np.random.default_rng(1)
    yield "random-600", random_batch(rng, 600, 24, 400, types=(0, 1, 2, 3))
    yield "chain-300", chain_batch(300)
    yield "ycsb-3000", d.gen_ycsb(n_txn=3000, zipf_theta=0.9)
    yield "ycsb-64K-0.9", d.gen_ycsb(n_txn=65536, zipf_theta=0.9)
    yield "tpcc-16K", d.gen_tpcc(n_txn=16384, num_wh=16)
    if not quick:
        yield "ycsb-1M-0.9", d.gen_ycsb(n_txn=1 << 20, zipf_theta=0.9)
        yield "ycsb-1M-0.99", d.gen_ycsb(n_txn=1 << 20, zipf_theta=0.99, seed=0xD3E7A002)
        yield "tpcc-256K", d.gen_tpcc(n_txn=262144, num_wh=128)
        yield "ycsb-200K-0.6", d.gen_ycsb(n_txn=200000, zipf_theta=0.6)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--time", type=int, default=20)
    ap.add_argument("--solver", type=int, default=4, help="4 stage solver, 3 sweep")
    args = ap.parse_args()
    import torch
    eng = d.Engine(0)
    eng.set_option(d._abi.OPT_SOLVER, args.solver)
    ok = True
    for name, b in cases(args.quick):
        erc, etn, _ = orc.occ(b)
        for dev in (False, True):
            bb = b.to_torch("cuda") if dev else b
            eng.tnc = 0
            rc, tn, st = eng.occ_validate_epoch(bb, want_tn=True)
            if dev:
                rc = rc.cpu().numpy()
                tn = tn.cpu().numpy().view(np.uint64)
            bad = int(np.count_nonzero(rc != erc))
            badt = int(np.count_nonzero(tn != etn))
            ok &= bad == 0 and badt == 0
            print(f"{name:14s} dev={int(dev)} n={b.n_txn} commits={st['n_commit']} "
                  f"stages={st['rounds']} p0={st['peel_prefix']} surv1={st['n_survivors']} "
                  f"fallback={st['fallback']} rc_bad={bad} tn_bad={badt} dev_ms={st['device_ms']:.3f}",
                  flush=True)
    if args.time:
        b = d.gen_ycsb(n_txn=1 << 20, zipf_theta=0.9)
        db = b.to_torch("cuda")
        out = torch.empty(b.n_txn, dtype=torch.uint8, device="cuda")
        for _ in range(3):
            eng.occ_validate_epoch(db, out_rc=out)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sts = [eng.occ_validate_epoch(db, out_rc=out)[2] for _ in range(args.time)]
        dt = (time.perf_counter() - t0) / args.time
        dm = float(np.mean([s["device_ms"] for s in sts]))
        erc, _, _ = orc.occ(b)
        par = bool(np.array_equal(out.cpu().numpy(), erc))
        print(f"headline 1M theta0.9: wall {dt*1e3:.3f} ms device {dm:.3f} ms "
              f"({sts[-1]['alg_bytes']/dm/1e6:.0f} GB/s alg, frac {sts[-1]['alg_bytes']/dm/1e6/8000:.3f}) "
              f"stages {sts[-1]['rounds']} parity {par}", flush=True)
        eng.set_profiling(True)
        p = eng.occ_validate_epoch(db, out_rc=out)[2]
        eng.set_profiling(False)
        print("profiled phases ms:", [round(x, 4) for x in p["phase_ms"]], flush=True)
    print("ALL OK" if ok else "MISMATCH", flush=True)
    eng.close()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
