#!/usr/bin/env python3
"""One headline epoch through the dataflow solver (solver 4) with
DCC_DF_DEBUG stamps (the engine prints per-wave timing, passes, refills,
polls and the decision curve to stderr); checks parity against the oracle.
    DCC_DF_DEBUG=1 python tools/df_diag.py [--txns N] [--theta T]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import _oracle as orc  # noqa: E402  (checker)
import deneva_amd as d  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--txns", type=int, default=1 << 20)
    ap.add_argument("--theta", type=float, default=0.9)
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0xD3E7A001)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    import torch
    b = d.gen_ycsb(n_txn=a.txns, zipf_theta=a.theta, seed=a.seed)
    erc, _, _ = orc.occ(b)
    db = b.to_torch("cuda:0")
    with d.Engine(0) as eng:
        eng.set_option(d._abi.OPT_SOLVER, 4)
        for r in range(a.reps):
            rc, _, st = eng.occ_validate_epoch(db)
            torch.cuda.synchronize()
            ok = np.array_equal(rc.cpu().numpy(), erc)
            print(f"rep {r}: device {st['device_ms']:.3f} ms survivors {st['n_survivors']} "
                  f"fallback {st['fallback']} parity {ok}", flush=True)
            sys.stderr.flush()


if __name__ == "__main__":
    main()
