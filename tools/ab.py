"""A/B timing of engine variants in ONE process (interleaved rounds), on the
bench batch.  Usage: python tools/ab.py [--txns N] [--theta T] [--reps R]"""
import argparse, json, os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import deneva_amd as d
from deneva_amd import _abi

ap = argparse.ArgumentParser()
ap.add_argument("--txns", type=int, default=1 << 20)
ap.add_argument("--theta", type=float, default=0.9)
ap.add_argument("--reps", type=int, default=10)
args = ap.parse_args()
b = d.gen_ycsb(n_txn=args.txns, zipf_theta=args.theta)
db = b.to_torch("cuda:0")
out = torch.empty(args.txns, dtype=torch.uint8, device="cuda:0")
variants = {
    "rc0": [(_abi.OPT_RECHECK, 0), (_abi.OPT_BATCH_MAX, 8)],
    "rc16k": [(_abi.OPT_RECHECK, 16384), (_abi.OPT_BATCH_MAX, 8)],
    "rc64k": [(_abi.OPT_RECHECK, 65536), (_abi.OPT_BATCH_MAX, 8)],
    "rc256k": [(_abi.OPT_RECHECK, 262144), (_abi.OPT_BATCH_MAX, 8)],
    "rcall": [(_abi.OPT_RECHECK, 1 << 40), (_abi.OPT_BATCH_MAX, 8)],
    "rc64k_b4": [(_abi.OPT_RECHECK, 65536), (_abi.OPT_BATCH_MAX, 4)],
    "rc64k_b16": [(_abi.OPT_RECHECK, 65536), (_abi.OPT_BATCH_MAX, 16)],
}
eng = d.Engine(0)
ref = None
res = {k: [] for k in variants}
for rep in range(args.reps + 1):
    for name, opts in variants.items():
        for o, v in opts:
            eng.set_option(o, v)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _, _, st = eng.occ_validate_epoch(db, out_rc=out)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        r = out.cpu().numpy()
        if ref is None:
            ref = r.copy()
        assert np.array_equal(r, ref), name
        if rep:
            res[name].append((dt * 1e3, st["device_ms"], st["rounds"]))
for name, v in res.items():
    a = np.array(v)
    print(json.dumps({"variant": name, "wall_ms_med": float(np.median(a[:, 0])),
                      "wall_ms_min": float(a[:, 0].min()), "dev_ms_med": float(np.median(a[:, 1])),
                      "rounds": int(a[0, 2])}))
