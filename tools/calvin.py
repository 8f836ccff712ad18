"""Time the Calvin engine on the C4 batch (1M txns x 16 keys, 16 partitions,
sequencer order), device-resident, with per-phase profiling."""
import argparse, json, os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import deneva_amd as d

ap = argparse.ArgumentParser()
ap.add_argument("--txns", type=int, default=1 << 20)
ap.add_argument("--theta", type=float, default=0.9)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--waves", action="store_true")
args = ap.parse_args()
b = d.gen_ycsb(n_txn=args.txns, zipf_theta=args.theta, part_cnt=16, chunk_txns=args.txns // 16,
               want_home=True)
home = b.meta["home"].astype(np.uint64)
seq = np.zeros(b.n_txn, np.uint64)
for h in np.unique(home):
    idx = np.nonzero(home == h)[0]
    seq[idx] = np.arange(idx.size, dtype=np.uint64)
b.order = (home << np.uint64(32)) | seq
db = b.to_torch("cuda:0")
eng = d.Engine(0)
for prof in (False, True):
    eng.set_profiling(prof)
    ts = []
    for r in range(args.reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g, rc, w, st = eng.calvin_order_epoch(db, want_group=True, want_wave=args.waves)
        torch.cuda.synchronize()
        if r:
            ts.append((time.perf_counter() - t0) * 1e3)
    print(json.dumps({"profiling": prof, "waves": args.waves, "wall_ms_med": float(np.median(ts)),
                      "device_ms": st["device_ms"], "phase_ms": st["phase_ms"],
                      "ready": st["n_commit"], "rounds": st["rounds"],
                      "alg_bytes": st["alg_bytes"],
                      "txns_per_s": args.txns / (st["device_ms"] * 1e-3)}))
