#!/usr/bin/env python3
"""Timing variants of the history window check (k_hist) on the SHIM epoch
(device-resident 1M YCSB batch, TS_CAS windows against the previous epoch's
~25K committed writes, commit tn + append).  Needs the DCC_EXPERIMENTS build:
DENEVA_AMD_LIB=deneva_amd/libdcc_exp.so.  DCC_HIST_VAR bits: 1 no probes,
2 no key bitmap, 4 no txn search, 8 no collision walks; DCC_FIN_VAR (x256):
1 no chain pushes, 2 no look-back wait, 4 no write-set emission, 8 no tn stores.  Prints device ms per epoch."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import _oracle as orc  # noqa: E402
import deneva_amd as d  # noqa: E402


def main():
    import torch
    n = 1 << 20
    rng = np.random.default_rng(0xD3E7A00C)
    prev = d.gen_ycsb(n_txn=n, zipf_theta=0.9, seed=0xD3E7A00D)
    _, ptn, ptnc = orc.occ(prev)
    off = np.asarray(prev.offsets, np.int64)
    owner = np.repeat(np.arange(n), np.diff(off))
    sel = (np.asarray(prev.acctype) == d.WR) & (ptn[owner] != 0)
    hk, ht = np.asarray(prev.keys, np.uint64)[sel].copy(), ptn[owner[sel]].astype(np.uint64)
    b = d.gen_ycsb(n_txn=n, zipf_theta=0.9)
    b.start_tn = (ptnc - rng.integers(0, ptnc + 1, size=n)).astype(np.uint64)
    b.finish_tn = (ptnc + rng.integers(0, 64, size=n)).astype(np.uint64)
    erc, _, _ = orc.occ(b, hist_keys=hk, hist_tn=ht, tnc=ptnc)
    db = b.to_torch("cuda:0")
    rc = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    tn = torch.empty(n, dtype=torch.int64, device="cuda:0")
    for var in [int(v) for v in (sys.argv[1:] or ["0", "1", "2", "4"])]:
        os.environ["DCC_HIST_VAR"] = str(var & 0xFF)
        os.environ["DCC_FIN_VAR"] = str(var >> 8)  # k_fin variants in the high byte
        eng = d.Engine(0)  # a fresh context: the epoch graph is captured with this variant
        ms = []
        for i in range(8):
            eng.history_clear()
            eng.history_append(hk, ht)
            eng.tnc = ptnc
            torch.cuda.synchronize()
            try:
                st = eng.occ_validate_epoch(db, want_tn=True, append_history=True, out_rc=rc, out_tn=tn)[2]
            except d.DccError:  # a timing variant's totals disagree: its kernel times still count
                st = {"device_ms": float("nan")}
            if i >= 3:
                ms.append(st["device_ms"])
        par = bool(np.array_equal(rc.cpu().numpy(), erc))
        print(f"DCC_HIST_VAR={var}: device {np.median(ms):.4f} ms, parity {par}", flush=True)
        eng.close()


if __name__ == "__main__":
    main()
