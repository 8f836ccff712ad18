"""Sweep stamps of one YCSB theta=0.9 epoch (measurement aid; experiments
build with DCC_SW_DEBUG=1 prints the per-level stamps to stderr):
  DENEVA_AMD_LIB=deneva_amd/libdcc_exp.so DCC_SW_DEBUG=1 python tools/filter_probe.py [n_txn]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import deneva_amd as d  # noqa: E402


def main():
    eng = d.Engine(0)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    b = d.gen_ycsb(n_txn=n, zipf_theta=0.9)
    db = b.to_torch("cuda:0")
    rc = torch.empty(b.n_txn, dtype=torch.uint8, device="cuda:0")
    for i in range(4):
        st = eng.occ_validate_epoch(db, out_rc=rc)[2]
        print(f"epoch {i}: device {st['device_ms']:.4f} ms", file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
