"""C2 (65,536 YCSB txns x 16 keys, theta 0.9) device time under level
schedules (measurement aid; experiments build for DCC_SW_PMAX):
  python tools/c2_probe.py [levels]  with DCC_SW_PMAX set in the environment."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _oracle as orc  # noqa: E402
import deneva_amd as d  # noqa: E402


def main():
    lv = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    eng = d.Engine(0)
    if lv:
        eng.set_option(d._abi.OPT_SWEEP_LEVELS, lv)
    out = []
    cases = (("C2", lambda: d.gen_ycsb(n_txn=65536, zipf_theta=0.9)),
             ("C2s", lambda: d.gen_ycsb(n_txn=65536, zipf_theta=0.9, seed=77)),
             ("C3", lambda: d.gen_tpcc(n_txn=262144, num_wh=128)),
             ("H", lambda: d.gen_ycsb(n_txn=1 << 20, zipf_theta=0.9)))
    only = os.environ.get("C2_ONLY")
    for tag, gen in cases:
        if only and tag != only:
            continue
        b = gen()
        db = b.to_torch("cuda:0")
        rc = torch.empty(b.n_txn, dtype=torch.uint8, device="cuda:0")
        ms = []
        for i in range(30):
            st = eng.occ_validate_epoch(db, out_rc=rc)[2]
            if i >= 5:
                ms.append(st["device_ms"])
        erc, _, _ = orc.occ(b)
        ok = np.array_equal(rc.cpu().numpy(), erc)
        out.append(f"{tag} {np.median(ms):.4f} ms rounds {st['rounds']} survivors {st['n_survivors']} parity {ok}")
    print(os.environ.get("DCC_SW_PMAX", "default"), "levels", lv, "|", " | ".join(out), flush=True)


if __name__ == "__main__":
    main()
