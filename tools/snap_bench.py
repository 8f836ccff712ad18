"""Times the C6 captured-snapshot config alone (for rocprofv3 kernel stats of
k_snap): python tools/snap_bench.py [steps]."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

import _oracle as orc  # noqa: E402  (checker only)
import bench  # noqa: E402
import deneva_amd as d  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st = [fn() for _ in range(steps)]
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps, st[-1]

    with d.Engine(0) as eng:
        r = bench.snapshot_config(eng, "cuda:0", timed, orc)
    print(r)
    assert r["parity_vs_oracle"]


if __name__ == "__main__":
    main()
