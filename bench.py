#!/usr/bin/env python3
"""bench.py — OCC-validated txns/s on MI355X (BASELINE.json metric).

A step is one OCC epoch decision (dcc_occ_validate_epoch) over a resident
synthetic YCSB batch: 1,048,576 txns x 16 keys, zipf theta 0.9, 16,777,216-key
table, TXN_WRITE_PERC = TUP_WRITE_PERC = 0.5 (SURVEY.md §8(d) "Headline").

    python bench.py [--gpus N] [--steps K] [--warmup W] [--txns N] [--theta T]

N > 1 is launched by torch.distributed.run (one rank per GPU, RCCL): keys are
hash-sharded across the ranks and every round joins a per-txn state allreduce.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Each lane of the pipelined headline is a HIP stream that needs a hardware
# queue of its own; HIP's default of 4 queues per process makes lanes share
# queues and serialise.  Set before HIP initialises.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 12:
    os.environ["GPU_MAX_HW_QUEUES"] = "12"

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)  # (a 20-epoch region is ~3 ms: host jitter moved it by 10 %)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--txns", type=int, default=1 << 20)
    ap.add_argument("--theta", type=float, default=0.9)
    ap.add_argument("--keys", type=int, default=16)
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0xD3E7A001)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=131072,
                    help="txns of the batch timed with the CPU reference restatement")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the other BASELINE configs (C2, C3, C4, C5) at N=1")
    ap.add_argument("--only", default="",
                    help="comma-separated secondary configs to run INSTEAD of the headline "
                         "(profiling aid): " + ",".join(CONFIGS))
    ap.add_argument("--solver", type=int, default=0,
                    help="OCC solver: 0 auto (= 3), 1 fixed-point rounds only, 3 sweep levels")
    ap.add_argument("--sweep-levels", type=int, default=0,
                    help="sweep levels per captured epoch (DCC_OPT_SWEEP_LEVELS; 0: the engine's "
                         "default)")
    ap.add_argument("--ro-split", type=int, default=-1,
                    help="DCC_OPT_RO_SPLIT (-1: the engine's default)")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: one fixed batch of --txns txns key-sharded over the "
                         "N ranks (BASELINE config C5 with --theta 0.99 --seed 0xD3E7A002); "
                         "default is weak scaling (N x --txns txns)")
    ap.add_argument("--pmc", default=next((p for p in (os.path.join(ROOT, "profiles", r, "pmc.json")
                                                       for r in ("r06", "r05", "r04")) if os.path.exists(p)),
                                          os.path.join(ROOT, "profiles", "r05", "pmc.json")),
                    help="PMC summary (tools/gpu_pmc_r05.sh -> tools/pmc_r05.py) the "
                         "roofline.traffic / l2_hit fields and each config's pmc block are read "
                         "from (the workloads it describes at N=1; null otherwise)")
    ap.add_argument("--pipeline", type=int, default=4,
                    help="lanes of the pipelined headline (dcc_occ_submit_epoch, DCC_OPT_PIPELINE): "
                         "consecutive epochs over that many distinct resident batches overlap on "
                         "the GPU (N=1; 0 = one epoch at a time)")
    ap.add_argument("--partition", type=int, default=0, choices=[0, 1],
                    help="pipeline lanes on their own CUs (DCC_OPT_PIPE_PARTITION): lane i of L "
                         "on 1/L of every XCD's CUs, CU-masked streams")
    ap.add_argument("--exchange", choices=["rccl", "host"], default="rccl",
                    help="N>1 status all-reduce: RCCL over xGMI (one GPU per rank), or "
                         "host/gloo (rehearsal: ranks may share one GPU)")
    return ap.parse_args()


def stream_copy_gbps(dev, mib=2048, reps=10):
    """Achievable HBM bandwidth on this GPU, the larger of two device copies
    of a `mib` MiB buffer (read + write bytes / time, HIP events): torch's
    copy_ and the engine's hand-written 16-B-per-lane copy kernel
    (dcc_copy_bandwidth; MI355X_MICROARCH.md measures ~6.3 TB/s for such a
    copy).  BASELINE.md §4: the measured peak is reported next to the spec."""
    return max(v for v in stream_copy_both(dev, mib, reps).values() if v)


def stream_copy_both(dev, mib=2048, reps=10):
    import ctypes as C
    import deneva_amd as d
    out = {"torch_copy": _torch_copy_gbps(dev, mib, reps), "copy16_kernel": None}
    with d.Engine(int(str(dev).split(":")[-1]) if ":" in str(dev) else 0) as e:
        g = C.c_double()
        if d._abi.lib.dcc_copy_bandwidth(e._h, mib << 20, reps, C.byref(g)) == 0:
            out["copy16_kernel"] = g.value
    return out


def _torch_copy_gbps(dev, mib=2048, reps=10):
    import torch
    n = mib << 20
    a = torch.empty(n, dtype=torch.uint8, device=dev)
    b = torch.empty(n, dtype=torch.uint8, device=dev)
    a.fill_(1)
    for _ in range(2):
        b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    del a, b
    return 2.0 * n / (ms * 1e-3) / 1e9


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_threads() -> int:
    """Host threads the multi-threaded CPU baselines use: this process's CPU
    affinity, capped by its share of the box (OMP_NUM_THREADS, 16 per GPU on
    the test pool, where affinity and nproc show the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    share = os.environ.get("OMP_NUM_THREADS", "")
    return max(1, min(n, int(share))) if share.isdigit() and int(share) > 0 else n


def prefix_batch(b, n):
    """The first n txns of a batch (a valid epoch of its own: the decisions
    of a prefix never depend on later txns)."""
    from deneva_amd import EpochBatch
    n = min(n, b.n_txn)
    off = np.asarray(b.offsets)[: n + 1].copy()
    cut = lambda a: None if a is None else np.asarray(a)[:n].copy()
    return EpochBatch(off, np.asarray(b.keys)[: off[-1]], np.asarray(b.acctype)[: off[-1]],
                      cut(b.start_tn), cut(b.finish_tn), cut(b.order))


def _kern_l2(pw, name):
    """L2 hit rate of the first kernel of a PMC workload summary whose name
    holds `name` (profiles/r05/pmc.json), or null."""
    for k, v in ((pw or {}).get("kernels") or {}).items():
        if name in k:
            return v.get("l2_hit")
    return None


def cpu_leg(fn, n, variant, sample_note):
    """Time one single-threaded CPU restatement of the reference algorithm
    (the checker's code, outside every GPU timing) on n txns."""
    t0 = time.perf_counter()
    out = fn()
    dt = time.perf_counter() - t0
    return out, {"txns_per_s": n / dt, "txns": n, "seconds": dt, "threads": 1, "kind": "port",
                 "variant": variant, "sample": sample_note}


def cpu_baseline(batch, sample: int):
    """The reference CPU path and its two faster restatements, timed on this
    host, on the same batch:
      (i)   REF-LITERAL: the literal OptCC epoch replay (active-list scan with
            test_valid pointer compares, occ.cpp:116-327; oracle/occ_ref.c),
            1 thread, on the first `sample` txns (O(N * commits * k^2), so
            bounded to ~10 s of CPU work);
      (ii)  HASH-SERIAL: serial hash-set scan, identical decisions, 1 thread,
            whole batch;
      (iii) ROUNDS-MT: the round-based fixed point (oracle/occ_mt.c) on every
            host thread this process may use, whole batch;
      (iv)  SWEEP-MT: the CPU form of the GPU sweep (oracle/occ_sweep_mt.c):
            serial prefixes on one thread, parallel read-only filters of the
            rest on every host thread -- the fastest host algorithm here.
    `value` is (i), the reference algorithm; the others are listed in
    `variants`, the fastest in `fastest_host`.  Each variant's decisions are
    checked against the others."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as orc  # checker / CPU baseline only
    from deneva_amd import EpochBatch

    threads = host_threads()
    n = min(sample, batch.n_txn)
    off = batch.offsets[: n + 1].copy()
    sub = EpochBatch(off, batch.keys[: off[-1]], batch.acctype[: off[-1]])
    t0 = time.perf_counter()
    rc_lit, _, _ = orc.occ(sub, literal=True)
    t_lit = time.perf_counter() - t0
    t0 = time.perf_counter()
    rc_hash, tn_hash, _ = orc.occ(batch)
    t_hash = time.perf_counter() - t0
    t0 = time.perf_counter()
    rc_mt, tn_mt, _, mt_rounds = orc.occ_rounds_mt(batch, threads)
    t_mt = time.perf_counter() - t0
    t_sw = []
    for _ in range(3):  # best of three (short: tens of ms)
        t0 = time.perf_counter()
        rc_sw, tn_sw, _, sw_levels = orc.occ_sweep_mt(batch, threads)
        t_sw.append(time.perf_counter() - t0)
    t_sw = min(t_sw)
    assert np.array_equal(rc_lit, rc_hash[:n])
    assert np.array_equal(rc_mt, rc_hash) and np.array_equal(tn_mt, tn_hash)
    assert np.array_equal(rc_sw, rc_hash) and np.array_equal(tn_sw, tn_hash)
    host = {"nproc": os.cpu_count(), "cpu_model": _cpu_model(), "threads_used": threads}
    return {"value": n / t_lit, "unit": "txns/s", "cores": 1, "kind": "port",
            "sample": f"REF-LITERAL: first {n} txns of the bench batch, literal OptCC epoch "
                      f"replay (oracle/occ_ref.c), {t_lit:.2f} s, 1 thread",
            "host": host,
            "variants": {
                "REF-LITERAL": {"txns_per_s": n / t_lit, "txns": n, "seconds": t_lit,
                                "threads": 1},
                "HASH-SERIAL": {"txns_per_s": batch.n_txn / t_hash, "txns": batch.n_txn,
                                "seconds": t_hash, "threads": 1},
                "ROUNDS-MT": {"txns_per_s": batch.n_txn / t_mt, "txns": batch.n_txn,
                              "seconds": t_mt, "threads": threads, "rounds": int(mt_rounds)},
                "SWEEP-MT": {"txns_per_s": batch.n_txn / t_sw, "txns": batch.n_txn,
                             "seconds": t_sw, "threads": threads, "levels": int(sw_levels)},
            },
            "fastest_host": {"variant": "SWEEP-MT", "txns_per_s": batch.n_txn / t_sw,
                             "threads": threads}}


def c4_order(b):
    """Sequencer order (origin = home partition, FIFO within the origin):
    sched_dequeue's (epoch, origin, FIFO) order (work_queue.cpp:105-151)."""
    home = b.meta["home"].astype(np.uint64)
    seq = np.zeros(b.n_txn, np.uint64)
    for h in np.unique(home):
        idx = np.nonzero(home == h)[0]
        seq[idx] = np.arange(idx.size, dtype=np.uint64)
    return (home << np.uint64(32)) | seq


def _timer(steps, warmup):
    import torch

    def timed(fn):
        for _ in range(warmup):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st = [fn() for _ in range(steps)]
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps, st[-1]
    return timed


def occ_config(eng, dev, timed, orc, tag):
    """C2 / C3 / C5: OCC epoch validation of one resident batch."""
    import torch
    import deneva_amd as d
    desc, gen = {
        "C2": ("YCSB OCC, 65,536 txns x 16 keys, theta=0.9",
               lambda: d.gen_ycsb(n_txn=65536, zipf_theta=0.9)),
        "C3": ("TPC-C NewOrder+Payment OCC, 128 warehouses, 262,144 txns",
               lambda: d.gen_tpcc(n_txn=262144, num_wh=128)),
        "C5": ("YCSB OCC, 1,048,576 txns x 16 keys, theta=0.99",
               lambda: d.gen_ycsb(n_txn=1 << 20, zipf_theta=0.99, seed=0xD3E7A002)),
    }[tag]
    b = gen()
    db = b.to_torch(dev)
    rc = torch.empty(b.n_txn, dtype=torch.uint8, device=dev)
    dt, st = timed(lambda: eng.occ_validate_epoch(db, out_rc=rc)[2])
    erc, _, _ = orc.occ(b)
    # the reference algorithm on the host: the literal OptCC epoch replay
    # (occ.cpp:116-327, oracle/occ_ref.c), on a prefix sized to ~5-10 s
    ns = {"C2": 65536, "C3": 65536, "C5": 262144}[tag]
    sub = prefix_batch(b, ns)
    (lrc, _, _), cpu = cpu_leg(lambda: orc.occ(sub, literal=True), sub.n_txn,
                               "REF-LITERAL (literal OptCC epoch replay, oracle/occ_ref.c)",
                               f"first {sub.n_txn} of {b.n_txn} txns")
    cpu["parity_vs_gpu"] = bool(np.array_equal(lrc, rc[: sub.n_txn].cpu().numpy()))
    return {"workload": desc, "txns_per_s": b.n_txn / dt, "ms_per_epoch": dt * 1e3,
            "cpu_baseline": cpu,
            "device_ms": st["device_ms"], "rounds": int(st["rounds"]),
            "commits": int(st["n_commit"]), "peel_prefix": int(st["peel_prefix"]),
            "survivors": int(st["n_survivors"]),
            "alg_GBps": st["alg_bytes"] / (st["device_ms"] * 1e-3) / 1e9,
            "parity_vs_oracle": bool(np.array_equal(rc.cpu().numpy(), erc))}


def calvin_config(eng, dev, timed, orc, tag="C4"):
    """C4: Calvin lock ordering, 16 partitions, 1M txns, sequencer order.
    C4 is the batch as the sequencers hand it over, origin by origin in FIFO
    order (the order is non-decreasing in index order; the engine detects that
    and skips its rank sort); C4_SHUF is the same txns captured with the 16
    origins interleaved (txn i from origin i % 16), so the engine must rank
    the order first."""
    import deneva_amd as d
    b = d.gen_ycsb(n_txn=1 << 20, zipf_theta=0.9, part_cnt=16, chunk_txns=65536, want_home=True)
    if tag == "C4_SHUF":
        b.meta["home"] = (np.arange(b.n_txn) % 16).astype(np.uint32)
    b.order = c4_order(b)
    db = b.to_torch(dev)
    res = {}
    import torch
    g_out = torch.empty(b.nnz, dtype=torch.int32, device=dev)  # reused across epochs
    rc_out = torch.empty(b.n_txn, dtype=torch.uint8, device=dev)

    def cv():
        g, rc, _, st = eng.calvin_order_epoch(db, want_group=True, out_group=g_out, out_rc=rc_out)
        res["g"], res["rc"] = g, rc
        return st
    dt, st = timed(cv)
    eg, erc, _ = orc.calvin(b)
    par = bool(np.array_equal(res["g"].cpu().numpy().astype(np.uint32)[:b.nnz], eg) and
               np.array_equal(res["rc"].cpu().numpy()[:b.n_txn], erc))
    # the reference's lock table on the host: the literal Row_lock CALVIN
    # replay (FIFO waiters, no barging, promotion on release; row_lock.cpp:
    # 52-381, oracle/calvin_ref.c) of the sequenced epoch's first txns
    sub = prefix_batch(b, 262144)
    _, cpu = cpu_leg(lambda: orc.calvin(sub, literal=True), sub.n_txn,
                     "REF-LITERAL (literal Row_lock CALVIN replay, oracle/calvin_ref.c)",
                     f"first {sub.n_txn} of {b.n_txn} txns (index order; sequenced by `order`)")
    return {"workload": "Calvin lock ordering, YCSB theta=0.9, 16 partitions, "
                        "1,048,576 txns x 16 keys, sequencer (origin, FIFO) order" +
                        (", origins interleaved in the capture" if tag == "C4_SHUF" else ""),
            "txns_per_s": b.n_txn / dt, "ms_per_epoch": dt * 1e3, "cpu_baseline": cpu,
            "device_ms": st["device_ms"], "ready_at_acquire": int(st["n_commit"]),
            "bucket_path": bool(st["fallback"]),
            "order_sorted_on_arrival": bool(np.all(np.diff(b.order.astype(np.int64)) >= 0)),
            "alg_GBps": st["alg_bytes"] / (st["device_ms"] * 1e-3) / 1e9,
            "hbm_frac": st["alg_bytes"] / (st["device_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "parity_vs_oracle": par}


def maat_config(eng, dev, timed, orc, tag="MAAT_C2"):
    """MaaT epoch validation on the C2 / headline
    YCSB shapes; each step starts from the same (empty) row timestamps."""
    import torch
    import deneva_amd as d
    n = 65536 if tag == "MAAT_C2" else 1 << 20
    b = d.gen_ycsb(n_txn=n, zipf_theta=0.9)
    db = b.to_torch(dev)
    rc = torch.empty(n, dtype=torch.uint8, device=dev)

    def step():
        eng.maat_rows_clear()
        return eng.maat_validate_epoch(db, want_cts=False, out_rc=rc)[2]
    dt, st = timed(step)
    erc, _, _ = orc.maat(b)
    # the reference algorithm on the host: the literal MaaT epoch replay
    # (Maat::validate / find_bound, Row_maat soft locks; maat.cpp:29-191,
    # row_maat.cpp:38-314, oracle/maat_ref.c) on the first 65,536 txns
    sub = prefix_batch(b, 65536)
    _, cpu = cpu_leg(lambda: orc.maat(sub, literal=True), sub.n_txn,
                     "REF-LITERAL (literal MaaT epoch replay, oracle/maat_ref.c)",
                     f"first {sub.n_txn} of {n} txns")
    return {"workload": f"MaaT epoch validation, YCSB {n} txns x 16 keys, theta=0.9, empty row "
                        f"timestamps",
            "txns_per_s": n / dt, "ms_per_epoch": dt * 1e3, "device_ms": st["device_ms"],
            "cpu_baseline": cpu,
            "rounds": int(st["rounds"]), "commits": int(st["n_commit"]),
            "alg_GBps": st["alg_bytes"] / (st["device_ms"] * 1e-3) / 1e9,
            "parity_vs_oracle": bool(np.array_equal(rc.cpu().numpy(), erc))}


def history_config(eng, dev, timed, orc, tag="HIST", n=1 << 18, epochs=8):
    """Multi-epoch OCC with the device history: each step runs
    `epochs` consecutive epochs from an empty history (tnc 0), every one with
    TS_CAS windows (start_tn, finish_tn] reaching about one epoch back, its
    committed writes appended on the device (DCC_OCC_APPEND_HISTORY, device
    pointers) and the history trimmed below the next windows.  The batches and
    their windows are built once, epoch by epoch, from the oracle's commit
    counter; the last step's decisions are checked against the oracle chain."""
    import torch
    import deneva_amd as d
    rng = np.random.default_rng(0xD3E7A00B)
    spread = n
    hk, ht = np.zeros(0, np.uint64), np.zeros(0, np.uint64)
    tnc, batches, floors, expect = 0, [], [], []
    for e in range(epochs):
        b = d.gen_ycsb(n_txn=n, zipf_theta=0.9, seed=0xD3E7A100 + e)
        b.start_tn = (tnc - rng.integers(0, spread, size=n)).clip(0).astype(np.uint64)
        b.finish_tn = (b.start_tn + rng.integers(0, 2 * spread, size=n)).astype(np.uint64)
        erc, etn, etnc = orc.occ(b, hist_keys=hk, hist_tn=ht, tnc=tnc)
        off = np.asarray(b.offsets, np.int64)
        owner = np.repeat(np.arange(n), np.diff(off))
        sel = (np.asarray(b.acctype) == d.WR) & (etn[owner] != 0)
        hk = np.concatenate([hk, np.asarray(b.keys, np.uint64)[sel]])
        ht = np.concatenate([ht, etn[owner[sel]]])
        floors.append(max(tnc - spread, 0))
        batches.append(b.to_torch(dev))
        expect.append(erc)
        tnc = etnc
    rcs = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(epochs)]
    acc = {}

    def step():
        eng.history_clear()
        eng.tnc = 0
        dev_ms, alg = 0.0, 0
        for e in range(epochs):
            if floors[e]:
                eng.history_trim(floors[e])
            st = eng.occ_validate_epoch(batches[e], append_history=True, out_rc=rcs[e])[2]
            dev_ms += st["device_ms"]
            alg += st["alg_bytes"]
        acc["hist"] = eng.history_size
        return {"device_ms": dev_ms, "alg_bytes": alg}
    dt, st = timed(step)
    par = all(np.array_equal(rcs[e].cpu().numpy(), expect[e]) for e in range(epochs))
    par = par and eng.tnc == tnc
    return {"workload": f"{epochs} consecutive OCC epochs of {n} YCSB txns x 16 keys (theta=0.9), "
                        f"TS_CAS windows ~1 epoch deep, device history append + trim",
            "txns_per_s": epochs * n / dt, "ms_per_epoch": dt * 1e3 / epochs,
            "device_ms_per_epoch": st["device_ms"] / epochs,
            "history_pairs_at_end": int(acc["hist"]), "history_pairs_untrimmed": int(hk.size),
            "alg_GBps": st["alg_bytes"] / (st["device_ms"] * 1e-3) / 1e9,
            "parity_vs_oracle": bool(par)}


def pipe_fin_config(eng, dev, timed, orc, tag="PIPE_FIN", n=1 << 20, lanes=4, k=40):
    """The headline stream with the reference's whole central_finish
    (occ.cpp:248-294) under its default TS_CLOCK: every epoch wants commit tn
    and appends its committed writes to the device history
    (DCC_OCC_APPEND_HISTORY), submitted through the pipeline
    (dcc_occ_submit_epoch): each lane decides its epoch and numbers / appends
    it on the device right behind the decision, from the device tnc and append
    position the epochs advance in submit order (DCC_OPT_PIPE_CHAIN; the
    context finishes an epoch itself when that could not: dcc_ctx::pipe_finish).  k
    epochs over `lanes` distinct resident batches from an empty history
    (merges of the delta into the base included); each lane's last epoch's
    decisions and tns are checked against the oracle (tn = the batch's own
    numbering from tnc 0 shifted by the tnc before the epoch)."""
    import torch
    import deneva_amd as d
    from collections import deque
    bs = [d.gen_ycsb(n_txn=n, zipf_theta=0.9, seed=0xD3E7A001 + i) for i in range(lanes)]
    dbs = [b.to_torch(dev) for b in bs]
    rcs = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(lanes)]
    tns = [torch.empty(n, dtype=torch.int64, device=dev) for _ in range(lanes)]
    exp = [orc.occ(b) for b in bs]  # (rc, tn from tnc 0, committed writers)
    eng.set_option(d._abi.OPT_PIPELINE, lanes)

    where = []

    def stream(kk):
        eng.history_clear()
        eng.tnc = 0
        where.clear()
        tnc_before = [0] * kk
        fl, t = deque(), 0
        for i in range(kk):
            tnc_before[i] = t
            t += exp[i % lanes][2]
            fl.append(eng.occ_submit_epoch(dbs[i % lanes], rcs[i % lanes], tns[i % lanes],
                                           append_history=True))
            if len(fl) >= lanes:
                where.append(eng.occ_wait_epoch(fl.popleft())["fin_where"])
        while fl:
            where.append(eng.occ_wait_epoch(fl.popleft())["fin_where"])
        return tnc_before

    stream(2 * lanes)  # warm-up: every lane's graph captured
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tnc_before = stream(k)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / k
    par = eng.tnc == sum(exp[i % lanes][2] for i in range(k))
    for i in range(k - lanes, k):
        erc, etn, _ = exp[i % lanes]
        want = np.where(etn != 0, etn + np.uint64(tnc_before[i]), np.uint64(0))
        par = par and np.array_equal(rcs[i % lanes].cpu().numpy(), erc)
        par = par and np.array_equal(tns[i % lanes].cpu().numpy().view(np.uint64), want)
    hist = eng.history_size
    eng.history_clear()
    eng.tnc = 0
    return {"workload": f"{k} consecutive OCC epochs of {n} YCSB txns x 16 keys (theta=0.9) through "
                        f"the pipeline ({lanes} lanes), each with commit tn and its committed writes "
                        f"appended to the device history (central_finish under TS_CLOCK)",
            "txns_per_s": n / dt, "ms_per_epoch": dt * 1e3,
            "history_pairs_at_end": int(hist),
            "finished_on_device": where.count(1), "finished_by_host": where.count(2),
            "parity_vs_oracle": bool(par),
            "parity_scope": "rc and tn of each lane's last epoch, tnc after the stream",
            "note": "a stream whose epochs carry TS_CAS windows reading the previous epochs' history "
                    "cannot overlap (each window needs the epoch before it finished): see HIST / SHIM"}


def shim_pipe_config(eng, dev, timed, orc, tag="SHIM_PIPE", n=1 << 20, lanes=4, k=24):
    """The shim's transfer form through the pipeline: what OccEpoch
    (deneva_amd/csrc/host/occ_epoch.h, Options::depth = 4) hands the engine
    under the reference's default TS_CLOCK -- HOST arrays in the compact
    pinned form (u32 keys, 2-bit access types), commit tn and the history
    append (central_finish) -- submitted with dcc_occ_submit_epoch, `lanes`
    epochs in flight: each lane's H2D copy overlaps the other lanes' kernels.
    Wall time per epoch over k epochs; each lane's last epoch's rc and tn
    checked against the oracle (tn shifted by the tnc before the epoch)."""
    import torch
    import deneva_amd as d
    from collections import deque
    b = d.gen_ycsb(n_txn=n, zipf_theta=0.9, seed=0xD3E7A00E)
    cb = eng.compact_host_batch(b)
    erc, etn, ecw = orc.occ(b)
    rcs = [eng.host_empty(n, np.uint8) for _ in range(lanes)]
    tns = [eng.host_empty(n, np.uint64) for _ in range(lanes)]
    eng.set_option(d._abi.OPT_PIPELINE, lanes)

    def stream(kk):
        eng.history_clear()
        eng.tnc = 0
        fl = deque()
        for i in range(kk):
            fl.append(eng.occ_submit_epoch(cb, rcs[i % lanes], tns[i % lanes], append_history=True))
            if len(fl) >= lanes:
                eng.occ_wait_epoch(fl.popleft())
        while fl:
            eng.occ_wait_epoch(fl.popleft())

    stream(2 * lanes)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stream(k)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / k
    par = eng.tnc == k * ecw
    for i in range(k - lanes, k):
        want = np.where(etn != 0, etn + np.uint64(i * ecw), np.uint64(0))
        par = par and np.array_equal(np.asarray(rcs[i % lanes]), erc)
        par = par and np.array_equal(np.asarray(tns[i % lanes]), want)
    h2d = sum(int(np.asarray(a).nbytes) for a in (cb.offsets, cb.keys, cb.acctype))
    eng.history_clear()
    eng.tnc = 0
    return {"workload": f"{k} consecutive OCC epochs of {n} YCSB txns x 16 keys (theta=0.9) from pinned "
                        f"host arrays in the shim's compact form, {lanes} epochs in flight, commit tn + "
                        f"history append (central_finish under TS_CLOCK)",
            "txns_per_s": n / dt, "ms_per_epoch": dt * 1e3, "h2d_MB": h2d / 1e6,
            "h2d_GBps_effective": h2d / dt / 1e9,
            "parity_vs_oracle": bool(par),
            "parity_scope": "rc and tn of each lane's last epoch, tnc after the stream"}


def _pcie_h2d_GBps(nbytes):
    """The link: a pinned host -> device copy of nbytes (torch, median of 5)."""
    import torch
    x = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    y = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    ts = []
    for _ in range(6):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        y.copy_(x, non_blocking=True)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return nbytes / float(np.median(ts[1:])) / 1e9


def shim_config(eng, dev, timed, orc, tag="SHIM", n=1 << 20, steps=6):
    """The shipped shim path at the headline size: what OccEpoch::close
    (deneva_amd/csrc/host/occ_epoch.h) hands the engine -- HOST arrays (H2D
    of the CSR and D2H of the decisions inside the call), per-txn TS_CAS
    windows (start_tn, finish_tn], commit tn wanted and the committed writes
    appended to the device history (DCC_OCC_APPEND_HISTORY, central_finish,
    occ.cpp:277-286).  Each step starts from the same history: the committed
    writes of the previous epoch of the same shape (tn 1..).  Legs:
      - compact pinned (the value): the batch in pinned memory in the compact
        transfer form the shim builds (u32 keys, 2-bit access types, u32
        timestamps: dcc.h DCC_KEYS_U32 ...), pinned outputs;
      - wide_pinned: the same call with full-width pinned arrays (u64 keys --
        the INTEGRATION.md binding that passes row_t* identities --, one byte
        per access type, u64 timestamps);
      - pageable_full: full-width pageable arrays;
      - device_resident: the batch and outputs in HBM -- the device time of
        the decision plus central_finish (window check, commit tn, history
        append) replayed from one captured graph.
    Wall time per call (host-synchronous API) and the call's device time
    (for host outputs it includes the D2H of rc and tn, which the graph
    holds)."""
    import torch
    import deneva_amd as d
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
    erc, etn, _ = orc.occ(b, hist_keys=hk, hist_tn=ht, tnc=ptnc)
    cb = eng.compact_host_batch(b)

    def pin(a, dt):
        out = eng.host_empty(np.asarray(a).size, dt)
        out[...] = np.asarray(a)
        return out
    wb = d.EpochBatch(pin(b.offsets, np.uint32), pin(b.keys, np.uint64), pin(b.acctype, np.uint8),
                      pin(b.start_tn, np.uint64), pin(b.finish_tn, np.uint64))
    db = b.to_torch(dev)
    out_rc, out_tn = eng.host_empty(n, np.uint8), eng.host_empty(n, np.uint64)
    d_rc = torch.empty(n, dtype=torch.uint8, device=dev)
    d_tn = torch.empty(n, dtype=torch.int64, device=dev)
    nbytes = lambda x: sum(int(a.nbytes) for a in (x.offsets, x.keys, x.acctype, x.start_tn,
                                                     x.finish_tn))
    h2d, h2d_wide = nbytes(cb), nbytes(wb)

    def run(batch, outs, k):
        walls, devs, res = [], [], None
        for i in range(k + 2):
            eng.history_clear()
            eng.history_append(hk, ht)
            eng.tnc = ptnc
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rc, tn, st = eng.occ_validate_epoch(batch, want_tn=True, append_history=True, **outs)
            if batch.on_device:
                torch.cuda.synchronize()
            w = time.perf_counter() - t0
            if i >= 2:  # warmup
                walls.append(w)
                devs.append(st["device_ms"])
            res = ((rc.cpu().numpy() if batch.on_device else np.asarray(rc)).copy(),
                   (tn.cpu().numpy() if batch.on_device else np.asarray(tn)).astype(np.uint64).copy())
        par = bool(np.array_equal(res[0], erc) and np.array_equal(res[1], etn))
        return float(np.median(walls)), float(np.median(devs)), par

    pinned_out = {"out_rc": out_rc, "out_tn": out_tn}
    wall, devm, par = run(cb, pinned_out, steps)
    wall_w, devm_w, par_w = run(wb, pinned_out, steps)
    wall_p, _, par_p = run(b, {}, 3)
    wall_d, devm_d, par_d = run(db, {"out_rc": d_rc, "out_tn": d_tn}, steps)
    eng.history_clear()
    eng.tnc = 0
    return {"workload": f"OCC epoch of {n} YCSB txns x 16 keys (theta=0.9) through the shim's path: "
                        f"host arrays, TS_CAS windows against a {hk.size}-pair history, commit tn, "
                        f"history append",
            "txns_per_s": n / wall, "ms_per_epoch": wall * 1e3, "device_ms": devm,
            "h2d_MB": h2d / 1e6, "pcie_h2d_GBps": _pcie_h2d_GBps(h2d),
            "h2d_GBps_in_call": h2d / 1e9 / max(wall - devm * 1e-3, 1e-9),
            "wide_pinned": {"ms_per_epoch": wall_w * 1e3, "device_ms": devm_w, "h2d_MB": h2d_wide / 1e6,
                            "parity_vs_oracle": par_w,
                            "note": "u64 keys (row_t* identities), byte access types, u64 timestamps"},
            "pageable_full": {"ms_per_epoch": wall_p * 1e3, "parity_vs_oracle": par_p},
            "device_resident": {"device_ms": devm_d, "ms_per_epoch": wall_d * 1e3,
                                "parity_vs_oracle": par_d,
                                "note": "batch and outputs in HBM: window check + decision + commit tn + "
                                        "history append, one graph replay"},
            "note": "wall includes H2D of the compact pinned CSR (h2d_MB), the on-device widening, "
                    "D2H of rc + tn into pinned outputs (inside the replayed graph, so in device_ms)",
            "parity_vs_oracle": par and par_w and par_p and par_d}


CONFIGS = {"C2": occ_config, "C3": occ_config, "C5": occ_config, "C4": calvin_config,
           "C4_SHUF": calvin_config,
           "C6": None, "HIST": history_config, "SHIM": shim_config, "SHIM_PIPE": shim_pipe_config,
           "PIPE_FIN": pipe_fin_config,
           "MAAT_C2": maat_config,
           "MAAT_1M": maat_config}


def secondary_configs(eng, local, steps=10, warmup=3, only=None):
    """The other BASELINE.json configs (and the §8(f) engines) on one GPU,
    each its own workload; inputs resident, decisions checked against the
    oracle outside the timing."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as orc  # checker only
    dev = f"cuda:{local}"
    timed = _timer(steps, warmup)
    out = {}
    for tag, fn in CONFIGS.items():
        if only and tag not in only:
            continue
        out[tag] = (snapshot_config(eng, dev, timed, orc) if tag == "C6"
                    else fn(eng, dev, timed, orc, tag))
        if tag == "SHIM":  # the INTEGRATION.md binding (row_t* keys): full-width pinned arrays
            w = out[tag]["wide_pinned"]
            out["SHIM_WIDE"] = {"workload": out[tag]["workload"] + ", full-width pinned arrays",
                                "txns_per_s": (1 << 20) / (w["ms_per_epoch"] * 1e-3), **w}
    return out


def snapshot_capture(n, seed=0xD3E7A006, max_active=8, n_hist=20000):
    """Synthetic live capture over the headline batch shape: txn i's critical
    section saw up to `max_active` of the 64 txns before it on the active list,
    a history head hist_top, and a TS_CAS window (start_tn, finish_tn]."""
    import deneva_amd as d
    rng = np.random.default_rng(seed)
    b = d.gen_ycsb(n_txn=n, zipf_theta=0.9)
    cnt = np.minimum(rng.integers(0, max_active + 1, size=n), np.arange(n))
    aoff = np.zeros(n + 1, np.uint32)
    aoff[1:] = np.cumsum(cnt)
    t = np.repeat(np.arange(n, dtype=np.int64), cnt)
    aidx = (t - 1 - rng.integers(0, 64, size=t.size) % np.maximum(t, 1)).astype(np.uint32)
    st = rng.integers(0, 1200, size=n).astype(np.uint64)
    ft = st + rng.integers(0, 8, size=n).astype(np.uint64)
    top = rng.integers(0, 1200, size=n).astype(np.uint64)
    hk = b.keys[rng.integers(0, b.nnz, size=n_hist)].astype(np.uint64)
    ht = rng.integers(1, 1200, size=n_hist).astype(np.uint64)
    return d.EpochBatch(b.offsets, b.keys, b.acctype, st, ft), aoff, aidx, top, hk, ht


def snapshot_config(eng, dev, timed, orc, n=1 << 20, check=131072):
    """C6: captured-snapshot validation (dcc_occ_validate_snapshot) of 1M
    captured YCSB txns; parity on the first `check` txns (a capture prefix only
    refers to earlier txns, so it is self-contained)."""
    import torch
    from deneva_amd import EpochBatch
    b, aoff, aidx, top, hk, ht = snapshot_capture(n)
    eng.history_clear()
    eng.history_append(hk, ht)
    db = b.to_torch(dev)
    t32 = lambda a: torch.from_numpy(a.view(np.int32)).to(dev)
    daoff, daidx = t32(aoff), t32(aidx)
    dtop = torch.from_numpy(top.view(np.int64)).to(dev)
    rc = torch.empty(n, dtype=torch.uint8, device=dev)
    dt, st = timed(lambda: eng.occ_validate_snapshot(db, daoff, daidx, dtop, out_rc=rc)[1])
    off = b.offsets[: check + 1]
    sub = EpochBatch(off, b.keys[: off[-1]], b.acctype[: off[-1]], b.start_tn[:check],
                     b.finish_tn[:check])
    erc = orc.occ_snapshot(sub, aoff[: check + 1], aidx[: aoff[check]], top[:check], hk, ht)
    eng.history_clear()
    return {"workload": "captured-snapshot OCC, 1,048,576 YCSB txns x 16 keys (theta=0.9), "
                        "<=8 captured active txns each, 20,000-pair history, TS_CAS windows",
            "txns_per_s": n / dt, "ms_per_epoch": dt * 1e3, "device_ms": st["device_ms"],
            "commits": int(st["n_commit"]), "alg_bytes": int(st["alg_bytes"]),
            "alg_GBps": st["alg_bytes"] / (st["device_ms"] * 1e-3) / 1e9,
            "parity_vs_oracle": bool(np.array_equal(rc[:check].cpu().numpy(), erc)),
            "parity_sample": f"first {check} txns"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import deneva_amd as d
    if args.only:
        torch.cuda.set_device(0)
        with d.Engine(0) as eng:
            eng.set_option(d._abi.OPT_SOLVER, args.solver)
            print(json.dumps(secondary_configs(eng, 0, steps=args.steps, warmup=args.warmup,
                                               only=args.only.split(","))), flush=True)
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.exchange == "host":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        if args.exchange == "rccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    # same batch on every rank (deterministic generator); weak scaling: the
    # epoch grows with the GPU count, each GPU holds 1/N of the accesses
    n_total = args.txns if args.strong else args.txns * world
    batch = d.gen_ycsb(n_txn=n_total, zipf_theta=args.theta, req_per_query=args.keys,
                       seed=args.seed)
    eng = d.Engine(local)
    eng.set_option(d._abi.OPT_SOLVER, args.solver)
    if args.sweep_levels:
        eng.set_option(d._abi.OPT_SWEEP_LEVELS, args.sweep_levels)
    if args.ro_split >= 0:
        eng.set_option(d._abi.OPT_RO_SPLIT, args.ro_split)
    if world > 1:
        if args.exchange == "rccl":
            uid = d.comm_unique_id() if rank == 0 else bytes(d._abi.UNIQUE_ID_BYTES)
            obj = [uid]
            dist.broadcast_object_list(obj, src=0)
            eng.comm_init(rank, world, obj[0])
        else:
            def allreduce_max(buf):
                t = torch.from_numpy(buf)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
            eng.comm_init_host(rank, world, allreduce_max)
    # every rank takes the whole epoch and keeps its key shard of the accesses
    # on its GPU (DCC_SHARD_SELF): the sweep's serial ranges come from the
    # rank's own copy, so ranks exchange only the filters' kill bits
    mine = batch
    dbatch = mine.to_torch(f"cuda:{local}")
    out_rc = torch.empty(n_total, dtype=torch.uint8, device=f"cuda:{local}")
    torch.cuda.synchronize()

    def step(profile=False):
        return eng.occ_validate_epoch(dbatch, out_rc=out_rc, shard_self=world > 1)[2]

    # Pipelined headline (N=1): consecutive epochs over L distinct resident
    # batches of the same workload (seeds seed, seed+1, ...), one per lane,
    # L epochs in flight (dcc_occ_submit_epoch).  Each step is
    # one whole epoch; every lane's decisions are checked after the run.
    lanes = args.pipeline if world == 1 else 0
    pipe_batches, pipe_outs = [], []
    if lanes:
        eng.set_option(d._abi.OPT_PIPELINE, lanes)
        eng.set_option(d._abi.OPT_PIPE_PARTITION, args.partition)
        pipe_batches = [batch] + [d.gen_ycsb(n_txn=n_total, zipf_theta=args.theta,
                                             req_per_query=args.keys, seed=args.seed + i)
                                  for i in range(1, lanes)]
        pipe_dev = [b.to_torch(f"cuda:{local}") for b in pipe_batches]
        pipe_outs = [torch.empty(n_total, dtype=torch.uint8, device=f"cuda:{local}")
                     for _ in range(lanes)]
        torch.cuda.synchronize()

    host_split = [0.0, 0.0]  # host seconds inside submit / wait (last run)

    def run_pipelined(k_steps):
        from collections import deque
        inflight, sts = deque(), []
        host_split[0] = host_split[1] = 0.0
        for k in range(k_steps):
            i = k % lanes
            t0 = time.perf_counter()
            inflight.append(eng.occ_submit_epoch(pipe_dev[i], pipe_outs[i]))
            t1 = time.perf_counter()
            host_split[0] += t1 - t0
            if len(inflight) >= lanes:
                sts.append(eng.occ_wait_epoch(inflight.popleft()))
                host_split[1] += time.perf_counter() - t1
        while inflight:
            sts.append(eng.occ_wait_epoch(inflight.popleft()))
        return sts

    def timed_region(fn):
        # barrier + sync on both sides, max over ranks
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        if world > 1:
            dev = f"cuda:{local}" if args.exchange == "rccl" else "cpu"
            t = torch.tensor([dt], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        return dt, out

    dt, pipe_stats = None, None
    if lanes:
        import gc
        run_pipelined(max(args.warmup, 3 * lanes))
        gc.collect()
        gc.disable()  # no collector pauses inside the timed loop
        try:
            dt, pipe_stats = timed_region(lambda: run_pipelined(args.steps))
        finally:
            gc.enable()
    # one epoch at a time: the single-epoch latency (device events per epoch)
    for _ in range(args.warmup):
        step()
    dt_lat, stats = timed_region(lambda: [step() for _ in range(args.steps)])
    if dt is None:
        dt = dt_lat

    # per-phase kernel times (HIP events on the engine stream), separate pass
    eng.set_profiling(True)
    prof = [step() for _ in range(max(3, min(args.steps, 10)))]
    eng.set_profiling(False)
    ph_ms = np.mean([p["phase_ms"] for p in prof], axis=0)
    ph_bytes = prof[-1]["phase_bytes"]
    # the one kernel that streams the whole epoch (every offset, key and access
    # type): the level-0 committed-key filter; reported as a
    # sub-field, the headline roofline is the whole epoch
    filt = {"kernel": "k_sw_filter (level 0: the committed-key filter over the whole epoch)",
            "alg_bytes_per_launch": int(ph_bytes[1]), "avg_launch_ms": float(ph_ms[1]),
            "achieved": ph_bytes[1] / (ph_ms[1] * 1e-3) / 1e9 if ph_ms[1] > 0 else None}
    if filt["achieved"] is not None:
        filt["frac"] = filt["achieved"] / HBM_PEAK_GBS

    copies = stream_copy_both(f"cuda:{local}") if rank == 0 else None
    copy_gbps = max(v for v in copies.values() if v) if copies else None
    s0 = stats[-1]
    ms_per_step = dt / args.steps * 1e3
    value = n_total * args.steps / dt
    dev_ms = float(np.mean([s["device_ms"] for s in stats]))
    lat_gbs = s0["alg_bytes"] / (dev_ms * 1e-3) / 1e9
    # the headline's roofline: algorithmic bytes of the epochs over the timed
    # region (throughput basis; wall clock, so host gaps count against it);
    # the single-epoch latency basis is kept beside it
    alg_per_epoch = (float(np.mean([s["alg_bytes"] for s in pipe_stats])) if pipe_stats
                     else float(s0["alg_bytes"]))
    epoch_gbs = alg_per_epoch * args.steps / dt / 1e9 if pipe_stats else lat_gbs
    basis_ms = dt / args.steps * 1e3 if pipe_stats else dev_ms  # time per epoch of the roofline

    # parity check of the measured decisions against the oracle (rank 0, N=1)
    parity = None
    cpu = None
    if rank == 0:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import _oracle as orc  # checker only, outside the timed region
        erc, _, _ = orc.occ(batch)
        parity = bool(np.array_equal(out_rc.cpu().numpy(), erc))
        pipe_parity = None
        if lanes:
            pipe_parity = [bool(np.array_equal(o.cpu().numpy(), erc if i == 0 else orc.occ(b)[0]))
                           for i, (b, o) in enumerate(zip(pipe_batches, pipe_outs))]
            parity = parity and all(pipe_parity)
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(batch, args.cpu_sample)
    secondary = None
    if world == 1 and not args.no_secondary:
        secondary = secondary_configs(eng, local)

    if rank == 0:
        # HBM traffic and L2 hit rates of one epoch (PMC FETCH_SIZE x2 +
        # WRITE_SIZE, TCC_HIT / (HIT + MISS), per dispatch, tools/gpu_pmc_r03.sh),
        # read from the committed summary named by --pmc: null for workloads
        # it does not describe (N > 1, other sizes)
        pmc = None
        if (os.path.exists(args.pmc) and world == 1 and n_total == 1 << 20 and args.theta == 0.9
                and args.keys == 16):
            try:
                pmc = json.load(open(args.pmc))
            except (OSError, ValueError):
                pmc = None
        hp = (pmc or {}).get("headline") or {}
        traffic = hp.get("epoch_bytes")
        traffic_src = (f"{os.path.relpath(args.pmc, ROOT)} ({pmc.get('source', '')}; "
                       f"{pmc.get('correction', '')})") if pmc else None
        if pmc and secondary:
            # per-workload traffic next to each config's own device time
            for tag, sec in secondary.items():
                pw = pmc.get(tag) or {}
                if not pw.get("epoch_bytes") or not isinstance(sec, dict):
                    continue
                ks = pw.get("kernels") or {}
                top = sorted(ks.items(), key=lambda kv: -(kv[1].get("fetch_bytes", kv[1].get("fetch_bytes_max", 0)) +
                                                          kv[1].get("write_bytes", kv[1].get("write_bytes_max", 0))))[:6]
                dms = sec.get("device_ms")
                sec["pmc"] = {
                    "source": traffic_src,
                    "epoch_traffic_bytes": pw.get("epoch_bytes"),
                    "epoch_l2_hit": pw.get("epoch_l2_hit"),
                    "actual_GBps": pw["epoch_bytes"] / (dms * 1e-3) / 1e9 if dms else None,
                    "top_kernels": {k: {"fetch_bytes": v.get("fetch_bytes", v.get("fetch_bytes_max")),
                                        "write_bytes": v.get("write_bytes", v.get("write_bytes_max")),
                                        "l2_hit": v.get("l2_hit")} for k, v in top}}
        line = {
            "metric": "OCC-validated txns/sec, YCSB theta=0.9",
            "value": value,
            "unit": "txns/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong" if args.strong else "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (deterministic YCSB generator, restated gen_requests_zipf)",
            "config": {
                "workload": f"YCSB OCC epoch validation, {n_total} txns x {args.keys} keys, "
                            f"zipf theta={args.theta}, 16,777,216-key table, 50% RO txns, "
                            f"50% WR tuples",
                "global_batch": n_total,
                "keys_per_txn": args.keys,
                "parallelism": (f"key-shard x{world} ({args.exchange} kill-bit all-gather, whole epoch per rank)" if world > 1
                                else "single GPU"),
            },
            "pipeline": ({
                "lanes": lanes,
                "partition": ("lane i on 1/lanes of every XCD's CUs (CU-masked streams)"
                              if args.partition else "every lane on the whole chip"),
                "ms_per_epoch_steady": dt / args.steps * 1e3,
                "txns_per_s": value,
                "batches": f"{lanes} distinct resident batches (seeds {args.seed:#x}+0..{lanes - 1}), "
                           f"epoch k on lane k mod {lanes}",
                "parity_vs_oracle_per_lane": pipe_parity,
                "epoch_span_ms_mean": float(np.mean([s["device_ms"] for s in pipe_stats])),
                "host_us_per_epoch": {"submit": host_split[0] / args.steps * 1e6,
                                      "wait": host_split[1] / args.steps * 1e6},
            } if pipe_stats else None),
            "single_epoch": {
                "ms_per_epoch_wall": dt_lat / args.steps * 1e3,
                "txns_per_s": n_total * args.steps / dt_lat,
                "device_ms": dev_ms,
                "alg_GBps": lat_gbs,
                "hbm_frac": lat_gbs / HBM_PEAK_GBS,
            },
            "roofline": {
                "bound": "hbm",
                "scope": ("whole epochs, throughput basis: algorithmic bytes of the K pipelined "
                          "epochs over the timed region's wall clock (SURVEY.md 8(d)); "
                          "single-epoch latency basis in single_epoch" if pipe_stats else
                          "whole epoch: every kernel of dcc_occ_validate_epoch, HIP events "
                          "around the epoch on the engine stream (SURVEY.md 8(d))"),
                "achieved": epoch_gbs,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": epoch_gbs / HBM_PEAK_GBS,
                "stream_copy_GBps": copy_gbps,
                "stream_copy_variants_GBps": copies,
                "frac_of_stream_copy": epoch_gbs / copy_gbps if copy_gbps else None,
                "traffic": traffic,
                # HBM bytes actually moved per second of epoch (PMC traffic / device time)
                "actual_GBps": (traffic / (basis_ms * 1e-3) / 1e9) if traffic else None,
                "traffic_source": traffic_src,
                "l2_hit": {"epoch": hp.get("epoch_l2_hit"),
                           "filter": _kern_l2(hp, "k_sw_filter"),
                           "serial_pass": _kern_l2(hp, "k_sw_seq"),
                           "pre_pass": _kern_l2(hp, "k_sw_pre")} if hp else None,
                "alg_bytes_per_launch": int(alg_per_epoch),
                "avg_launch_ms": basis_ms,
                "streaming_kernel": filt,
            },
            "epoch": {
                "device_ms": dev_ms,
                "alg_bytes": int(s0["alg_bytes"]),
                "alg_GBps": lat_gbs,
                "hbm_frac": lat_gbs / HBM_PEAK_GBS,
                "rounds": int(s0["rounds"]),
                "commits": int(s0["n_commit"]),
                "aborts": int(s0["n_abort"]),
                "phase_ms": [float(x) for x in ph_ms],
                "phases": ["level-0 tile lists+serial pass+committed set",
                           "level-0 filter kernel", "level-0 compaction+later levels",
                           "prep+final"],
                "peel_prefix": int(s0["peel_prefix"]),
                "survivors": int(s0["n_survivors"]),
                "parity_vs_oracle": parity,
            },
            "cpu_baseline": cpu,
            "other_configs": secondary,
        }
        print(json.dumps(line), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
