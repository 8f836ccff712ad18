"""ctypes view of oracle/liboracle.so — the CPU restatements used as the checker.

TEST INFRASTRUCTURE ONLY (see oracle/oracle.h): imported by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg, never by deneva_amd.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB = os.path.join(ORACLE_DIR, "liboracle.so")


def _load():
    srcs = [os.path.join(ORACLE_DIR, f) for f in ("occ_ref.c", "occ_mt.c", "occ_sweep_mt.c", "calvin_ref.c", "maat_ref.c", "oracle.h", "kmap.h")]
    if not os.path.exists(LIB) or any(os.path.getmtime(s) > os.path.getmtime(LIB) for s in srcs
                                      if os.path.exists(s)):
        subprocess.run(["make", "-C", ORACLE_DIR], check=True, capture_output=True)
    lib = C.CDLL(LIB)
    P = C.c_void_p
    lib.oracle_occ_replay.argtypes = [C.c_uint64, P, P, P, P, P, C.c_uint64, P, P,
                                      C.POINTER(C.c_uint64), P, P]
    lib.oracle_occ_hash.argtypes = lib.oracle_occ_replay.argtypes
    lib.oracle_occ_snapshot.argtypes = [C.c_uint64, P, P, P, P, P, P, P, P, C.c_uint64, P, P, P]
    lib.oracle_occ_snapshot.restype = C.c_int
    lib.oracle_occ_rounds_mt.argtypes = [C.c_uint64, P, P, P, C.c_int, C.POINTER(C.c_uint64), P,
                                         P, C.POINTER(C.c_uint32)]
    lib.oracle_occ_rounds_mt.restype = C.c_int
    lib.oracle_occ_sweep_mt.argtypes = lib.oracle_occ_rounds_mt.argtypes
    lib.oracle_occ_sweep_mt.restype = C.c_int
    lib.oracle_occ_round_status.argtypes = [C.c_uint64, P, P, P, P, P]
    lib.oracle_calvin_replay.argtypes = [C.c_uint64, P, P, P, P, P, P, P]
    lib.oracle_calvin_formula.argtypes = lib.oracle_calvin_replay.argtypes
    lib.oracle_maat_replay.argtypes = [C.c_uint64, P, P, P, C.c_int, C.c_uint64, P, P, P, P, P]
    lib.oracle_maat_formula.argtypes = lib.oracle_maat_replay.argtypes
    for f in (lib.oracle_occ_replay, lib.oracle_occ_hash, lib.oracle_occ_round_status,
              lib.oracle_calvin_replay, lib.oracle_calvin_formula, lib.oracle_maat_replay,
              lib.oracle_maat_formula):
        f.restype = C.c_int
    return lib


lib = _load()


def _p(a):
    return None if a is None else np.ascontiguousarray(a).ctypes.data


def _arr(a, dt):
    return None if a is None else np.ascontiguousarray(a, dt)


def occ(batch, hist_keys=None, hist_tn=None, tnc=0, literal=False):
    """Returns (rc u8[n], tn u64[n], tnc_after)."""
    n = batch.n_txn
    off = _arr(batch.offsets, np.uint32)
    keys = _arr(batch.keys, np.uint64)
    at = _arr(batch.acctype, np.uint8)
    st = _arr(batch.start_tn, np.uint64)
    ft = _arr(batch.finish_tn, np.uint64)
    hk = _arr(hist_keys, np.uint64)
    ht = _arr(hist_tn, np.uint64)
    nh = 0 if hk is None else hk.shape[0]
    rc = np.empty(max(n, 1), np.uint8)
    tn = np.empty(max(n, 1), np.uint64)
    t = C.c_uint64(tnc)
    fn = lib.oracle_occ_replay if literal else lib.oracle_occ_hash
    r = fn(n, _p(off), _p(keys), _p(at), _p(st), _p(ft), nh, _p(hk), _p(ht), C.byref(t),
           rc.ctypes.data, tn.ctypes.data)
    if r != 0:
        raise RuntimeError(f"oracle occ failed: {r}")
    return rc[:n], tn[:n], t.value


def occ_rounds_mt(batch, nthreads, tnc=0):
    """ROUNDS-MT CPU baseline: returns (rc u8[n], tn u64[n], tnc_after, rounds)."""
    n = batch.n_txn
    off = _arr(batch.offsets, np.uint32)
    keys = _arr(batch.keys, np.uint64)
    at = _arr(batch.acctype, np.uint8)
    rc = np.empty(max(n, 1), np.uint8)
    tn = np.empty(max(n, 1), np.uint64)
    t = C.c_uint64(tnc)
    rounds = C.c_uint32(0)
    r = lib.oracle_occ_rounds_mt(n, _p(off), _p(keys), _p(at), int(nthreads), C.byref(t),
                                 rc.ctypes.data, tn.ctypes.data, C.byref(rounds))
    if r != 0:
        raise RuntimeError(f"oracle rounds-mt failed: {r}")
    return rc[:n], tn[:n], t.value, rounds.value


def occ_sweep_mt(batch, nthreads, tnc=0):
    """SWEEP-MT CPU baseline: returns (rc u8[n], tn u64[n], tnc_after, levels)."""
    n = batch.n_txn
    off = _arr(batch.offsets, np.uint32)
    keys = _arr(batch.keys, np.uint64)
    at = _arr(batch.acctype, np.uint8)
    rc = np.empty(max(n, 1), np.uint8)
    tn = np.empty(max(n, 1), np.uint64)
    t = C.c_uint64(tnc)
    lv = C.c_uint32(0)
    r = lib.oracle_occ_sweep_mt(n, _p(off), _p(keys), _p(at), int(nthreads), C.byref(t),
                                rc.ctypes.data, tn.ctypes.data, C.byref(lv))
    if r != 0:
        raise RuntimeError(f"oracle sweep-mt failed: {r}")
    return rc[:n], tn[:n], t.value, lv.value


def occ_snapshot(batch, active_off, active_idx, hist_top=None, hist_keys=None, hist_tn=None):
    """Literal captured-snapshot validation; returns rc u8[n]."""
    n = batch.n_txn
    off = _arr(batch.offsets, np.uint32)
    keys = _arr(batch.keys, np.uint64)
    at = _arr(batch.acctype, np.uint8)
    st = _arr(batch.start_tn, np.uint64)
    ft = _arr(batch.finish_tn, np.uint64)
    top = _arr(hist_top, np.uint64)
    ao = _arr(active_off, np.uint32)
    ai = _arr(active_idx, np.uint32)
    if ai is not None and ai.shape[0] == 0:
        ai = np.zeros(1, np.uint32)
    hk = _arr(hist_keys, np.uint64)
    ht = _arr(hist_tn, np.uint64)
    nh = 0 if hk is None else hk.shape[0]
    rc = np.empty(max(n, 1), np.uint8)
    r = lib.oracle_occ_snapshot(n, _p(off), _p(keys), _p(at), _p(st), _p(ft), _p(top), _p(ao),
                                _p(ai), nh, _p(hk), _p(ht), rc.ctypes.data)
    if r != 0:
        raise RuntimeError(f"oracle occ snapshot failed: {r}")
    return rc[:n]


def occ_round_status(batch, state):
    n = batch.n_txn
    off = _arr(batch.offsets, np.uint32)
    keys = _arr(batch.keys, np.uint64)
    at = _arr(batch.acctype, np.uint8)
    state = _arr(state, np.uint8)
    out = np.empty(max(n, 1), np.uint8)
    r = lib.oracle_occ_round_status(n, _p(off), _p(keys), _p(at), _p(state), out.ctypes.data)
    if r != 0:
        raise RuntimeError("oracle round status failed")
    return out[:n]


def calvin(batch, literal=False):
    """Returns (group u32[nnz], rc u8[n], wave u32[n])."""
    n, nnz = batch.n_txn, batch.nnz
    off = _arr(batch.offsets, np.uint32)
    keys = _arr(batch.keys, np.uint64)
    at = _arr(batch.acctype, np.uint8)
    order = _arr(batch.order, np.uint64)
    g = np.empty(max(nnz, 1), np.uint32)
    rc = np.empty(max(n, 1), np.uint8)
    w = np.empty(max(n, 1), np.uint32)
    fn = lib.oracle_calvin_replay if literal else lib.oracle_calvin_formula
    r = fn(n, _p(off), _p(keys), _p(at), _p(order), g.ctypes.data, rc.ctypes.data, w.ctypes.data)
    if r != 0:
        raise RuntimeError(f"oracle calvin failed: {r}")
    return g[:nnz], rc[:n], w[:n]


def calvin_held(batch, held_keys, held_acctype, literal=True):
    """Calvin against a pre-seeded lock table: the held requests (per row,
    owners first, then waiters) are replayed through Row_lock first as
    one-request pseudo-txns, then the epoch in sequence order (the literal
    oracle_calvin_replay over the combined batch).  Returns the epoch's
    (group u32[nnz], rc u8[n])."""
    from deneva_amd import EpochBatch
    h = int(len(held_keys))
    n = batch.n_txn
    off = _arr(batch.offsets, np.uint32).astype(np.uint64)
    coff = np.concatenate([np.arange(h + 1, dtype=np.uint64), h + off[1:]]).astype(np.uint32)
    ckeys = np.concatenate([np.asarray(held_keys, np.uint64), _arr(batch.keys, np.uint64)])
    cat = np.concatenate([np.asarray(held_acctype, np.uint8), _arr(batch.acctype, np.uint8)])
    if batch.order is None:
        pos = np.arange(n, dtype=np.uint64)
    else:
        seq = np.argsort(_arr(batch.order, np.uint64), kind="stable")
        pos = np.empty(n, np.uint64)
        pos[seq] = np.arange(n, dtype=np.uint64)
    corder = np.concatenate([np.arange(h, dtype=np.uint64), np.uint64(h) + pos])
    cb = EpochBatch(coff, ckeys, cat, order=corder)
    g, rc, _ = calvin(cb, literal=literal)
    return g[h:], rc[h:]


def maat(batch, row_keys=None, row_lr=None, row_lw=None, rw_all=False, literal=False):
    """MaaT epoch (oracle_maat_replay / _formula).  Returns (rc u8[n],
    cts u64[n], (keys, lr, lw) of every row touched or pre-seeded, after)."""
    n = batch.n_txn
    off = _arr(batch.offsets, np.uint32)
    keys = _arr(batch.keys, np.uint64)
    at = _arr(batch.acctype, np.uint8)
    pre_k = np.zeros(0, np.uint64) if row_keys is None else np.asarray(row_keys, np.uint64)
    rk = np.unique(np.concatenate([pre_k, keys if keys is not None else np.zeros(0, np.uint64)]))
    lr = np.zeros(rk.size, np.uint64)
    lw = np.zeros(rk.size, np.uint64)
    if pre_k.size:
        pos = np.searchsorted(rk, pre_k)
        lr[pos] = np.asarray(row_lr, np.uint64)
        lw[pos] = np.asarray(row_lw, np.uint64)
    rc = np.empty(max(n, 1), np.uint8)
    cts = np.empty(max(n, 1), np.uint64)
    fn = lib.oracle_maat_replay if literal else lib.oracle_maat_formula
    r = fn(n, _p(off), _p(keys), _p(at), 1 if rw_all else 0, rk.size, _p(rk), _p(lr), _p(lw),
           rc.ctypes.data, cts.ctypes.data)
    if r != 0:
        raise RuntimeError(f"oracle maat failed: {r}")
    return rc[:n], cts[:n], (rk, lr, lw)
