"""A genuinely concurrent OptCC run, simulated on the CPU, with capture.

TEST INFRASTRUCTURE ONLY.  Worker threads interleave txns through
start -> validate (critical section) -> finish, as WorkerThread does under
central OCC:
  * start:     start_tn = get_ts()                  worker_thread.cpp:500-502
  * validate:  critical section (occ.cpp:137-158): finish_tn = get_ts(),
               finish_active = active list, his = history head; non-read-only
               txns push their write set on `active`; then the history window
               (occ.cpp:167-180, read set only) and the active check (:185-199);
               an aborting txn unlinks itself from `active` (:219-235)
  * finish:    central_finish (occ.cpp:248-294): unlink, and on commit
               tn = ++tnc and push on `history`
get_ts is TS_CAS (manager.cpp:41-70: a global counter +1 per call), so the
history window opens.  The run decides every txn itself; it also records the
capture (hist_top, active_off, active_idx, start_tn, finish_tn) that
dcc_occ_validate_snapshot must reproduce the decisions from.
"""
from __future__ import annotations

import heapq

import numpy as np

WR = 1


def simulate(offsets, keys, acctype, n_threads=8, seed=0, hist0=None, tnc0=0,
             exec_span=(1, 40), finish_span=(1, 20)):
    """Run the txns of the CSR batch (in index order of arrival, round-robin
    over threads).  hist0 = [(tn, [keys])] committed before the run.
    Returns dict with the capture, the live decisions and the final history."""
    rng = np.random.default_rng(seed)
    n = len(offsets) - 1
    rsets, wsets = [], []
    for t in range(n):
        a, b = int(offsets[t]), int(offsets[t + 1])
        ks, ts = keys[a:b], acctype[a:b]
        wsets.append(set(int(k) for k, ty in zip(ks, ts) if ty == WR))
        rsets.append(set(int(k) for k, ty in zip(ks, ts) if ty != WR))
    clock = 0
    tnc = tnc0
    history = list(hist0 or [])  # ascending tn; head = last
    active = []                  # txn ids whose wset is on the active list
    start_tn = np.zeros(n, np.uint64)
    finish_tn = np.zeros(n, np.uint64)
    hist_top = np.zeros(n, np.uint64)
    act_lists = [None] * n
    rc = np.zeros(n, np.uint8)
    commit_tn = np.zeros(n, np.uint64)
    queues = [list(range(th, n, n_threads)) for th in range(n_threads)]
    ev = []  # (time, seq, thread, phase, txn)
    seq = 0
    for th in range(n_threads):
        if queues[th]:
            heapq.heappush(ev, (int(rng.integers(0, 5)), seq, th, 0, queues[th].pop(0)))
            seq += 1
    while ev:
        now, _, th, phase, t = heapq.heappop(ev)
        nxt = None
        if phase == 0:  # start
            clock += 1
            start_tn[t] = clock
            nxt = (now + int(rng.integers(*exec_span)), 1)
        elif phase == 1:  # validate: critical section, then the checks
            clock += 1
            finish_tn[t] = clock
            snap = list(active)
            act_lists[t] = snap
            hist_top[t] = history[-1][0] if history else 0
            his = list(history)  # the stack as seen now
            ro = not wsets[t]
            if not ro:
                active.append(t)
            valid = True
            if finish_tn[t] > start_tn[t]:
                for tn, hk in reversed(his):
                    if tn > finish_tn[t]:
                        continue
                    if tn <= start_tn[t]:
                        break
                    if rsets[t] & set(hk):
                        valid = False
                        break
            if valid:
                for j in snap:
                    if wsets[j] & (rsets[t] | wsets[t]):
                        valid = False
                        break
            rc[t] = 0 if valid else 2
            if not valid:
                if t in active:
                    active.remove(t)
            else:
                nxt = (now + int(rng.integers(*finish_span)), 2)
        else:  # finish
            if wsets[t]:
                active.remove(t)
                tnc += 1
                commit_tn[t] = tnc
                history.append((tnc, sorted(wsets[t])))
        if nxt is not None:
            heapq.heappush(ev, (nxt[0], seq, th, nxt[1], t))
            seq += 1
        elif queues[th]:
            heapq.heappush(ev, (now + 1, seq, th, 0, queues[th].pop(0)))
            seq += 1
    aoff = np.zeros(n + 1, np.uint32)
    for t in range(n):
        aoff[t + 1] = aoff[t] + len(act_lists[t])
    aidx = np.array([j for t in range(n) for j in act_lists[t]], np.uint32)
    hk = np.array([k for tn, ks in history for k in ks], np.uint64)
    ht = np.array([tn for tn, ks in history for k in ks], np.uint64)
    return dict(start_tn=start_tn, finish_tn=finish_tn, hist_top=hist_top, active_off=aoff,
                active_idx=aidx, rc=rc, commit_tn=commit_tn, hist_keys=hk, hist_tn=ht, tnc=tnc)
