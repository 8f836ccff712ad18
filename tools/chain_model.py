"""CPU model of the chained central_finish protocol (TEST INFRASTRUCTURE ONLY).

Device side (occ_history.hip k_fin_prep / k_fin, OccFinArgs::ctl): the
context's FinCtl {tnc, hist_m, seq}.  Epoch s's chained finish runs on its
lane after its decision and after the previous epoch's last submitted work
(its lane's ev_done: that epoch's chained finish, or its decision when it has
none).  k_fin_prep snapshots FinCtl; k_fin numbers the epoch from the
snapshot only when snapshot.seq == s, and its last workgroup advances FinCtl
to {tnc + commits, hist_m + pairs, s + 1} only when the epoch was final
(status 1); a not-final epoch numbered from a current snapshot writes pairs
but does not advance (status 2); a stale snapshot writes nothing (status 0).

Host side (occ_pipe.cpp pipe_complete_front): epochs complete in submit
order.  Status 1: the host's tnc / delta size follow the totals.  Otherwise
(and for an epoch without a finish) the host finishes the epoch itself from
its own tnc / delta size and, when chained epochs are in flight behind it,
enqueues chain_set(s + 1) = {host tnc, delta size, s + 1} on the epoch's lane
stream -- a device write that lands at some later time, in any order with
the other lanes' work.

`run` interleaves every step under a seeded scheduler and returns the
numbering each epoch finally got (the accepted device one or the host's)
next to the serial chain's.  `check_seq=False` models chaining without the
sequence check (every finish numbers from whatever FinCtl holds)."""
from __future__ import annotations

import random


def serial(epochs):
    """(tn base, append position) of every epoch in the serial chain."""
    out, tnc, hm = [], 0, 0
    for e in epochs:
        out.append((tnc, hm) if e["fin"] else None)
        tnc += e["c"]
        hm += e["w"] if e["fin"] else 0
    return out


def run(epochs, seed, check_seq=True):
    """epochs: dicts {c: commits, w: pairs, fin: chained finish, final:
    decided inside its graph}.  Returns (numbering, serial numbering)."""
    rng = random.Random(seed)
    K = len(epochs)
    ctl = {"tnc": 0, "hm": 0, "seq": 1}  # reset at the first submit (nothing in flight)
    host = {"tnc": 0, "hm": 0}
    decided = [False] * K
    snap = [None] * K
    fin_done = [False] * K
    status = [None] * K
    numbering = [None] * K
    completed = 0
    pending_sets = []  # chain_set writes not yet landed: (tnc, hm, seq)

    def ev_done(s):  # the last submitted work of epoch s has run
        return fin_done[s] if epochs[s]["fin"] else decided[s]

    while completed < K:
        acts = []
        for s in range(K):
            if not decided[s]:
                acts.append(("decide", s))
            elif epochs[s]["fin"] and snap[s] is None and (s == 0 or ev_done(s - 1)):
                acts.append(("prep", s))
            elif epochs[s]["fin"] and snap[s] is not None and not fin_done[s]:
                acts.append(("fin", s))
        for q in range(len(pending_sets)):
            acts.append(("set", q))
        s = completed
        if decided[s] and (not epochs[s]["fin"] or fin_done[s]):
            acts.append(("complete", s))
        kind, x = rng.choice(acts)
        if kind == "decide":
            decided[x] = True
        elif kind == "prep":
            snap[x] = dict(ctl)
        elif kind == "fin":
            e, sn = epochs[x], snap[x]
            fin_done[x] = True
            if check_seq and sn["seq"] != x + 1:
                status[x] = 0
            elif e["final"]:
                status[x] = 1
                numbering[x] = (sn["tnc"], sn["hm"])
                ctl.update(tnc=sn["tnc"] + e["c"], hm=sn["hm"] + e["w"], seq=x + 2)
            else:
                status[x] = 2
        elif kind == "set":
            t, h, q = pending_sets.pop(x)
            ctl.update(tnc=t, hm=h, seq=q)
        else:  # complete epoch x, in submit order
            e = epochs[x]
            if e["fin"] and status[x] == 1:
                assert (host["tnc"], host["hm"]) == numbering[x] or not check_seq
                host["tnc"] += e["c"]
                host["hm"] += e["w"]
            else:
                if e["fin"]:
                    numbering[x] = (host["tnc"], host["hm"])
                    host["hm"] += e["w"]
                host["tnc"] += e["c"]
                if any(epochs[y]["fin"] for y in range(x + 1, K)):
                    pending_sets.append((host["tnc"], host["hm"], x + 2))
            completed += 1
    return numbering, serial(epochs)


def random_epochs(rng, k):
    return [{"c": rng.randrange(0, 50), "w": rng.randrange(0, 200), "fin": rng.random() < 0.8,
             "final": rng.random() < 0.7} for _ in range(k)]
