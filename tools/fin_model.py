"""CPU model of central_finish's single-pass look-back and of the host's
look-back buffer policy (TEST INFRASTRUCTURE ONLY).

Device side (deneva_amd/csrc/occ_history.hip, k_fin): workgroup b counts its
committed writers (its aggregate) and publishes it under the launch's tag
(status = tag << 2 | 1); it then looks back over its predecessors 64 at a
time -- each lane spins until predecessor j's status carries the tag, the
wave sums the aggregates down to the nearest inclusive value -- and publishes
its inclusive prefix (status = tag << 2 | 2).  Workgroup 0 publishes its
inclusive value directly.  The last workgroup's inclusive value is the
epoch's total; each workgroup numbers its commits from its exclusive prefix
(occ.cpp:283-284: tn = ++tnc in index order).

Host side (occ_driver.hip, occ_begin): the words are never reset between
launches (the tag tells launches apart); they are zeroed only when the buffer
is (re)allocated.  `policy`:
  * "pointer" -- round 5: zeroed only when the allocation's address changed;
  * "realloc" -- the fix: zeroed on every reallocation.

The allocator model hands a growing buffer back at its old address with the
grown tail holding what the space's previous owner left there: here the
look-back words of another context on the same GPU (the shards of a
multi-GPU context share one device), which run the same tag sequence.

`run_launch` interleaves the workgroups' steps under a seeded scheduler: any
interleaving the hardware could produce (a workgroup's publish may come after
a later workgroup's look-back reads; a workgroup only waits where k_fin
spins)."""
from __future__ import annotations

import random

LANES = 64


def grow(words, blocks, policy, stale_tail):
    """DevBuf::ensure growing `words` in place to `blocks` entries (the tail
    from `stale_tail`), then the policy.  Returns (words, cleared)."""
    old_cap = len(words)
    tail = [list(w) for w in stale_tail[: blocks - old_cap]]
    tail += [[0, 0, 0] for _ in range(blocks - old_cap - len(tail))]
    words = words + tail
    same_address = True
    cleared = (not same_address) if policy == "pointer" else len(words) != old_cap
    if cleared:
        words = [[0, 0, 0] for _ in words]
    return words, cleared


def run_launch(lb, counts, tag, seed):
    """One k_fin launch over len(counts) workgroups on look-back words lb
    (per workgroup [status, agg, inc]).  Returns (total, exclusive prefixes)."""
    nb = len(counts)
    rng = random.Random(seed)

    def wg(b):
        yield  # dispatched; nothing published yet
        own = counts[b]
        if b == 0:
            lb[0][2] = own
            lb[0][0] = (tag << 2) | 2
            return 0
        lb[b][1] = own
        lb[b][0] = (tag << 2) | 1
        yield
        P, hi = 0, b - 1
        while hi >= 0:
            window = [j for j in range(hi, hi - LANES, -1) if j >= 0]
            while any((lb[j][0] >> 2) != tag for j in window):  # the lanes spin
                yield
            inc = [(lb[j][0] & 3) == 2 for j in window]
            stop = inc.index(True) if any(inc) else len(window) - 1
            P += sum(lb[window[q]][2] if inc[q] else lb[window[q]][1] for q in range(stop + 1))
            if any(inc):
                break
            hi -= LANES
        lb[b][2] = P + own
        lb[b][0] = (tag << 2) | 2
        return P

    gens = {b: wg(b) for b in range(nb)}
    prefix = [None] * nb
    live = list(range(nb))
    while live:
        b = rng.choice(live)
        try:
            next(gens[b])
        except StopIteration as e:
            prefix[b] = e.value
            live.remove(b)
    return lb[nb - 1][2], prefix


def scenario(policy, seed, small=6, big=40):
    """Context B ran a launch (tag 1) on `small` workgroups; context A, on the
    same GPU, ran its launches one tag ahead (a second central_finish of an
    epoch takes a fresh tag) and freed its buffer; B's buffer grows in place
    over it for its next launch (tag 2, `big` workgroups).  Returns
    (B's total, the true total, B's prefixes all right)."""
    rng = random.Random(seed)
    B = [[0, 0, 0] for _ in range(small)]
    run_launch(B, [rng.randrange(0, 5) for _ in range(small)], 1, seed)
    A = [[0, 0, 0] for _ in range(big)]
    run_launch(A, [rng.randrange(0, 3) for _ in range(big)], 2, seed + 1)
    B, _ = grow(B, big, policy, A[small:])
    counts = [rng.randrange(0, 5) for _ in range(big)]
    tot, pre = run_launch(B, counts, 2, seed + 2)
    return tot, sum(counts), pre == [sum(counts[:b]) for b in range(big)]


def dispatch_model(order, seed, xcds=4, slots=2, grid=12, launches=2):
    """Several k_fin launches sharing one GPU (key shards of one context, or
    rank processes): workgroup b of each launch is dealt to XCD b % xcds,
    each XCD dispatches its share in b order as its `slots` free up, in any
    interleaving between the launches.  A running workgroup has published
    its aggregate; it finishes (publishes inclusive, frees its slot) once its
    look-back sees every predecessor's status down to the nearest inclusive
    one.  `order`: "blockidx" (the scan position is blockIdx, round 5) or
    "ticket" (the position is the order in which workgroups started: the
    fix).  Returns "done" or "deadlock" (no workgroup can start or finish)."""
    rng = random.Random(seed)
    pend = [[[b for b in range(grid) if b % xcds == x] for x in range(xcds)] for _ in range(launches)]
    free = [slots] * xcds
    status = [[0] * grid for _ in range(launches)]  # 0 none, 1 aggregate, 2 inclusive
    running = []  # (launch, position, xcd)
    tickets = [0] * launches
    done = 0
    while done < launches * grid:
        acts = []
        for L in range(launches):
            for x in range(xcds):
                if pend[L][x] and free[x] > 0:
                    acts.append(("start", L, x))
        for k, (L, p, x) in enumerate(running):
            j = p - 1
            ok = True
            while j >= 0:
                if status[L][j] == 0:
                    ok = False
                    break
                if status[L][j] == 2:
                    break
                j -= 1
            if ok:
                acts.append(("finish", k))
        if not acts:
            return "deadlock"
        a = rng.choice(acts)
        if a[0] == "start":
            _, L, x = a
            b = pend[L][x].pop(0)
            free[x] -= 1
            p = b if order == "blockidx" else tickets[L]
            tickets[L] += 1
            status[L][p] = 2 if p == 0 else 1
            if p == 0:  # workgroup 0 publishes its inclusive value and is done
                free[x] += 1
                done += 1
            else:
                running.append((L, p, x))
        else:
            L, p, x = running.pop(a[1])
            status[L][p] = 2
            free[x] += 1
            done += 1
    return "done"
