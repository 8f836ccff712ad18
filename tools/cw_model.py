#!/usr/bin/env python3
"""CPU model of the one-CU Calvin wave walk (deneva_amd/csrc/calvin_wave.hip).

Replays the kernel's protocol step for step -- slot codes, the 16-bit LDS
fields, the two LDS regions, the staged per-txn bounds, the global maxima and
the flush / refill / next-chunk hand-offs -- with small chunks so that every
hand-off is exercised, and checks the waves against the oracle.  A design
check for the protocol (no GPU); the GPU tests check the kernel itself.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

NONE = 0xFFFFFFFF
F_NONE, F_FLAG = 0xFFFF, 0x8000


def model(b, C=128, sub=64, helpers=False, broken=None):
    """helpers: the helper-workgroup protocol (k_cw_walk<LR, true>): groups
    two chunks away through LDS, three or more through the global maxima on
    the helpers, a chunk ahead.  Each helper iteration reads its inputs at the
    earliest point the kernel allows (right after the staging waves raise P)
    and its writes land at the latest (right before the staging iteration that
    waits for them), so a read of a value not yet final, or a write landing
    after its reader, shows as a mismatch against the oracle.  broken (a check
    of the check): "no_wait" stages chunk c+1 without waiting for helper
    iteration c-1's writes; "three_is_two" lets the helpers take groups that
    ended two chunks back (not yet published when they read)."""
    import _oracle as orc
    g, rc, wv = orc.calvin(b)
    n = b.n_txn
    off = np.asarray(b.offsets, np.int64)
    keys = np.asarray(b.keys, np.uint64)
    maxlen = int(np.diff(off).max())
    lg = max(0, (maxlen - 1).bit_length())
    L = 1 << lg
    H = C * L
    nch = (n + C - 1) // C
    seq = np.argsort(np.asarray(b.order), kind="stable") if b.order is not None else np.arange(n)
    seqpos = np.empty(n, np.int64)
    seqpos[seq] = np.arange(n)
    # per row: requests in sequence order -> groups -> last member code
    recs = {}
    for t in range(n):
        for x in range(off[t], off[t + 1]):
            if g[x] == NONE:
                continue
            recs.setdefault(int(keys[x]), []).append((seqpos[t], x - off[t], int(g[x]), t, x))
    prevc = np.full(nch * H, NONE, np.int64)
    ownc = np.full(nch * H, NONE, np.int64)
    for k, lst in recs.items():
        lst.sort()
        last = {}
        for (q, j, gg, t, x) in lst:
            last[gg] = (q << lg) | j  # the sequence-last member (sorted in order)
        for (q, j, gg, t, x) in lst:
            s = (q << lg) | j
            if gg > 0:
                prevc[s] = last[gg - 1]
            if gg + 1 in last:
                ownc[s] = last[gg]
    # 16-bit fields (k_cw_link)
    rec16 = np.zeros(nch * H, np.int64)
    for s in range(nch * H):
        q = s >> lg
        c = q // C
        fp = fo = F_NONE
        if prevc[s] != NONE:
            pc, loc = divmod(int(prevc[s]), H)
            if pc + 1 >= c:
                intra = pc == c and ((loc >> lg) // sub) == ((q - c * C) // sub)
                fp = ((pc & 1) * H + loc) | (F_FLAG if intra else 0)
        if ownc[s] != NONE:
            oc, loc = divmod(int(ownc[s]), H)
            if oc == c:
                fo = (c & 1) * H + loc
            elif oc == c + 1:
                fo = (((c + 1) & 1) * H + loc) | F_FLAG
        rec16[s] = fp | (fo << 16)
    # marks: slots read by a request of their own sub-chunk
    mark = np.zeros(nch * H + 1, bool)
    for s_ in range(nch * H):
        fp = rec16[s_] & F_NONE
        if fp < 0xFFFE and fp & F_FLAG:
            mark[prevc[s_]] = True
    mark[-1] = False
    # the walk
    sgm = np.zeros(2 * H + 1, np.int64)  # last entry: the zero slot
    ZERO = 2 * H
    mg = np.zeros(nch * H, np.int64)
    sE = np.zeros((2, C), np.int64)
    swt = np.zeros((2, C), np.int64)
    wave = np.zeros(n, np.int64)
    rounds = 0
    ini = None
    sEg = np.zeros((nch + 1, C), np.int64)  # helpers: bounds per chunk (+1 applied)
    wsq = np.zeros((nch + 1, C), np.int64)  # helpers: published waves per chunk
    pending = []  # helper writes not landed yet: ("mg", slot, v) / ("sE", chunk, ql, v)
    for c in range(nch + 1):
        if helpers:
            # ---- (A) chunk c-1 published: its region (final) and its waves
            if c >= 1:
                cp = c - 1
                for l in range(H):
                    mg[cp * H + l] = sgm[(cp & 1) * H + l]
                wsq[cp] = swt[cp & 1]
            # ---- (B) chunk c+1 staged, after helper iteration c-1's writes
            late = pending if broken == "no_wait" else []
            for w_ in ([] if broken == "no_wait" else pending):
                if w_[0] == "mg":
                    mg[w_[1]] = max(mg[w_[1]], w_[2])
                else:
                    sEg[w_[1]][w_[2]] = max(sEg[w_[1]][w_[2]], w_[3])
            pending = []
            if c + 1 < nch:
                c1 = c + 1
                ini = [mg[c1 * H + l] for l in range(H)]
                for ql in range(C):
                    e = sEg[c1][ql] if c1 >= 2 else 0
                    for j in range(L):
                        pc = prevc[c1 * H + (ql << lg) + j]
                        if pc != NONE and pc // H == c - 1 and broken != "three_is_two":  # two back: LDS
                            e = max(e, sgm[((c - 1) & 1) * H + pc - (pc // H) * H] + 1)
                    sE[c1 & 1][ql] = e
            else:
                ini = [0] * H
            for w_ in late:  # (broken: the writes land after their reader)
                if w_[0] == "mg":
                    mg[w_[1]] = max(mg[w_[1]], w_[2])
                else:
                    sEg[w_[1]][w_[2]] = max(sEg[w_[1]][w_[2]], w_[3])
            own = [ownc[c * H + l] if c < nch else NONE for l in range(H)]
            ownq = [ownc[(c - 1) * H + l] if 1 <= c <= nch else NONE for l in range(H)]
            # ---- helper iteration c reads now (P = c), its writes land later
            if c + 2 < nch:
                if c >= 1:
                    cp = c - 1
                    for l in range(H):
                        oc = ownc[cp * H + l]
                        if oc != NONE and oc // H >= c + 2:  # three or more ahead
                            pending.append(("mg", int(oc), int(wsq[cp][l >> lg])))
                c2 = c + 2
                for ql in range(C):
                    e = 0
                    for j in range(L):
                        pc = prevc[c2 * H + (ql << lg) + j]
                        lim = c if broken == "three_is_two" else c - 1
                        if pc != NONE and pc // H <= lim:  # three or more back
                            e = max(e, mg[pc] + 1)
                    pending.append(("sE", c2, ql, int(e)))
            if c >= 1:
                cp = c - 1
                for ql in range(min(C, n - cp * C)):
                    wave[seq[cp * C + ql]] = swt[cp & 1][ql]
        # ---- helpers (disjoint from the walker's data)
        if helpers:
            pass
        elif c >= 1:
            cp = c - 1
            for l in range(H):
                oc = ownc[cp * H + l]
                if oc != NONE and oc // H >= c + 1:
                    mg[oc] = max(mg[oc], swt[cp & 1][l >> lg])
        if c + 1 < nch and not helpers:
            c1 = c + 1
            for ql in range(min(C, n - c1 * C)):
                e = 0
                for j in range(L):
                    pc = prevc[c1 * H + (ql << lg) + j]
                    if pc == NONE:
                        continue
                    ch = pc // H
                    if ch + 2 > c1:
                        continue
                    v = sgm[((c - 1) & 1) * H + pc - ch * H] if ch + 1 == c else mg[pc]
                    e = max(e, v + 1)
                sE[c1 & 1][ql] = e
        if not helpers:
            ini = [mg[(c + 1) * H + l] if c + 1 < nch else 0 for l in range(H)]
            own = [(rec16[c * H + l] >> 16) if c < nch else F_NONE for l in range(H)]
        if c >= 1 and not helpers:
            cp = c - 1
            for ql in range(min(C, n - cp * C)):
                wave[seq[cp * C + ql]] = swt[cp & 1][ql]
        # ---- walker
        if c < nch:
            nq = min(C, n - c * C)
            r = c & 1
            for s0 in range(0, nq, sub):
                lanes = range(s0, min(nq, s0 + sub))
                cur = {ql: [rec16[((c * C + ql) << lg) + j] for j in range(L)] for ql in lanes}
                slot = lambda ql, j: ((c * C + ql) << lg) + j
                # round 1: every previous group; base = all but the intra ones
                base, ival, w = {}, {}, {}
                intra = {}
                for ql in lanes:
                    b_, i_ = sE[r][ql], 0
                    intra[ql] = []
                    for f in cur[ql]:
                        fp = f & F_NONE
                        if fp >= 0xFFFE:
                            continue
                        val = sgm[fp & 0x7FFF] + 1
                        if fp & F_FLAG:
                            i_ = max(i_, val)
                            intra[ql].append(fp & 0x7FFF)
                        else:
                            b_ = max(b_, val)
                    base[ql], w[ql] = b_, max(b_, i_)
                rounds += 1
                if any(intra[ql] for ql in lanes):
                    # hot own slots: publish to a slot an intra request reads
                    hot = {ql: [(f >> 16) for j, f in enumerate(cur[ql])
                                if (f >> 16) < F_FLAG and mark[ownc[slot(ql, j)]]] for ql in lanes}
                    while True:
                        for ql in lanes:
                            for o in hot[ql]:
                                sgm[o] = max(sgm[o], w[ql])
                        changed = False
                        for ql in lanes:
                            nw = max([base[ql]] + [sgm[i] + 1 for i in intra[ql]])
                            if nw != w[ql] and hot[ql]:
                                changed = True
                            w[ql] = nw
                        rounds += 1
                        if not changed:
                            break
                for ql in lanes:
                    for f in cur[ql]:
                        fo = f >> 16
                        if fo < F_FLAG:
                            sgm[fo] = max(sgm[fo], w[ql])
                    swt[r][ql] = w[ql]
        # ---- boundary
        rn = (c + 1) & 1
        if helpers:
            # refill (no flush: chunk c-1 was published in (A)), then chunk c's
            # members of groups ending in chunk c+1 and chunk c-1's of groups
            # ending in chunk c+1 (exactly two ahead; its waves still in swt)
            if c + 1 < nch:
                for l in range(H):
                    sgm[rn * H + l] = ini[l]
            if c < nch:
                for l in range(H):
                    o = own[l]
                    if o != NONE and o // H == c + 1:
                        sgm[rn * H + o - (c + 1) * H] = max(sgm[rn * H + o - (c + 1) * H],
                                                             swt[c & 1][l >> lg])
                    o = ownq[l]
                    if o != NONE and o // H == c + 1:
                        sgm[rn * H + o - (c + 1) * H] = max(sgm[rn * H + o - (c + 1) * H],
                                                             swt[(c - 1) & 1][l >> lg])
            continue
        for l in range(H):
            if c >= 1:
                mg[(c - 1) * H + l] = sgm[rn * H + l]
            if c + 1 < nch:
                sgm[rn * H + l] = ini[l]
        if c < nch:
            for l in range(H):
                f = own[l]
                if f != F_NONE and (f & F_FLAG):
                    sgm[f & 0x7FFF] = max(sgm[f & 0x7FFF], swt[c & 1][l >> lg])
    ok = np.array_equal(wave.astype(np.uint32), wv)
    print(f"n={n} L={L} C={C} chunks={nch} helpers={helpers} max_wave={int(wv.max())} "
          f"rounds={rounds} matches_oracle={ok}")
    if not ok:
        bad = np.nonzero(wave.astype(np.uint32) != wv)[0]
        print("first mismatches", [(int(t), int(wave[t]), int(wv[t])) for t in bad[:8]])
    return ok


if __name__ == "__main__":
    from helpers import c4_batch, random_batch
    rng = np.random.default_rng(5)
    ok = True
    for hp in (False, True):
        for nt, C, sub in ((2048, 128, 64), (3000, 64, 16), (1024, 64, 64)):
            ok &= model(c4_batch(nt), C, sub, helpers=hp)
        for seed in range(3):
            b = random_batch(np.random.default_rng(seed), 900, 12, 40, p_write=0.4)
            ok &= model(b, 64, 16, helpers=hp)
    sys.exit(0 if ok else 1)
