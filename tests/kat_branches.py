"""Loader of the hand-derived branch KATs (tests/golden/kat_branches.json):
each case as an EpochBatch plus its options and expected outputs."""
from __future__ import annotations

import json
import os

import numpy as np

from helpers import make_batch

PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "kat_branches.json")


def cases(kind):
    """[(name, batch, case dict)] for kind in {"occ", "calvin", "maat"}."""
    data = json.load(open(PATH))
    out = []
    for c in data[kind]:
        b = make_batch([[(int(k), int(a)) for k, a in t] for t in c["txns"]],
                       start_tn=c.get("start_tn"), finish_tn=c.get("finish_tn"))
        out.append((c["name"], b, c))
    return out


def hist(c):
    if "hist_keys" not in c:
        return None, None
    return np.asarray(c["hist_keys"], np.uint64), np.asarray(c["hist_tn"], np.uint64)


def rows(c):
    if not c.get("rows"):
        return None, None, None
    k, lr, lw = c["rows"]
    return (np.asarray(k, np.uint64), np.asarray(lr, np.uint64), np.asarray(lw, np.uint64))
