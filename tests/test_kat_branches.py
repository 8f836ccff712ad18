"""CPU: the oracle against the hand-derived known-answer case of every
decision branch of the reference path (tests/golden/kat_branches.json; the
derivations cite occ.cpp, row_lock.cpp, maat.cpp and row_maat.cpp).  These
pin the oracle to the reference's code, which cannot be built here."""
import numpy as np
import pytest

import _oracle as orc
from kat_branches import cases, hist, rows


@pytest.mark.parametrize("literal", [True, False])
@pytest.mark.parametrize("name,b,c", cases("occ"), ids=[n for n, _, _ in cases("occ")])
def test_occ_branch(name, b, c, literal):
    hk, ht = hist(c)
    rc, tn, _ = orc.occ(b, hist_keys=hk, hist_tn=ht, tnc=c.get("tnc", 0), literal=literal)
    assert list(rc) == c["rc"], c["why"]
    assert list(tn) == c["tn"], c["why"]


@pytest.mark.parametrize("literal", [True, False])
@pytest.mark.parametrize("name,b,c", cases("calvin"), ids=[n for n, _, _ in cases("calvin")])
def test_calvin_branch(name, b, c, literal):
    g, rc, w = orc.calvin(b, literal=literal)
    assert list(g) == c["group"], c["why"]
    assert list(rc) == c["rc"], c["why"]
    assert list(w) == c["wave"], c["why"]


@pytest.mark.parametrize("literal", [True, False])
@pytest.mark.parametrize("name,b,c", cases("maat"), ids=[n for n, _, _ in cases("maat")])
def test_maat_branch(name, b, c, literal):
    rk, lr, lw = rows(c)
    rc, cts, (ek, elr, elw) = orc.maat(b, rk, lr, lw, rw_all=c.get("read_and_prewrite", False),
                                       literal=literal)
    assert list(rc) == c["rc"], c["why"]
    assert list(cts) == c["cts"], c["why"]
    k, r, w = c["rows_after"]
    got = {int(x): (int(y), int(z)) for x, y, z in zip(ek, elr, elw)}
    for x, y, z in zip(k, r, w):
        assert got[x] == (y, z), c["why"]
