"""GPU: the engine against the hand-derived known-answer case of every
decision branch (tests/golden/kat_branches.json), through the C ABI: OCC
(every solver), Calvin grant groups / readiness / waves, MaaT decisions,
commit timestamps and row timestamps."""
import numpy as np
import pytest

from deneva_amd._abi import OPT_SOLVER
from kat_branches import cases, hist, rows

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("solver", [0, 1, 3])
@pytest.mark.parametrize("name,b,c", cases("occ"), ids=[n for n, _, _ in cases("occ")])
def test_occ_branch(engine, name, b, c, solver):
    hk, ht = hist(c)
    engine.set_option(OPT_SOLVER, solver)
    engine.history_clear()
    try:
        if hk is not None:
            engine.history_append(hk, ht)
        engine.tnc = c.get("tnc", 0)
        rc, tn, _ = engine.occ_validate_epoch(b, want_tn=True)
    finally:
        engine.history_clear()
        engine.set_option(OPT_SOLVER, 0)
    assert list(np.asarray(rc)) == c["rc"], c["why"]
    assert list(np.asarray(tn)) == c["tn"], c["why"]


@pytest.mark.parametrize("name,b,c", cases("calvin"), ids=[n for n, _, _ in cases("calvin")])
def test_calvin_branch(engine, name, b, c):
    g, rc, w, _ = engine.calvin_order_epoch(b, want_group=True, want_wave=True)
    assert list(np.asarray(g)) == c["group"], c["why"]
    assert list(np.asarray(rc)) == c["rc"], c["why"]
    assert list(np.asarray(w)) == c["wave"], c["why"]


@pytest.mark.parametrize("name,b,c", cases("maat"), ids=[n for n, _, _ in cases("maat")])
def test_maat_branch(engine, name, b, c):
    rk, lr, lw = rows(c)
    engine.maat_rows_clear()
    if rk is not None:
        engine.maat_rows_set(rk, lr, lw)
    rc, cts, _ = engine.maat_validate_epoch(b, read_and_prewrite=c.get("read_and_prewrite", False))
    assert list(np.asarray(rc)) == c["rc"], c["why"]
    assert list(np.asarray(cts)) == c["cts"], c["why"]
    k, r, w = c["rows_after"]
    glr, glw = engine.maat_rows_get(np.asarray(k, np.uint64))
    assert list(glr) == r and list(glw) == w, c["why"]
    engine.maat_rows_clear()
