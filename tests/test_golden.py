"""CPU: the oracle still reproduces every committed golden fixture.

tests/golden/*.dccb freeze the literal-replay decisions (RC, commit tn, grant
group, wave) on seeded batches in the C1-C4 shapes.  Both OCC restatements
(the literal active-list replay of occ.cpp:116-327 and the serial hash scan)
and both Calvin restatements (the literal Row_lock simulation of
row_lock.cpp:52-381 and the per-row formula) must match them exactly, so
the checker the GPU suite trusts cannot drift unnoticed.
"""
import numpy as np
import pytest

import _oracle as orc
from golden_cases import ALL_FIXTURES, CALVIN_FIXTURES, OCC_FIXTURES, history_epochs, load


def test_every_fixture_is_covered():
    import os
    from golden_cases import GOLDEN
    on_disk = sorted(f for f in os.listdir(GOLDEN) if f.endswith(".dccb"))
    assert on_disk == sorted(ALL_FIXTURES)


@pytest.mark.parametrize("name", OCC_FIXTURES)
@pytest.mark.parametrize("literal", [True, False])
def test_occ_fixture(name, literal):
    b, info, dec = load(name)
    assert dec["rc"] is not None and dec["commit_tn"] is not None
    rc, tn, tnc = orc.occ(b, tnc=info["tnc_before"], literal=literal)
    assert np.array_equal(rc, dec["rc"])
    assert np.array_equal(tn, dec["commit_tn"])
    assert tnc == info["tnc_before"] + int(np.count_nonzero(dec["commit_tn"]))
    # the fixtures are not degenerate: both outcomes occur
    assert 0 < int(np.count_nonzero(dec["rc"] == 0)) < b.n_txn


@pytest.mark.parametrize("literal", [True, False])
def test_history_fixtures(literal):
    eps = history_epochs()
    for e, (b, info, dec, hk, ht) in enumerate(eps):
        rc, tn, _ = orc.occ(b, hist_keys=hk, hist_tn=ht, tnc=info["tnc_before"], literal=literal)
        assert np.array_equal(rc, dec["rc"]), f"epoch {e}"
        assert np.array_equal(tn, dec["commit_tn"]), f"epoch {e}"
    # epoch 1's windows really reach the history: dropping it changes decisions
    b, info, dec, _, _ = eps[1]
    rc, _, _ = orc.occ(b, tnc=info["tnc_before"], literal=literal)
    assert not np.array_equal(rc, dec["rc"])


@pytest.mark.parametrize("name", CALVIN_FIXTURES)
@pytest.mark.parametrize("literal", [True, False])
def test_calvin_fixture(name, literal):
    b, _, dec = load(name)
    assert b.order is not None
    g, rc, w = orc.calvin(b, literal=literal)
    assert np.array_equal(g, dec["group"])
    assert np.array_equal(rc, dec["rc"])
    assert np.array_equal(w, dec["wave"])
