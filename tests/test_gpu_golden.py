"""GPU: the engine against the committed golden vectors (not a live oracle run).

Every tests/golden/*.dccb fixture is replayed through the C ABI from host and
from device pointers; RC, commit tn, tnc, grant groups, readiness and waves
must equal the stored literal-replay decisions bit for bit
(occ.cpp:116-294, row_lock.cpp:52-381).
"""
import numpy as np
import pytest

import deneva_amd as d
from golden_cases import CALVIN_FIXTURES, OCC_FIXTURES, history_epochs, load

pytestmark = pytest.mark.gpu


def _dev(b, device):
    return b.to_torch(device) if device else b


@pytest.mark.parametrize("name", OCC_FIXTURES)
@pytest.mark.parametrize("device", [False, True])
def test_occ_golden(engine, name, device):
    b, info, dec = load(name)
    engine.history_clear()
    engine.tnc = info["tnc_before"]
    rc, tn, st = engine.occ_validate_epoch(_dev(b, "cuda" if device else None), want_tn=True)
    rc = rc.cpu().numpy() if device else rc
    tn = tn.cpu().numpy().view(np.uint64) if device else tn
    assert np.array_equal(rc, dec["rc"])
    assert np.array_equal(tn, dec["commit_tn"])
    assert st["n_commit"] == int(np.count_nonzero(dec["rc"] == 0))
    assert engine.tnc == info["tnc_before"] + int(np.count_nonzero(dec["commit_tn"]))


def test_history_golden(engine):
    """Two epochs: the first appends its committed writes (central_finish,
    occ.cpp:277-286); the second's (start_tn, finish_tn] windows see them."""
    engine.history_clear()
    for e, (b, info, dec, _, _) in enumerate(history_epochs()):
        engine.tnc = info["tnc_before"]
        rc, tn, _ = engine.occ_validate_epoch(b, want_tn=True, append_history=True)
        assert np.array_equal(rc, dec["rc"]), f"epoch {e}"
        assert np.array_equal(tn, dec["commit_tn"]), f"epoch {e}"
    engine.history_clear()


@pytest.mark.parametrize("name", CALVIN_FIXTURES)
@pytest.mark.parametrize("device", [False, True])
def test_calvin_golden(engine, name, device):
    b, _, dec = load(name)
    g, rc, w, st = engine.calvin_order_epoch(_dev(b, "cuda" if device else None),
                                             want_group=True, want_wave=True)
    if device:
        g, rc, w = (x.cpu().numpy() for x in (g, rc, w))
    assert np.array_equal(g.astype(np.uint32), dec["group"])
    assert np.array_equal(rc, dec["rc"])
    assert np.array_equal(w.astype(np.uint32), dec["wave"])
    assert st["n_commit"] == int(np.count_nonzero(dec["rc"] == 0))
