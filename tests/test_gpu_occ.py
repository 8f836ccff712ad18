"""GPU parity of the OCC epoch validator against the oracle (bit-exact RC / tn)."""
import numpy as np
import pytest

import _oracle as orc
import deneva_amd as d

pytestmark = pytest.mark.gpu


def check(engine, b, **kw):
    engine.tnc = 0
    rc, tn, st = engine.occ_validate_epoch(b, want_tn=True)
    erc, etn, _ = orc.occ(b, tnc=0, **kw)
    assert np.array_equal(np.asarray(rc), erc), f"rc mismatch at {np.nonzero(np.asarray(rc) != erc)[0][:10]}"
    return rc, tn, etn, st


@pytest.mark.parametrize("theta", [0.6, 0.9, 0.99])
@pytest.mark.parametrize("n", [1000, 65536])
def test_ycsb_parity(engine, theta, n):
    b = d.gen_ycsb(n_txn=n, zipf_theta=theta)
    engine.tnc = 0
    rc, tn, etn, st = check(engine, b)
    assert np.array_equal(np.asarray(tn), etn)
    assert st["n_commit"] + st["n_abort"] == n
    assert st["rounds"] >= 1


def test_ycsb_1m_parity(engine):
    b = d.gen_ycsb(n_txn=1 << 20, zipf_theta=0.9)
    engine.tnc = 0
    rc, tn, etn, st = check(engine, b)
    assert np.array_equal(np.asarray(tn), etn)
