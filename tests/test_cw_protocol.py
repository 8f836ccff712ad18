"""The one-CU Calvin wave walk's protocol (calvin_wave.hip), replayed on the
CPU by tools/cw_model.py with small chunks so that every hand-off (LDS window,
far bounds, next-chunk members, flush / refill, intra rounds; with helper
workgroups: publication, two-chunk LDS cases, helper reads and writes) is exercised,
against the oracle's waves (oracle_calvin_formula, calvin_ref.c:196-257).
The GPU kernel itself is checked by the -m gpu Calvin tests."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

import cw_model  # noqa: E402
from helpers import c4_batch, random_batch  # noqa: E402


def test_c4_shape():
    assert cw_model.model(c4_batch(768), C=64, sub=16)


def test_ragged_random():
    b = random_batch(np.random.default_rng(11), 400, 12, 30, p_write=0.4)
    assert cw_model.model(b, C=64, sub=16)


# The helper-workgroup protocol (k_cw_walk<LR, true>): helper reads at the
# earliest point the kernel allows, their writes at the latest.
def test_helpers_c4_shape():
    assert cw_model.model(c4_batch(768), C=64, sub=16, helpers=True)


def test_helpers_ragged_random():
    b = random_batch(np.random.default_rng(11), 400, 12, 30, p_write=0.4)
    assert cw_model.model(b, C=64, sub=16, helpers=True)


def test_helpers_model_catches_broken_orders():
    # staging without waiting for the helpers, and helpers reading groups
    # that ended two chunks back (not published when they read): both wrong
    for broken in ("no_wait", "three_is_two"):
        assert not cw_model.model(c4_batch(768), C=64, sub=16, helpers=True, broken=broken)
