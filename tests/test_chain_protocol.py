"""The chained central_finish protocol of pipelined epochs (FinCtl's sequence
check in k_fin_prep / k_fin, occ_history.hip; the host's accept / finish /
chain_set at completion, occ_pipe.cpp), replayed on the CPU by
tools/chain_model.py under seeded adversarial interleavings: decisions, the
finishes' snapshots, their FinCtl advances and the host's chain_set writes
landing in any order the lanes' streams allow.  Every epoch's commit-tn base
and append position must be the serial chain's (occ.cpp:277-286: tn =
++tnc in submit order).  The GPU side: test_gpu_pipeline.py's chained
streams."""
import os
import random
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

import chain_model as cm  # noqa: E402


def test_every_interleaving_numbers_serially():
    for seed in range(400):
        rng = random.Random(seed)
        eps = cm.random_epochs(rng, rng.choice([1, 2, 3, 5, 8, 13]))
        got, want = cm.run(eps, seed)
        assert got == want, (seed, eps)


def test_all_final_chains_on_the_device():
    """Every epoch final and chained: after the first, the device numbers
    them in order whatever the interleaving (nothing falls back)."""
    for seed in range(200):
        eps = [{"c": 3 + i, "w": 10 * i, "fin": True, "final": True} for i in range(6)]
        got, want = cm.run(eps, seed)
        assert got == want


def test_not_final_epochs_and_epochs_without_finish():
    """A not-final epoch (more levels after its graph) and epochs without a
    finish between chained ones: the host numbers them and moves FinCtl past
    them; stale chain_set writes that land late only stall the chain."""
    for seed in range(300):
        eps = [{"c": 5, "w": 7, "fin": True, "final": True},
               {"c": 4, "w": 0, "fin": False, "final": True},
               {"c": 6, "w": 9, "fin": True, "final": False},
               {"c": 2, "w": 3, "fin": True, "final": True},
               {"c": 1, "w": 0, "fin": False, "final": True},
               {"c": 8, "w": 11, "fin": True, "final": True}]
        got, want = cm.run(eps, seed)
        assert got == want, seed


def test_without_the_sequence_check_numbering_breaks():
    """Chaining without the check (a finish numbers from whatever FinCtl
    holds) gives wrong numbers on some interleavings -- why k_fin_prep
    snapshots seq and k_fin refuses a stale snapshot."""
    bad = 0
    for seed in range(300):
        rng = random.Random(seed)
        eps = cm.random_epochs(rng, 6)
        got, want = cm.run(eps, seed, check_seq=False)
        bad += got != want
    assert bad > 0
