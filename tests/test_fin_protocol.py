"""central_finish's look-back protocol (k_fin, occ_history.hip) and the
host's look-back buffer policy (occ_driver.hip occ_begin), replayed on the
CPU by tools/fin_model.py under seeded adversarial interleavings.

Round 5 saw one 'central_finish numbered 339 txns, 480 committed writers'
(two shards of a multi-GPU context on one GPU, commit tn wanted).  The model
reproduces that failure class from the round-5 buffer policy -- look-back
words zeroed only when the allocation's address changes, so a buffer grown
in place keeps a tail of another context's words under the same tag
sequence, which the look-back takes as predecessors' inclusive prefixes --
and shows the fixed policy (zero on every reallocation) exact on every
interleaving.  The GPU side is checked by
test_gpu_multi.py::test_multi_occ_growing_epochs_share_one_gpu."""
import os
import random
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

import fin_model  # noqa: E402


def test_lookback_exact_on_clean_words():
    """Every interleaving numbers every workgroup from the sum of its
    predecessors' commits (occ.cpp:283-284), across windows of 64."""
    for seed in range(60):
        rng = random.Random(seed)
        nb = rng.choice([1, 2, 3, 63, 64, 65, 130, 200])
        counts = [rng.randrange(0, 6) for _ in range(nb)]
        lb = [[0, 0, 0] for _ in range(nb)]
        for tag in (1, 2, 3):  # the words are reused launch after launch
            tot, pre = fin_model.run_launch(lb, counts, tag, seed * 3 + tag)
            assert tot == sum(counts)
            assert pre == [sum(counts[:b]) for b in range(nb)]


def test_round5_policy_takes_foreign_prefixes():
    """The round-5 policy: some interleavings read another context's words
    in the grown tail (the failure class of the round-5 mismatch)."""
    bad = 0
    for seed in range(200):
        tot, want, ok = fin_model.scenario("pointer", seed)
        bad += (tot != want) or not ok
    assert bad > 0


def test_fixed_policy_is_exact():
    for seed in range(200):
        tot, want, ok = fin_model.scenario("realloc", seed)
        assert tot == want and ok, seed


def test_blockidx_lookback_can_deadlock_when_launches_share_the_gpu():
    """The cause of the round-5/6 totals mismatches (the round-6 diagnostic:
    a workgroup's look-back timed out with every word published by the end):
    two look-back launches sharing the GPU, each workgroup's scan position
    its blockIdx.  Workgroups are dealt round-robin to the XCDs; a workgroup
    whose predecessor is still waiting for a slot on another XCD -- held by
    the other launch's spinning workgroups -- waits forever (the bounded
    spin then fails the epoch)."""
    outcomes = {fin_model.dispatch_model("blockidx", s) for s in range(300)}
    assert "deadlock" in outcomes


def test_ticket_lookback_never_deadlocks():
    """The fix: a workgroup's scan position is a ticket taken when it starts,
    so all its predecessors have started (and published) -- every schedule
    completes, also with more launches than the slots can hold at once."""
    for s in range(300):
        assert fin_model.dispatch_model("ticket", s) == "done", s
        assert fin_model.dispatch_model("ticket", s, launches=3, grid=20) == "done", s
