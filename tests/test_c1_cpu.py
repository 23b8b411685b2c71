"""The joinable C1 fixture (tests/golden/c1) and its preparation by the CPU restatement of the
reference's data path (oracle/data_prep.py): counts, feature width (F = 605) and checksums must
reproduce tests/golden/c1/c1_expected.json, and the injected RNG streams must be a pure function
of (epoch, step, batch) so the oracle and ttamm runs see the same negatives and masks."""

from __future__ import annotations

import json
from pathlib import Path

import torch

from c1_helpers import N, Streams, load_c1, loader

HERE = Path(__file__).resolve().parent


def test_c1_fixture_preparation_reproduces_expected():
    import make_c1_fixture as fx

    want = json.loads((HERE / "golden" / "c1" / "c1_expected.json").read_text())
    got = fx.summary(fx.prepare())
    assert got == want
    assert got["feature_dim"] == 605  # 300 category + 300 author + 3 numeric + 2 title columns


def test_c1_loader_has_short_last_batch_and_streams_are_deterministic():
    c1 = load_c1()
    sizes = [u.numel() for u, _ in loader(c1, 0)]
    assert sizes[:-1] == [256] * (len(sizes) - 1) and 0 < sizes[-1] < 256
    b1 = next(iter(loader(c1, 1)))
    b1_again = next(iter(loader(c1, 1)))
    assert torch.equal(b1[0], b1_again[0]) and not torch.equal(b1[0], next(iter(loader(c1, 0)))[0])
    s = Streams(c1, 1)
    n1, m1 = s(3, *b1)
    n2, m2 = s(3, *b1)
    assert torch.equal(n1, n2) and torch.equal(m1["item"][0], m2["item"][0])
    assert n1.shape == (256, N)
    for u, row in zip(b1[0].tolist(), n1.tolist()):  # negatives exclude the user's positives
        assert not set(row) & c1.positives[u]


def test_sampled_candidates_follow_the_reference_rng_order():
    """ttamm's host candidate builder (numpy setdiff) draws exactly the candidates of the
    reference's list(set(range(n)) - blocked) + rng.choice loop (training.py:979-987), in the
    same list order — checked on the C1 validation users with one rng stream for both."""
    import numpy as np

    from ttamm.retrieval import sampled_candidates

    c1 = load_c1()
    groups: dict[int, list[int]] = {}
    for u, i in c1.val_pairs:
        groups.setdefault(u, []).append(i)
    users = sorted(groups)[:300]
    truth = {u: set(groups[u]) for u in users}
    got = sampled_candidates(users, truth, c1.train_positive_map, num_items=c1.num_items, candidate_samples=50,
                             rng=np.random.default_rng(1234 * 997 + 1))
    rng = np.random.default_rng(1234 * 997 + 1)
    for u, lst in zip(users, got):
        cands = set(truth[u])
        available = list(set(range(c1.num_items)) - set(c1.train_positive_map.get(u, set())))
        cands.update(int(n) for n in rng.choice(available, size=min(50, len(available)), replace=False).tolist())
        assert lst == list(cands), u


def test_sampled_candidates_dense_blocked_sets_follow_cpython_order():
    """A user blocking n / 4 items or more: CPython's set difference then builds a new, smaller
    table whose iteration order is not ascending (n = 100 with 90 blocked iterates 96..99 before
    90..95), so rng.choice over it picks different items than over the sorted array.  The builder
    must follow the reference's list(set(range(n)) - blocked) order on both sides of the n / 4
    threshold."""
    import numpy as np

    from ttamm.retrieval import sampled_candidates

    n = 100
    gen = np.random.default_rng(7)
    for nblocked in (0, 10, 24, 25, 26, 60, 90, 99):
        blocked = set(gen.choice(n, size=nblocked, replace=False).tolist())
        free = sorted(set(range(n)) - blocked)
        truth = {0: {free[0]}}
        got = sampled_candidates([0], truth, {0: blocked}, num_items=n, candidate_samples=8,
                                 rng=np.random.default_rng(11))[0]
        rng = np.random.default_rng(11)
        cands = set(truth[0])
        available = list(set(range(n)) - blocked)
        budget = max(0, min(8, len(available)))
        if budget:
            cands.update(int(x) for x in rng.choice(available, size=budget, replace=False).tolist())
        assert got == list(cands), nblocked
    # the non-ascending case does occur at this size (the test exercises the new-set path)
    assert list(set(range(n)) - set(range(90))) != sorted(set(range(n)) - set(range(90)))
