"""f4: binary interaction / feature files and the epoch order (ttamm/data.py, ttamm.h
ttamm_epoch_batch), CPU side: file round trips and header checks, the oracle's epoch order is a
permutation with DataLoader batch semantics, and the loader refuses host tensors (no CPU
fallback)."""

from __future__ import annotations

import numpy as np
import pytest
import torch

import ttamm
from oracle import data_perm


def test_interactions_round_trip(tmp_path):
    g = torch.Generator().manual_seed(1)
    u = torch.randint(0, 50, (1001,), generator=g)
    v = torch.randint(0, 700, (1001,), generator=g)
    meta = ttamm.save_interactions(tmp_path / "i.bin", u, v, num_users=50, num_items=700)
    assert (meta.n, meta.num_users, meta.num_items) == (1001, 50, 700)
    lu, lv, m2 = ttamm.load_interactions(tmp_path / "i.bin", device="cpu")
    assert m2 == meta and torch.equal(lu, u) and torch.equal(lv, v)
    assert lu.dtype == torch.long


def test_interaction_file_checks(tmp_path):
    u = torch.tensor([0, 1, 2])
    with pytest.raises(ValueError):
        ttamm.save_interactions(tmp_path / "x.bin", u, torch.tensor([0, 1]))
    with pytest.raises(ValueError):
        ttamm.save_interactions(tmp_path / "x.bin", u, torch.tensor([0, 1, -1]))
    with pytest.raises(ValueError):
        ttamm.save_interactions(tmp_path / "x.bin", u, torch.tensor([0, 1, 5]), num_items=5)
    ttamm.save_interactions(tmp_path / "ok.bin", u, torch.tensor([0, 1, 2]))
    raw = (tmp_path / "ok.bin").read_bytes()
    (tmp_path / "cut.bin").write_bytes(raw[:-8])
    with pytest.raises(ValueError):
        ttamm.load_interactions(tmp_path / "cut.bin", device="cpu")
    (tmp_path / "bad.bin").write_bytes(b"NOTTTAMM" + raw[8:])
    with pytest.raises(ValueError):
        ttamm.load_interactions(tmp_path / "bad.bin", device="cpu")
    with pytest.raises(ValueError):  # a feature file is not an interaction file
        ttamm.save_features(tmp_path / "f.bin", torch.zeros(2, 3))
        ttamm.load_interactions(tmp_path / "f.bin", device="cpu")


def test_features_round_trip_padded(tmp_path):
    x = torch.randn(37, 605, generator=torch.Generator().manual_seed(2))
    ttamm.save_features(tmp_path / "f.bin", x)
    y = ttamm.load_features(tmp_path / "f.bin", device="cpu")
    assert y.shape == (37, 605) and y.stride(0) == 608 and torch.equal(y, x)
    full = y.as_strided((37, 608), (608, 1))
    assert torch.count_nonzero(full[:, 605:]) == 0


@pytest.mark.parametrize("n", [0, 1, 2, 3, 4, 5, 17, 1000, (1 << 16) + 3])
def test_epoch_order_is_a_permutation(n):
    for epoch in (0, 1, 7):
        order = data_perm.epoch_order(n, seed=1234, epoch=epoch)
        assert order.dtype == np.int64 and sorted(order.tolist()) == list(range(n))
    assert np.array_equal(data_perm.epoch_order(n, 5, 0, shuffle=False), np.arange(n))


def test_epoch_order_depends_on_seed_and_epoch():
    a = data_perm.epoch_order(10000, 1, 0)
    assert np.array_equal(a, data_perm.epoch_order(10000, 1, 0))
    assert not np.array_equal(a, data_perm.epoch_order(10000, 1, 1))
    assert not np.array_equal(a, data_perm.epoch_order(10000, 2, 0))
    # a shuffle, not a near-identity: few fixed points, positions spread
    assert (a == np.arange(10000)).sum() < 20


def test_epoch_batches_follow_dataloader_semantics():
    u = np.arange(1003, dtype=np.int64)
    v = u * 10
    bs = data_perm.epoch_batches(u, v, 100, seed=3, epoch=0)
    assert [len(b[0]) for b in bs] == [100] * 10 + [3]  # drop_last=False: the short last batch
    seen = np.concatenate([b[0] for b in bs])
    assert sorted(seen.tolist()) == u.tolist()
    assert all(np.array_equal(b[1], b[0] * 10) for b in bs)


def test_loader_rejects_host_tensors():
    u = torch.arange(10)
    with pytest.raises(RuntimeError):
        ttamm.DeviceInteractionLoader(u, u, 4)
    with pytest.raises(ValueError):
        ttamm.DeviceInteractionLoader(u.int(), u.int(), 4)
