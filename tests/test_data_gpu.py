"""f4 on the GPU: ttamm_epoch_batch against the oracle's epoch order (oracle/data_perm.py,
bit-exact), the loader's DataLoader semantics, and one C1 epoch trained from binary files
through DeviceInteractionLoader — the same losses, bit for bit, as the same batches handed to
the step from the host."""

from __future__ import annotations

import numpy as np
import pytest
import torch

import ttamm
from oracle import data_perm

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,bs", [(1, 1), (3, 2), (4, 4), (5, 2), (1000, 96), ((1 << 20) + 7, 8192), (21244, 256)])
def test_epoch_batch_matches_oracle(n, bs):
    dev = torch.device("cuda")
    u = torch.arange(n, dtype=torch.long, device=dev) * 3
    v = torch.arange(n, dtype=torch.long, device=dev) * 5 + 1
    for seed, epoch in ((0, 0), (1234, 3), (2**63 + 5, 11)):
        ld = ttamm.DeviceInteractionLoader(u, v, bs, seed=seed)
        ld.set_epoch(epoch)
        bl = list(ld)  # one epoch
        got_u = torch.cat([b[0] for b in bl]).cpu().numpy()
        got_v = torch.cat([b[1] for b in bl]).cpu().numpy()
        order = data_perm.epoch_order(n, seed, epoch)
        assert np.array_equal(got_u, order * 3)
        assert np.array_equal(got_v, order * 5 + 1)
        assert ld.epoch == epoch + 1


def test_loader_batches_and_epochs():
    dev = torch.device("cuda")
    n = 10_007
    u = torch.randint(0, 500, (n,), device=dev)
    v = torch.randint(0, 900, (n,), device=dev)
    ld = ttamm.DeviceInteractionLoader(u, v, 1000)
    e0 = list(ld)
    assert [b[0].numel() for b in e0] == [1000] * 10 + [7]
    e1 = list(ld)
    pairs0 = sorted(zip(torch.cat([b[0] for b in e0]).tolist(), torch.cat([b[1] for b in e0]).tolist()))
    assert pairs0 == sorted(zip(u.tolist(), v.tolist()))
    assert not torch.equal(e0[0][0], e1[0][0])  # a new order every epoch
    keep = ttamm.DeviceInteractionLoader(u, v, 1000, drop_last=True)
    assert len(keep) == 10 and all(b[0].numel() == 1000 for b in keep)
    ident = ttamm.DeviceInteractionLoader(u, v, 1000, shuffle=False)
    assert torch.equal(torch.cat([b[0] for b in ident]), u)


def test_c1_epoch_from_binary_files_matches_host_batches(tmp_path):
    """The C1 fixture saved as binary files, loaded to HBM, one epoch through the device loader
    vs the same batches (the oracle's order) fed from the host: identical per-step losses."""
    from torch import nn

    from c1_helpers import LOSS_WEIGHTS, TOWER_CFG, Streams, build_oracle_model, load_c1

    c1 = load_c1()
    dev = torch.device("cuda")
    ttamm.save_interactions(tmp_path / "train.bin", c1.train[:, 0], c1.train[:, 1], num_users=c1.num_users,
                            num_items=c1.num_items)
    ttamm.save_features(tmp_path / "items.bin", c1.item_features)
    ttamm.save_features(tmp_path / "users.bin", c1.user_features)
    users, items, meta = ttamm.load_interactions(tmp_path / "train.bin", dev)
    itf = ttamm.load_features(tmp_path / "items.bin", dev)
    uf = ttamm.load_features(tmp_path / "users.bin", dev)
    assert meta.n == c1.train.shape[0]

    def run(batches):
        om = build_oracle_model(c1)
        ue = ttamm.build_tower_encoder(TOWER_CFG, num_embeddings=c1.num_users, feature_dim=605, device=dev)
        ie = ttamm.build_tower_encoder(TOWER_CFG, num_embeddings=c1.num_items, feature_dim=605, device=dev)
        mm = ttamm.AdaptiveMimicMechanism(num_users=c1.num_users, num_items=c1.num_items, embedding_dim=96).to(dev)
        model = ttamm.TwoTowerModel(ue, ie, similarity=nn.CosineSimilarity(dim=-1), adaptive_mimic=mm)
        model.load_state_dict({k: v.to(dev) for k, v in om.state_dict().items()})
        dense, sparse = ttamm._collect_parameter_groups(model)
        opts = [torch.optim.AdamW(dense, lr=1e-3, weight_decay=0.01), torch.optim.SparseAdam(sparse, lr=1e-3)]
        steps = []
        ttamm.train_one_epoch(model, batches, optimizers=opts, criterion=nn.BCEWithLogitsLoss(),
                              negatives_per_positive=5, num_items=c1.num_items, user_positive_items=c1.positives,
                              user_features=uf, item_features=itf, device=dev, loss_weights=LOSS_WEIGHTS,
                              item_category_tensor=c1.categories.to(dev), major_category_id=c1.major,
                              batch_hook=Streams(c1, 0), step_losses=steps)
        return torch.stack(steps).cpu()

    loader = ttamm.DeviceInteractionLoader(users, items, 256, seed=99)
    on_device = run(loader)
    host = [(torch.as_tensor(bu), torch.as_tensor(bv)) for bu, bv in
            data_perm.epoch_batches(c1.train[:, 0].numpy(), c1.train[:, 1].numpy(), 256, seed=99, epoch=0)]
    from_host = run(host)
    assert on_device.shape[0] == len(host) == 83
    assert torch.equal(on_device, from_host)
