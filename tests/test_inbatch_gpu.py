"""In-batch negatives (ttamm.h ttamm_step_args.in_batch; BASELINE configs C2 / C4) against the
oracle's definition (oracle/cpu_reference.py train_step(in_batch=True): S = U P^T over the
batch's positives with label 1 on the diagonal, then the sampled negatives, one BCE mean over
B (B + N) logits).  Same tolerances as the sampled-mode parity tests: loss and every gradient
1e-5 norm-wise relative (tests/helpers.rel_err); three real steps as test_three_steps_match_oracle.

Shapes cover: D not a multiple of 32 (padded MFMA blocks), batches that are not a multiple of the
kernel's 128-row blocks or 64-column tiles, several column splits (B > 64 x 8), N = 0 (pure
in-batch), D = 128 (C4 width) and D = 96 with the C2 MLP."""

from __future__ import annotations

import pytest
import torch

import ttamm
from helpers import LOSS_WEIGHTS, Shape, make_problem, named_optimizer_state, rel_err
from oracle import cpu_reference as ref

pytestmark = pytest.mark.gpu

TOL = 1e-5


def _run_oracle(prob, *, lr=1e-3, betas=(0.9, 0.999)):
    from helpers import clone_model, set_lr

    model = clone_model(prob.model)
    opts = ref.build_optimizers(model, lr=lr or 1e-3, betas=betas, weight_decay=0.01)
    set_lr(opts, lr)
    res = []
    for (users, pos, neg, um, im) in prob.batches:
        res.append(ref.train_step(model, opts, users, pos, neg, user_features=prob.user_features,
                                  item_features=prob.item_features, loss_weights=LOSS_WEIGHTS,
                                  user_keep_masks=um, item_keep_masks=im, in_batch=True))
    return model, opts, res


def _run_ttamm(prob, *, lr=1e-3, betas=(0.9, 0.999)):
    from gpu_helpers import ttamm_model_from, ttamm_optimizers

    model = ttamm_model_from(prob)
    opts = ttamm_optimizers(model, lr=lr, betas=betas)
    eng = ttamm.FusedTrainStep(model, opts, negatives_per_positive=prob.shape.N, positives=prob.positives,
                               user_features=prob.user_features.cuda(), item_features=prob.item_features.cuda(),
                               loss_weights=LOSS_WEIGHTS, max_batch=prob.shape.B, in_batch_negatives=True)
    losses = []
    for (users, pos, neg, um, im) in prob.batches:
        eng.step(users.cuda(), pos.cuda(), neg.cuda().reshape(-1) if prob.shape.N else None,
                 keep_masks={"user": [m.cuda() for m in um], "item": [m.cuda() for m in im]})
        losses.append(eng.last_losses())
    eng.finish()
    return model, opts, losses


SHAPES = [
    Shape(),
    Shape(N=0),
    Shape(U=50, I=300, F=37, H=24, D=12, B=40, N=3, gate_hidden=20, hidden_dims=(24,)),
    Shape(U=400, I=2000, F=605, H=192, D=96, B=300, N=5, hidden_dims=(192,)),
    Shape(U=300, I=1500, F=40, H=64, D=128, B=200, N=0, hidden_dims=(64,)),
    Shape(U=3000, I=5000, F=20, H=32, D=32, B=2100, N=2, hidden_dims=(32,)),
    Shape(mimic=False, N=2),
]
IDS = ["tiny", "n0", "odd-d12", "c2-dims", "d128-n0", "multisplit", "nomimic"]


@pytest.mark.parametrize("shape", SHAPES, ids=IDS)
def test_inbatch_gradients_match_oracle(shape):
    prob = make_problem(shape, steps=1)
    om, oo, ores = _run_oracle(prob, lr=0.0, betas=(0.0, 0.999))
    tm, to, tres = _run_ttamm(prob, lr=0.0, betas=(0.0, 0.999))
    for key in ("total", "bce", "mimic_user", "mimic_item"):
        o = getattr(ores[0], key)
        assert abs(tres[0][key] - o) <= TOL * abs(o), (key, tres[0][key], o)
    og = {n: st["exp_avg"] for n, st in named_optimizer_state(om, oo).items()}
    tg = {n: st["exp_avg"] for n, st in named_optimizer_state(tm, to).items()}
    assert set(og) == set(tg)
    for name in og:
        err = rel_err(tg[name], og[name])
        assert err <= TOL, f"{name}: rel err {err:.3e}"


@pytest.mark.parametrize("shape", [Shape(), Shape(N=0, sparse=False)], ids=["tiny", "n0-dense-id"])
def test_inbatch_three_steps_match_oracle(shape):
    prob = make_problem(shape, steps=3)
    om, oo, ores = _run_oracle(prob)
    tm, to, tres = _run_ttamm(prob)
    for o, t in zip(ores, tres):
        assert abs(t["total"] - o.total) <= 1e-5 * abs(o.total)
    osd, tsd = om.state_dict(), tm.state_dict()
    for n in osd:
        d = (tsd[n].cpu() - osd[n]).abs().max().item()
        assert d <= 1e-3 * 1e-3 * 50, f"{n}: max abs diff {d:.3e}"


def test_inbatch_epoch_through_drop_in_matches_oracle():
    """One C1 epoch (DataLoader, short last batch, L_cal on) in in-batch mode with 2 sampled
    negatives, through ttamm.train_one_epoch vs the oracle loop: per-step loss 1e-5."""
    from torch import nn

    from c1_helpers import LOSS_WEIGHTS as LW
    from c1_helpers import TOWER_CFG, Streams, build_oracle_model, load_c1, loader

    c1 = load_c1()
    om = build_oracle_model(c1)
    dev = torch.device("cuda")
    ue = ttamm.build_tower_encoder(TOWER_CFG, num_embeddings=c1.num_users, feature_dim=605, device=dev)
    ie = ttamm.build_tower_encoder(TOWER_CFG, num_embeddings=c1.num_items, feature_dim=605, device=dev)
    mm = ttamm.AdaptiveMimicMechanism(num_users=c1.num_users, num_items=c1.num_items, embedding_dim=96).to(dev)
    model = ttamm.TwoTowerModel(ue, ie, similarity=nn.CosineSimilarity(dim=-1), adaptive_mimic=mm)
    model.load_state_dict({k: v.to(dev) for k, v in om.state_dict().items()})

    class Two(Streams):  # 2 sampled negatives per positive
        def __call__(self, step, users, pos):
            neg, masks = super().__call__(step, users, pos)
            b = users.shape[0]
            return neg[:, :2].contiguous(), {"user": masks["user"], "item": [masks["item"][0][: b * 3]]}

    o_steps = []
    ref.train_one_epoch(om, loader(c1, 0), ref.build_optimizers(om, lr=1e-3, weight_decay=0.01),
                        negatives_per_positive=2, num_items=c1.num_items, positives=c1.positives,
                        user_features=c1.user_features, item_features=c1.item_features, loss_weights=LW,
                        item_category_tensor=c1.categories, major_category_id=c1.major, batch_hook=Two(c1, 0),
                        step_losses=o_steps, in_batch=True)
    dense, sparse = ttamm._collect_parameter_groups(model)
    opts = [torch.optim.AdamW(dense, lr=1e-3, weight_decay=0.01), torch.optim.SparseAdam(sparse, lr=1e-3)]
    t_steps = []
    ttamm.train_one_epoch(model, loader(c1, 0), optimizers=opts, criterion=nn.BCEWithLogitsLoss(),
                          negatives_per_positive=2, num_items=c1.num_items, user_positive_items=c1.positives,
                          user_features=c1.user_features.to(dev), item_features=c1.item_features.to(dev), device=dev,
                          loss_weights=LW, item_category_tensor=c1.categories.to(dev), major_category_id=c1.major,
                          batch_hook=Two(c1, 0), step_losses=t_steps, in_batch_negatives=True)
    t = [float(v[0]) for v in torch.stack(t_steps).cpu()]
    o = [r.total for r in o_steps]
    assert len(t) == len(o) == 83
    worst = max(abs(a - b) / abs(b) for a, b in zip(t, o))
    print(f"\nC1 in-batch epoch: max per-step rel diff {worst:.2e}, last loss {o[-1]:.5f}")
    assert worst <= 1e-5
