"""Category-alignment loss (training.py:530-579, applied at :805-820) in the fused step on
MI355X vs the CPU oracle's restatement (oracle/cpu_reference.py category_alignment_loss).

Same parameters, injected negatives and dropout masks; gradients exported through the
lr = 0 / beta1 = 0 optimizer step (exp_avg == grad).  Tolerance: 1e-5 norm-wise relative on
the loss terms and every gradient (tests/helpers.rel_err).  Covered: several categories with
singletons (skipped), a major category spanning more than one 256-row piece, the major
category absent from the batch and a single-category batch (both give 0 and no gradient), a
large weight so the L_cal gradient dominates, and three real Adam steps."""

from __future__ import annotations

import pytest
import torch

import ttamm
from helpers import LOSS_WEIGHTS, Shape, make_problem, named_optimizer_state, rel_err, set_lr
from oracle import cpu_reference as ref

pytestmark = pytest.mark.gpu


def _categories(I: int, C: int, major_share: float, seed: int) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    cats = torch.randint(1, max(2, C), (I,), generator=g) if C > 1 else torch.zeros(I, dtype=torch.long)
    cats[torch.rand(I, generator=g) < major_share] = 0
    return cats


def _run(prob, cats, major, lw, *, lr=0.0, betas=(0.0, 0.999)):
    from gpu_helpers import ttamm_model_from, ttamm_optimizers

    # oracle
    om = ref.build_model(prob.shape.tower_cfg(), num_users=prob.shape.U, num_items=prob.shape.I,
                         user_feature_dim=prob.shape.F, item_feature_dim=prob.shape.F, mimic=prob.shape.mimic)
    om.load_state_dict(prob.model.state_dict())
    oo = ref.build_optimizers(om, lr=lr or 1e-3, betas=betas)
    set_lr(oo, lr)
    ores = []
    for (users, pos, neg, um, im) in prob.batches:
        ores.append(ref.train_step(om, oo, users, pos, neg, user_features=prob.user_features,
                                   item_features=prob.item_features, loss_weights=lw, user_keep_masks=um,
                                   item_keep_masks=im, item_category_tensor=cats, major_category_id=major))
    # ttamm
    tm = ttamm_model_from(prob)
    to = ttamm_optimizers(tm, lr=lr, betas=betas)
    eng = ttamm.FusedTrainStep(tm, to, negatives_per_positive=prob.shape.N, positives=prob.positives,
                               user_features=prob.user_features.cuda(), item_features=prob.item_features.cuda(),
                               loss_weights=lw, max_batch=prob.shape.B, item_category_tensor=cats.cuda(),
                               major_category_id=major)
    tres = []
    for (users, pos, neg, um, im) in prob.batches:
        eng.step(users.cuda(), pos.cuda(), neg.cuda().reshape(-1),
                 keep_masks={"user": [m.cuda() for m in um], "item": [m.cuda() for m in im]})
        tres.append(eng.last_losses())
    eng.finish()
    return (om, oo, ores), (tm, to, tres)


def _check_grads(om, oo, tm, to, tol=1e-5):
    og = {n: st["exp_avg"] for n, st in named_optimizer_state(om, oo).items()}
    tg = {n: st["exp_avg"] for n, st in named_optimizer_state(tm, to).items()}
    assert set(og) == set(tg)
    for n in og:
        err = rel_err(tg[n], og[n])
        assert err <= tol, f"{n}: rel err {err:.3e}"


@pytest.mark.parametrize(
    "shape,C,share,lam",
    [
        (Shape(B=64, N=5), 6, 0.5, 0.01),            # several categories, singletons skipped
        (Shape(B=64, N=5), 3, 0.8, 10.0),            # L_cal gradient dominates; major > 256 rows
        (Shape(U=50, I=300, F=37, H=24, D=12, B=40, N=3, gate_hidden=20, hidden_dims=(24,)), 5, 0.4, 5.0),
        (Shape(B=64, N=5, mimic=False), 4, 0.6, 5.0),
    ],
    ids=["default-weight", "dominant", "odd", "nomimic"],
)
def test_category_alignment_matches_oracle(shape, C, share, lam):
    prob = make_problem(shape, steps=1)
    cats = _categories(shape.I, C, share, seed=3)
    lw = {**LOSS_WEIGHTS, "category_alignment": lam}
    (om, oo, ores), (tm, to, tres) = _run(prob, cats, 0, lw)
    o, t = ores[0], tres[0]
    assert o.category_alignment > 0
    assert abs(t["category_alignment"] - o.category_alignment) <= 1e-5 * o.category_alignment
    assert abs(t["total"] - o.total) <= 1e-5 * abs(o.total)
    _check_grads(om, oo, tm, to)


@pytest.mark.parametrize("case", ["major-absent", "one-category"])
def test_category_alignment_zero_cases(case):
    shape = Shape(B=32, N=5)
    prob = make_problem(shape, steps=1)
    if case == "one-category":  # every item in one category: <= 1 unique category -> 0
        cats = torch.zeros(shape.I, dtype=torch.long)
    else:  # the major id (0) is a valid category that no item carries
        cats = 1 + _categories(shape.I, 3, 0.0, seed=5)
    major = 0
    lw = {**LOSS_WEIGHTS, "category_alignment": 5.0}
    (om, oo, ores), (tm, to, tres) = _run(prob, cats, major, lw)
    assert ores[0].category_alignment == 0.0
    assert tres[0]["category_alignment"] == 0.0
    assert abs(tres[0]["total"] - ores[0].total) <= 1e-5 * abs(ores[0].total)
    _check_grads(om, oo, tm, to)


def test_category_alignment_three_adam_steps():
    shape = Shape(B=64, N=5)
    prob = make_problem(shape, steps=3)
    cats = _categories(shape.I, 5, 0.5, seed=9)
    lw = {**LOSS_WEIGHTS, "category_alignment": 2.0}
    (om, oo, ores), (tm, to, tres) = _run(prob, cats, 0, lw, lr=1e-3, betas=(0.9, 0.999))
    for o, t in zip(ores, tres):
        assert abs(t["total"] - o.total) <= 1e-5 * abs(o.total)
        assert abs(t["category_alignment"] - o.category_alignment) <= 1e-4 * max(o.category_alignment, 1e-12)
    osd, tsd = om.state_dict(), tm.state_dict()
    for n in osd:
        d = (tsd[n].cpu() - osd[n]).abs().max().item()
        assert d <= 5e-5, f"{n}: max abs diff {d:.3e}"
