"""Fused training step on MI355X vs the CPU oracle (same parameters, injected negatives and
dropout keep-masks).  Tolerances: loss and gradients 1e-5 norm-wise relative
(max|ours - oracle| / max|oracle| per tensor, tests/helpers.rel_err)."""

import pytest
import torch

from helpers import Shape, make_problem, named_optimizer_state, rel_err, run_oracle

pytestmark = pytest.mark.gpu

GRAD_TOL = 1e-5


def _grads_by_name(model, opts):
    """With lr = 0 and beta1 = 0 a single Adam/SparseAdam step leaves exp_avg == grad
    exactly (lerp weight 1; (g - 0) * 1), and parameters unchanged."""
    return {n: st["exp_avg"] for n, st in named_optimizer_state(model, opts).items()}


@pytest.mark.parametrize(
    "shape",
    [
        Shape(),
        Shape(dropout=0.0, hidden_dims=(16,)),
        Shape(U=50, I=300, F=37, H=24, D=12, B=40, N=3, gate_hidden=20, hidden_dims=(24,)),
        Shape(U=64, I=512, F=20, D=16, B=64, N=5, hidden_dims=(32, 24)),
        Shape(mimic=False),
        Shape(sparse=False),
    ],
    ids=["tiny", "nodrop", "odd", "2hidden", "nomimic", "dense-id"],
)
def test_step_gradients_match_oracle(shape):
    from gpu_helpers import run_ttamm

    prob = make_problem(shape, steps=1)
    om, oo, ores = run_oracle(prob, lr=0.0, betas=(0.0, 0.999))
    tm, to, tres = run_ttamm(prob, lr=0.0, betas=(0.0, 0.999))
    assert abs(tres[0]["total"] - ores[0].total) <= GRAD_TOL * abs(ores[0].total)
    assert abs(tres[0]["bce"] - ores[0].bce) <= GRAD_TOL * abs(ores[0].bce)
    if shape.mimic:
        assert abs(tres[0]["mimic_user"] - ores[0].mimic_user) <= GRAD_TOL * abs(ores[0].mimic_user)
        assert abs(tres[0]["mimic_item"] - ores[0].mimic_item) <= GRAD_TOL * abs(ores[0].mimic_item)
    og = _grads_by_name(om, oo)
    tg = _grads_by_name(tm, to)
    assert set(og) == set(tg)
    for name in og:
        err = rel_err(tg[name], og[name])
        assert err <= GRAD_TOL, f"{name}: rel err {err:.3e}"
    # lr = 0: parameters untouched
    for (n, p), (_, q) in zip(om.state_dict().items(), tm.state_dict().items()):
        assert torch.equal(q.cpu(), p), n


@pytest.mark.parametrize("shape", [Shape(), Shape(sparse=False)], ids=["tiny", "dense-id"])
def test_three_steps_match_oracle(shape):
    from gpu_helpers import run_ttamm

    prob = make_problem(shape, steps=3)
    om, oo, ores = run_oracle(prob)
    tm, to, tres = run_ttamm(prob)
    for o, t in zip(ores, tres):
        assert abs(t["total"] - o.total) <= 1e-5 * abs(o.total)
    osd, tsd = om.state_dict(), tm.state_dict()
    for n in osd:
        # Adam normalises each update to ~lr: compare the parameter *change* relative to lr.
        d = (tsd[n].cpu() - osd[n]).abs().max().item()
        assert d <= 1e-3 * 1e-3 * 50, f"{n}: max abs diff {d:.3e}"
    ost, tst = named_optimizer_state(om, oo), named_optimizer_state(tm, to)
    for n in ost:
        assert rel_err(tst[n]["exp_avg"], ost[n]["exp_avg"]) <= 1e-4, n
        assert rel_err(tst[n]["exp_avg_sq"], ost[n]["exp_avg_sq"]) <= 1e-4, n
        assert float(tst[n]["step"]) == float(ost[n]["step"]), n
