"""The reference's other dense-group optimizers through the fused step (training.py:1311-1333,
restated in oracle/cpu_reference.build_optimizers):

  * ``optimizer: adam`` — torch.optim.Adam with coupled L2 weight decay, the reference's default
    when ``training.optimizer`` is unset (training.py:1311, :1316-1318).  Untouched mimic-table
    rows then step with g = weight_decay * p every step; the fused step replays that deferred
    (replay_kernel<false, ...>) or sweeps it eagerly;
  * ``optimizer: sgd`` — torch.optim.SGD(lr, weight_decay, momentum) (training.py:1324-1330;
    sgd.py _single_tensor_sgd): the momentum buffer created by the first step, untouched mimic
    rows moved by weight decay and momentum every step (an eager sweep), or not at all without
    either.

Tolerances (the sampled-mode parity tests'): one step 1e-5 norm-wise on every parameter change
and optimizer buffer; three steps 5e-5 on SGD parameter changes, Adam as test_three_steps_match_oracle
(parameters 5e-5 absolute, moments 1e-4)."""

from __future__ import annotations

import pytest
import torch

from helpers import Shape, make_problem, named_optimizer_state, rel_err, run_oracle

pytestmark = pytest.mark.gpu


def _deltas(model, init):
    return {n: (v.detach().cpu() - init[n]) for n, v in model.state_dict().items()}


SGD_CASES = [
    (Shape(), 0.9, 0.01),
    (Shape(), 0.0, 0.01),
    (Shape(), 0.0, 0.0),
    (Shape(sparse=False), 0.9, 0.01),
    (Shape(fusion="concat", dropout=0.0), 0.5, 0.0),
]
SGD_IDS = ["momentum-wd", "wd-only", "plain", "dense-id-momentum", "concat-momentum"]


@pytest.mark.parametrize("steps", [1, 3])
@pytest.mark.parametrize("shape,momentum,wd", SGD_CASES, ids=SGD_IDS)
def test_sgd_matches_oracle(shape, momentum, wd, steps):
    from gpu_helpers import run_ttamm

    prob = make_problem(shape, steps=steps)
    init = {k: v.clone() for k, v in prob.model.state_dict().items()}
    # lr 0.5: SGD moves parameters by lr * g, large enough that every change is far above fp32 noise
    om, oo, ores = run_oracle(prob, lr=0.5, weight_decay=wd, optimizer="sgd", momentum=momentum)
    tm, to, tres = run_ttamm(prob, lr=0.5, weight_decay=wd, optimizer="sgd", momentum=momentum)
    tol = 1e-5 if steps == 1 else 5e-5
    for o, t in zip(ores, tres):
        assert abs(t["total"] - o.total) <= tol * abs(o.total)
    od, td = _deltas(om, init), _deltas(tm, init)
    sparse_adam = {n for n, st in named_optimizer_state(om, oo).items() if "exp_avg" in st}
    for n in od:
        if n in sparse_adam:
            # the sparse ID tables stay under SparseAdam (training.py:1341-1345) at the same lr: a
            # normalised step, compared as test_three_steps_match_oracle does (5 % of lr)
            d = (td[n] - od[n]).abs().max().item()
            assert d <= 0.05 * 0.5, f"{n}: SparseAdam max abs diff {d:.3e}"
            continue
        if od[n].abs().max() == 0:  # untouched (plain SGD: a row no batch reached)
            assert td[n].abs().max() == 0, n
            continue
        err = rel_err(td[n], od[n])
        assert err <= tol, f"{n}: parameter change rel err {err:.3e}"
    ost, tst = named_optimizer_state(om, oo), named_optimizer_state(tm, to)
    assert set(ost) == set(tst)
    for n in ost:
        assert set(ost[n]) == set(tst[n]), n  # SGD: momentum_buffer iff momentum; SparseAdam: its moments
        for k in ("momentum_buffer", "exp_avg", "exp_avg_sq"):
            if k in ost[n]:
                err = rel_err(tst[n][k], ost[n][k])
                assert err <= (tol if k == "momentum_buffer" else 1e-4), f"{n}: {k} rel err {err:.3e}"


@pytest.mark.parametrize("deferred", [True, False], ids=["deferred", "eager"])
@pytest.mark.parametrize("steps", [1, 3])
def test_adam_coupled_l2_matches_oracle(steps, deferred):
    """Adam with L2 weight decay (the reference default): the deferred replay of the untouched
    rows (g = wd * p each step) and the eager sweep both against the oracle."""
    from gpu_helpers import run_ttamm

    shape = Shape()
    prob = make_problem(shape, steps=steps)
    om, oo, ores = run_oracle(prob, optimizer="adam")
    tm, to, tres = run_ttamm(prob, optimizer="adam", deferred_adamw=deferred)
    for o, t in zip(ores, tres):
        assert abs(t["total"] - o.total) <= 1e-5 * abs(o.total)
    osd, tsd = om.state_dict(), tm.state_dict()
    for n in osd:
        d = (tsd[n].cpu() - osd[n]).abs().max().item()
        assert d <= 5e-5, f"{n}: max abs diff {d:.3e}"  # 5 % of lr, test_three_steps_match_oracle's bound
    ost, tst = named_optimizer_state(om, oo), named_optimizer_state(tm, to)
    for n in ost:
        tol = 1e-5 if steps == 1 else 1e-4
        assert rel_err(tst[n]["exp_avg"], ost[n]["exp_avg"]) <= tol, n
        assert rel_err(tst[n]["exp_avg_sq"], ost[n]["exp_avg_sq"]) <= tol, n
        assert float(tst[n]["step"]) == float(ost[n]["step"]) == steps, n
    # coupled L2 really acted on the untouched mimic rows: their moments are non-zero
    m = tst["adaptive_mimic.item_augmented.weight"]["exp_avg"]
    assert (m.abs().sum(dim=1) > 0).all()


def test_sgd_deferred_creates_momentum_buffers():
    """FusedTrainStep(deferred_adamw=True) with SGD defers the g = 0 table steps too (the replay's
    sgd_elem path), and the first step still creates torch's momentum buffers in place."""
    import ttamm
    from gpu_helpers import ttamm_model_from, ttamm_optimizers
    from helpers import LOSS_WEIGHTS

    prob = make_problem(Shape(), steps=1)
    tm = ttamm_model_from(prob)
    opts = ttamm_optimizers(tm, optimizer="sgd", momentum=0.9)
    eng = ttamm.FusedTrainStep(tm, opts, negatives_per_positive=prob.shape.N, positives=prob.positives,
                               user_features=prob.user_features.cuda(), item_features=prob.item_features.cuda(),
                               loss_weights=LOSS_WEIGHTS, max_batch=prob.shape.B, deferred_adamw=True)
    assert len(eng._deferred) == 2  # both mimic tables carry last_step
    assert "momentum_buffer" not in opts[0].state.get(tm.adaptive_mimic.item_augmented.weight, {})
    u, p, n, um, im = prob.batches[0]
    eng.step(u.cuda(), p.cuda(), n.cuda().reshape(-1), keep_masks={"user": [x.cuda() for x in um],
                                                                    "item": [x.cuda() for x in im]})
    assert opts[0].state[tm.adaptive_mimic.item_augmented.weight]["momentum_buffer"].shape == (prob.shape.I, 8)
    eng.finish()


@pytest.mark.parametrize("m0,m1", [(0.9, 0.0), (0.0, 0.9)], ids=["momentum-off", "momentum-on"])
def test_sgd_momentum_switch_between_zero_and_nonzero_rejected(m0, m1):
    """what the kernels' moment slots alias (momentum buffer or parameter) and whether
    g = 0 table rows are deferred are fixed when the step is built, so a later switch of SGD
    momentum between zero and non-zero raises ValueError before any state is written (torch would
    leave the buffers alone; the replay would overwrite them)."""
    import ttamm
    from gpu_helpers import ttamm_model_from, ttamm_optimizers
    from helpers import LOSS_WEIGHTS

    prob = make_problem(Shape(), steps=2)
    model = ttamm_model_from(prob)
    opts = ttamm_optimizers(model, lr=0.5, weight_decay=0.01, optimizer="sgd", momentum=m0)
    eng = ttamm.FusedTrainStep(model, opts, negatives_per_positive=prob.shape.N, positives=prob.positives,
                               user_features=prob.user_features.cuda(), item_features=prob.item_features.cuda(),
                               loss_weights=LOSS_WEIGHTS, max_batch=prob.shape.B)
    users, pos, neg, um, im = prob.batches[0]
    kw = dict(keep_masks={"user": [m.cuda() for m in um], "item": [m.cuda() for m in im]})
    eng.step(users.cuda(), pos.cuda(), neg.cuda().reshape(-1), **kw)
    before = {k: v.clone() for k, v in model.state_dict().items()}
    opts[0].param_groups[0]["momentum"] = m1
    users, pos, neg, um, im = prob.batches[1]
    with pytest.raises(ValueError, match="momentum"):
        eng.step(users.cuda(), pos.cuda(), neg.cuda().reshape(-1),
                 keep_masks={"user": [m.cuda() for m in um], "item": [m.cuda() for m in im]})
    opts[0].param_groups[0]["momentum"] = m0
    eng.finish()
    for k, v in model.state_dict().items():
        if "augmented" not in k:  # the mimic tables' deferred g = 0 rows move at finish
            assert torch.equal(v, before[k]), k
