"""Out-of-range ids (nn.Embedding raises IndexError, encoders.py:222-223 / adaptive_mimic.py:97-105).

The fused step checks every batch id on the device (ttamm.h TTAMM_STATUS_INDEX_OUT_OF_RANGE):
a bad id never reads or writes outside a table, the failing step and every later one write
nothing, and ``finish()`` raises IndexError with the model and optimizer state equal to the
state after the last good step (the reference raises inside the failing batch, before its
backward).  The module entry points raise before launching anything."""

from __future__ import annotations

import pytest
import torch

import ttamm
from helpers import LOSS_WEIGHTS, Shape, make_problem

pytestmark = pytest.mark.gpu


def _engine(prob, *, sparse=True, deferred=True):
    from gpu_helpers import ttamm_model_from

    model = ttamm_model_from(prob)
    dense, sp = ttamm._collect_parameter_groups(model)
    if not sparse:
        dense, sp = dense + sp, []
    opts = [torch.optim.AdamW(dense, lr=1e-3, weight_decay=0.01)]
    if sp:
        opts.append(torch.optim.SparseAdam(sp, lr=1e-3))
    eng = ttamm.FusedTrainStep(model, opts, negatives_per_positive=prob.shape.N, positives=prob.positives,
                               user_features=prob.user_features.cuda(), item_features=prob.item_features.cuda(),
                               loss_weights=LOSS_WEIGHTS, max_batch=prob.shape.B, seed=5, deferred_adamw=deferred,
                               replay_slices=3)
    return model, opts, eng


def _state(model, opts):
    out = {k: v.detach().clone() for k, v in model.state_dict().items()}
    for i, o in enumerate(opts):
        for j, (p, st) in enumerate(o.state.items()):
            for k, v in st.items():
                out[f"opt{i}.{j}.{k}"] = v.detach().clone() if torch.is_tensor(v) else torch.tensor(float(v))
    return out


def _batches(prob, n):
    gen = torch.Generator().manual_seed(9)
    out = []
    for _ in range(n):
        users = torch.randint(0, prob.shape.U, (prob.shape.B,), generator=gen)
        pos = torch.tensor([sorted(prob.positives[int(u)])[0] for u in users], dtype=torch.long)
        neg = torch.randint(0, prob.shape.I, (prob.shape.B * prob.shape.N,), generator=gen)
        out.append((users, pos, neg))
    return out


@pytest.mark.parametrize(
    "where,bad,sparse,deferred",
    [
        ("pos", 256, True, True),      # == item rows
        ("pos", -1, True, False),
        ("user", 64, True, True),      # == user rows
        ("user", -7, False, True),
        ("neg", 10**9, True, True),
        ("neg", -2, False, False),
    ],
)
def test_step_raises_index_error_and_keeps_last_good_state(where, bad, sparse, deferred):
    prob = make_problem(Shape(), seed=4)
    batches = _batches(prob, 3)
    # reference state: only the first (good) step
    m1, o1, e1 = _engine(prob, sparse=sparse, deferred=deferred)
    u, p, n = batches[0]
    e1.step(u.cuda(), p.cuda(), n.cuda())
    loss1 = e1.finish()
    want = _state(m1, o1)
    # the same first step, then a step with one bad id, then a good step (skipped too)
    m2, o2, e2 = _engine(prob, sparse=sparse, deferred=deferred)
    for k, (u, p, n) in enumerate(batches):
        u, p, n = u.clone(), p.clone(), n.clone()
        if k == 1:
            {"pos": p, "user": u, "neg": n}[where][5] = bad
        e2.step(u.cuda(), p.cuda(), n.cuda())
    with pytest.raises(IndexError, match="index out of range"):
        e2.finish()
    got = _state(m2, o2)
    assert want.keys() == got.keys()
    for k in want:
        assert torch.equal(want[k].cpu(), got[k].cpu()), k
    assert e2.loss_accum[1].item() == prob.shape.B  # only the good step's positives were accumulated
    assert loss1 == pytest.approx(e2.loss_accum[0].item() / e2.loss_accum[1].item(), rel=0, abs=0)


def test_bad_first_step_leaves_tables_untouched():
    prob = make_problem(Shape(), seed=6)
    model, opts, eng = _engine(prob)
    before = {k: v.detach().clone() for k, v in model.state_dict().items()}
    u, p, n = _batches(prob, 1)[0]
    p[0] = prob.shape.I + 3
    eng.step(u.cuda(), p.cuda(), n.cuda())
    with pytest.raises(IndexError):
        eng.finish()
    for k, v in model.state_dict().items():
        assert torch.equal(v, before[k]), k
    for o in opts:
        for st in o.state.values():
            assert float(st["step"]) == 0.0


def test_module_entry_points_raise_index_error():
    prob = make_problem(Shape(), seed=7)
    from gpu_helpers import ttamm_model_from

    model = ttamm_model_from(prob).eval()
    feats = prob.item_features.cuda()
    with torch.no_grad():
        bad = torch.tensor([0, prob.shape.I], dtype=torch.long, device="cuda")
        with pytest.raises(IndexError):
            model.item_encoder({"indices": bad, "features": feats[:2]})
        with pytest.raises(IndexError):
            model.adaptive_mimic.augment_items(bad, torch.zeros((2, prob.shape.D), device="cuda"))
        with pytest.raises(IndexError):
            model.user_encoder({"indices": torch.tensor([-1], device="cuda")})


def test_c_abi_gather_never_reads_outside_the_table():
    """The C ABI (no Python check) writes zero rows for ids outside the table."""
    lib = ttamm._lib.load()
    for D in (96, 128, 6):  # wide, wide, scalar paths
        table = torch.randn((100, D), device="cuda")
        idx = torch.tensor([3, -1, 100, 99, 1 << 40, 0], dtype=torch.long, device="cuda")
        out = torch.full((6, D), 7.0, device="cuda")
        ttamm._lib.check(lib.ttamm_gather_rows(table.data_ptr(), 100, D, idx.data_ptr(), 6, out.data_ptr(), D,
                                               ttamm._lib.stream_handle()))
        torch.cuda.synchronize()
        ok = torch.tensor([True, False, False, True, False, True], device="cuda")
        assert torch.equal(out[ok], table[idx[ok]])
        assert torch.count_nonzero(out[~ok]) == 0
