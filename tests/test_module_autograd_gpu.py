"""Module-level autograd (ttamm/autograd.py): the reference's own loop body — training.py:738-827,
restated here call for call (``model.user_encoder(...)``, ``model.item_encoder(...)`` twice,
``model.adaptive_mimic(...)`` and ``augment_items``, the logits and BCE in torch, ``backward()``,
the caller's AdamW + SparseAdam) — run with ttamm's modules on the MI355X, against the CPU
oracle's step on the same parameters, batch and negatives.  Dropout p = 0 (the module path
draws its masks from an on-device Philox stream, not torch's CPU one).

Tolerances: one step at lr = 0, betas (0, 0.999) — exp_avg == the gradient on both sides —
1e-5 norm-wise relative per tensor (the tests' rel_err); three real AdamW / SparseAdam steps:
parameters within 5e-5 absolute (Adam normalises each update to ~lr), as the fused step's
three-step test."""

from __future__ import annotations

import pytest
import torch
from torch import nn

import ttamm
from helpers import LOSS_WEIGHTS, Shape, make_problem, named_optimizer_state, rel_err, run_oracle

pytestmark = pytest.mark.gpu


def reference_loop_body(model, optimizers, users, pos, neg, user_features, item_features, criterion, lw, N):
    """training.py:738-827 (the sampler's output given as ``neg``)."""
    for opt in optimizers:
        opt.zero_grad()
    user_inputs = {"indices": users, "features": user_features.index_select(0, users)}
    pos_item_inputs = {"indices": pos, "features": item_features.index_select(0, pos)}
    user_embeddings_base = model.user_encoder(user_inputs)
    pos_item_embeddings_base = model.item_encoder(pos_item_inputs)
    mimic_module = model.adaptive_mimic
    if mimic_module is not None:
        user_embeddings, pos_item_embeddings, mimic_user_loss, mimic_item_loss = mimic_module(
            user_indices=users, item_indices=pos, user_embedding=user_embeddings_base,
            item_embedding=pos_item_embeddings_base)
    else:
        user_embeddings, pos_item_embeddings = user_embeddings_base, pos_item_embeddings_base
        mimic_user_loss = mimic_item_loss = None
    pos_logits = (user_embeddings * pos_item_embeddings).sum(dim=-1)
    neg_flat = neg.view(-1)
    neg_inputs = {"indices": neg_flat, "features": item_features.index_select(0, neg_flat)}
    neg_item_embeddings_base = model.item_encoder(neg_inputs)
    if mimic_module is not None:
        neg_item_embeddings = mimic_module.augment_items(neg_flat, neg_item_embeddings_base)
    else:
        neg_item_embeddings = neg_item_embeddings_base
    neg_item_embeddings = neg_item_embeddings.view(-1, N, user_embeddings.shape[-1])
    neg_logits = (user_embeddings.unsqueeze(1) * neg_item_embeddings).sum(dim=-1)
    logits = torch.cat([pos_logits, neg_logits.reshape(-1)], dim=0)
    labels = torch.cat([torch.ones_like(pos_logits), torch.zeros_like(neg_logits.reshape(-1))], dim=0)
    total_loss = criterion(logits, labels)
    if mimic_user_loss is not None and lw["mimic_user"] > 0:
        total_loss = total_loss + lw["mimic_user"] * mimic_user_loss
    if mimic_item_loss is not None and lw["mimic_item"] > 0:
        total_loss = total_loss + lw["mimic_item"] * mimic_item_loss
    total_loss.backward()
    for opt in optimizers:
        opt.step()
    return float(total_loss.item())


def _ttamm_model(prob, shape):
    cfg = shape.tower_cfg()
    ue = ttamm.build_tower_encoder(cfg, num_embeddings=shape.U, feature_dim=shape.F, device="cuda")
    ie = ttamm.build_tower_encoder(cfg, num_embeddings=shape.I, feature_dim=shape.F, device="cuda")
    mm = ttamm.AdaptiveMimicMechanism(num_users=shape.U, num_items=shape.I, embedding_dim=shape.P).cuda() \
        if shape.mimic else None
    model = ttamm.TwoTowerModel(ue, ie, similarity=ttamm.DotProductSimilarity(), adaptive_mimic=mm)
    model.load_state_dict({k: v.cuda() for k, v in prob.model.state_dict().items()}, strict=True)
    return model


def _run_modules(prob, shape, *, lr, betas, steps):
    model = _ttamm_model(prob, shape)
    model.train()
    dense, sparse = ttamm._collect_parameter_groups(model)
    opts = [torch.optim.AdamW(dense, lr=lr or 1e-3, weight_decay=0.01, betas=betas)]
    if sparse:
        opts.append(torch.optim.SparseAdam(sparse, lr=lr or 1e-3, betas=betas))
    for o in opts:
        for g in o.param_groups:
            g["lr"] = lr
    uf, itf = prob.user_features.cuda(), prob.item_features.cuda()
    crit = nn.BCEWithLogitsLoss()
    lw = {"mimic_user": LOSS_WEIGHTS["mimic_user"], "mimic_item": LOSS_WEIGHTS["mimic_item"]}
    losses = []
    for users, pos, neg, _, _ in prob.batches[:steps]:
        losses.append(reference_loop_body(model, opts, users.cuda(), pos.cuda(), neg.cuda(), uf, itf, crit, lw,
                                          shape.N))
    torch.cuda.synchronize()
    return model, opts, losses


SHAPES = [
    Shape(dropout=0.0),
    Shape(dropout=0.0, sparse=False),
    Shape(dropout=0.0, fusion="sum"),
    Shape(dropout=0.0, fusion="concat"),
    Shape(dropout=0.0, fusion="concat", feature_out=12, concat_out=20),
    Shape(dropout=0.0, activation="gelu", hidden_dims=(16, 12)),
    Shape(dropout=0.0, mimic=False),
    Shape(dropout=0.0, padding_idx=5),
    Shape(U=64, I=512, F=605, H=192, D=96, B=96, N=5, hidden_dims=(192,), dropout=0.0),
]
IDS = ["gated", "dense-id", "sum", "concat", "concat-out20", "gelu-2hidden", "nomimic", "padding", "c2-dims"]


@pytest.mark.parametrize("shape", SHAPES, ids=IDS)
def test_reference_loop_body_gradients_match_oracle(shape):
    prob = make_problem(shape, steps=1)
    om, oo, ores = run_oracle(prob, lr=0.0, betas=(0.0, 0.999))
    tm, to, tl = _run_modules(prob, shape, lr=0.0, betas=(0.0, 0.999), steps=1)
    assert abs(tl[0] - ores[0].total) <= 1e-5 * abs(ores[0].total), (tl[0], ores[0].total)
    og, tg = named_optimizer_state(om, oo), named_optimizer_state(tm, to)
    assert set(og) == set(tg)
    for name in og:
        err = rel_err(tg[name]["exp_avg"], og[name]["exp_avg"])
        assert err <= 1e-5, f"{name}: rel err {err:.3e}"


@pytest.mark.parametrize("shape", [Shape(dropout=0.0), Shape(dropout=0.0, sparse=False, padding_idx=3)],
                         ids=["sparse-id", "dense-id-padding"])
def test_reference_loop_body_three_steps_match_oracle(shape):
    prob = make_problem(shape, steps=3)
    om, oo, ores = run_oracle(prob)
    tm, to, tl = _run_modules(prob, shape, lr=1e-3, betas=(0.9, 0.999), steps=3)
    for o, t in zip(ores, tl):
        assert abs(t - o.total) <= 1e-5 * abs(o.total)
    osd, tsd = om.state_dict(), tm.state_dict()
    for n in osd:
        d = (tsd[n].cpu() - osd[n]).abs().max().item()
        assert d <= 5e-5, f"{n}: max abs diff {d:.3e}"


def test_feature_fusion_gate_forward_backward_match_torch():
    """FeatureFusionGate.forward on its own (encoders.py:164-168), autograd to both inputs and
    the gate's parameters, against the same module's torch CPU forward / backward."""
    torch.manual_seed(3)
    D, n = 32, 300
    gate = ttamm.FeatureFusionGate(D).cuda()
    ref = nn.Sequential(nn.Linear(2 * D, D), nn.ReLU(), nn.Linear(D, D), nn.Sigmoid())
    ref.load_state_dict({k: v.cpu() for k, v in gate.gate_network.state_dict().items()})
    e = torch.randn(n, D, requires_grad=True)
    f = torch.randn(n, D, requires_grad=True)
    g = ref(torch.cat([e, f], dim=-1))
    out_ref = g * e + (1.0 - g) * f
    w = torch.randn(n, D)
    (out_ref * w).sum().backward()
    e2 = e.detach().cuda().requires_grad_(True)
    f2 = f.detach().cuda().requires_grad_(True)
    out = gate(e2, f2)
    assert rel_err(out, out_ref) <= 1e-5
    (out * w.cuda()).sum().backward()
    assert rel_err(e2.grad, e.grad) <= 1e-5
    assert rel_err(f2.grad, f.grad) <= 1e-5
    for (name, p), q in zip(gate.gate_network.named_parameters(), ref.parameters()):
        assert rel_err(p.grad, q.grad) <= 1e-5, name


def test_train_mode_dropout_runs_and_is_reproducible():
    """Dropout p > 0 in train mode: the module path draws its masks on the device (Philox keyed
    by torch's seeded generator), so two seeded runs agree bit for bit and the gradient differs
    from the eval-mode (no-dropout) one."""
    shape = Shape(dropout=0.3)
    prob = make_problem(shape, steps=1)

    def grads(train: bool):
        torch.manual_seed(17)
        model = _ttamm_model(prob, shape)
        model.train(train)
        users, pos, neg, _, _ = prob.batches[0]
        out = model.item_encoder({"indices": pos.cuda(), "features": prob.item_features.cuda()[pos.cuda()]})
        out.square().sum().backward()
        return model.item_encoder.feature_encoder.network[0].weight.grad.clone()

    a, b, c = grads(True), grads(True), grads(False)
    assert torch.equal(a, b)
    assert not torch.equal(a, c)


def test_mse_target_gradient_matches_torch():
    """ttamm's F.mse_loss (adaptive_mimic._mse) with a target that requires grad: both inputs get
    F.mse_loss's gradients (the reference detaches the target; an undetached one is not dropped)."""
    from ttamm.adaptive_mimic import _mse

    torch.manual_seed(5)
    x = torch.randn(40, 16, device="cuda", requires_grad=True)
    y = torch.randn(40, 16, device="cuda", requires_grad=True)
    _mse(x, y).backward()
    x2, y2 = x.detach().clone().requires_grad_(True), y.detach().clone().requires_grad_(True)
    torch.nn.functional.mse_loss(x2, y2).backward()
    assert rel_err(x.grad, x2.grad) <= 1e-6 and rel_err(y.grad, y2.grad) <= 1e-6
    y3 = y.detach().clone().requires_grad_(True)  # only the target requires grad
    _mse(x.detach(), y3).backward()
    assert rel_err(y3.grad, y2.grad) <= 1e-6


def test_tower_forward_with_mimic_rows_under_autograd():
    """encoders.tower_forward(..., mimic_table=) in train mode: the tower's training forward plus
    table[idx] with the table's gradient (adaptive_mimic.py:88-95), not the eval kernel."""
    from ttamm.encoders import tower_forward

    shape = Shape(dropout=0.0)
    prob = make_problem(shape, steps=1)
    model = _ttamm_model(prob, shape)
    model.train()
    users, pos, _, _, _ = prob.batches[0]
    table = model.adaptive_mimic.item_augmented.weight
    feats = prob.item_features.cuda()[pos.cuda()]
    out = tower_forward(model.item_encoder, pos.cuda(), features=feats, mimic_table=table)
    assert out.grad_fn is not None
    base = model.item_encoder({"indices": pos.cuda(), "features": feats})
    assert rel_err(out, base + table[pos.cuda()]) <= 1e-6
    w = torch.randn_like(out)
    (out * w).sum().backward()
    want = torch.zeros_like(table).index_add_(0, pos.cuda(), w)
    assert rel_err(table.grad, want) <= 1e-6
    assert model.item_encoder.embedding.weight.grad is not None


@pytest.mark.parametrize("D", [128, 256])
def test_bf16_tower_fused_gate_matches_generic_gate(D, monkeypatch):
    """The module path (ttamm_tower_forward / _backward) of a bf16 gated tower at D == Hg in
    {128, 256}: the fused bf16 gate (gate16.hip, its weight images formed in each call) against the
    generic two-GEMM gate (TTAMM_GENERIC_GATE=1) on the same rows and output gradient, at the bf16
    tolerance of the step tests (2e-3 max-norm, 2e-5 mean, per tensor)."""
    import copy

    shape = Shape(U=900, I=900, F=40, H=D, D=D, hidden_dims=(D,), matmul_dtype="bf16", dropout=0.0)
    torch.manual_seed(7)
    enc0 = ttamm.build_tower_encoder(shape.tower_cfg(), num_embeddings=900, feature_dim=40, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(7)
    R = 1300  # 11 blocks of 128 rows, the last one partial
    idx = torch.randint(0, 900, (R,), device="cuda", generator=g)
    feats = torch.randn((R, 40), device="cuda", generator=g)
    dT = torch.randn((R, D), device="cuda", generator=g)
    res = {}
    for mode in ("fused", "generic"):
        if mode == "generic":
            monkeypatch.setenv("TTAMM_GENERIC_GATE", "1")
        else:
            monkeypatch.delenv("TTAMM_GENERIC_GATE", raising=False)
        enc = copy.deepcopy(enc0)
        out = enc({"indices": idx, "features": feats})
        out.backward(dT)
        torch.cuda.synchronize()
        grads = {n: (p.grad.to_dense() if p.grad.is_sparse else p.grad).clone()
                 for n, p in enc.named_parameters() if p.grad is not None}
        res[mode] = (out.detach().clone(), grads)
    (of, gf), (og, gg) = res["fused"], res["generic"]
    assert rel_err(of, og) <= 2e-3
    assert set(gf) == set(gg) and gf
    for n in gg:
        err = rel_err(gf[n], gg[n])
        mean = ((gf[n].double() - gg[n].double()).abs().mean() / gg[n].double().abs().max().clamp_min(1e-30)).item()
        assert err <= 2e-3, f"{n}: rel err {err:.3e}"
        assert mean <= 2e-5, f"{n}: mean rel err {mean:.3e}"
