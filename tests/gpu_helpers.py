"""Builders for the ttamm (MI355X) side of parity tests."""

from __future__ import annotations

import torch

import ttamm
from helpers import LOSS_WEIGHTS, Problem, set_lr


def ttamm_model_from(prob: Problem, device="cuda"):
    s = prob.shape
    cfg = s.tower_cfg()
    torch.manual_seed(0)
    ue = ttamm.build_tower_encoder(cfg, num_embeddings=s.U, feature_dim=s.F, device=device)
    ie = ttamm.build_tower_encoder(cfg, num_embeddings=s.I, feature_dim=s.F, device=device)
    mm = ttamm.AdaptiveMimicMechanism(num_users=s.U, num_items=s.I, embedding_dim=s.P).to(device) if s.mimic else None
    model = ttamm.TwoTowerModel(ue, ie, similarity=ttamm.DotProductSimilarity(), adaptive_mimic=mm)
    missing = model.load_state_dict({k: v.to(device) for k, v in prob.model.state_dict().items()}, strict=True)
    assert not missing.missing_keys and not missing.unexpected_keys
    return model


def ttamm_optimizers(model, *, lr=1e-3, betas=(0.9, 0.999), weight_decay=0.01, optimizer="adamw", momentum=0.0):
    """training.py:1311-1350 on the ttamm model (the same construction as oracle.build_optimizers)."""
    dense, sparse = ttamm._collect_parameter_groups(model)
    if optimizer == "sgd":
        opts = [torch.optim.SGD(dense, lr=lr or 1e-3, weight_decay=weight_decay, momentum=momentum)]
    else:
        cls = torch.optim.AdamW if optimizer == "adamw" else torch.optim.Adam
        opts = [cls(dense, lr=lr or 1e-3, weight_decay=weight_decay, betas=betas)]
    if sparse:
        opts.append(torch.optim.SparseAdam(sparse, lr=lr or 1e-3, betas=betas))
    set_lr(opts, lr)
    return opts


def run_ttamm(prob: Problem, *, lr=1e-3, betas=(0.9, 0.999), weight_decay=0.01, steps=None, device="cuda",
              gradient_clip_norm=None, optimizer="adamw", momentum=0.0, deferred_adamw=True):
    model = ttamm_model_from(prob, device)
    opts = ttamm_optimizers(model, lr=lr, betas=betas, weight_decay=weight_decay, optimizer=optimizer,
                            momentum=momentum)
    eng = ttamm.FusedTrainStep(
        model, opts, negatives_per_positive=prob.shape.N, positives=prob.positives,
        user_features=prob.user_features.to(device), item_features=prob.item_features.to(device),
        loss_weights=LOSS_WEIGHTS, max_batch=prob.shape.B, gradient_clip_norm=gradient_clip_norm,
        deferred_adamw=deferred_adamw,
    )
    losses = []
    for (users, pos, neg, um, im) in prob.batches[: steps or len(prob.batches)]:
        eng.step(users.to(device), pos.to(device), neg.to(device).reshape(-1),
                 keep_masks={"user": [m.to(device) for m in um], "item": [m.to(device) for m in im]})
        losses.append(eng.last_losses())
    eng.finish()
    return model, opts, losses
