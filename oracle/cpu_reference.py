"""PyTorch-CPU restatement of the reference training step (TEST INFRASTRUCTURE ONLY).

See oracle/__init__.py for scope and pinning status.  Module classes here mirror the
reference's parameter layout so ``state_dict`` keys are interchangeable with
ttamm's modules (and with the reference's checkpoints, training.py:173-181).
"""

from __future__ import annotations

import math
import time
from dataclasses import dataclass
from typing import Any, Iterable, Mapping, Sequence

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn


# ---------------------------------------------------------------------------------------
# modules (reference: src/models/encoders.py, adaptive_mimic.py, two_tower.py)
# ---------------------------------------------------------------------------------------
class FeatureEncoderWrapper(nn.Module):  # encoders.py:81-90
    def __init__(self, network: nn.Module, output_dim: int) -> None:
        super().__init__()
        self.network = network
        self.output_dim = output_dim


class FeatureFusionGate(nn.Module):  # encoders.py:149-168
    def __init__(self, dim: int, hidden_dim: int | None = None) -> None:
        super().__init__()
        h = hidden_dim or dim
        self.gate_network = nn.Sequential(nn.Linear(2 * dim, h), nn.ReLU(), nn.Linear(h, dim), nn.Sigmoid())


class OracleTower(nn.Module):  # encoders.py:171-219 (constructor) — forward is tower_forward below
    def __init__(self, embedding: nn.Embedding, feature_encoder, fusion: str, gate, matmul_dtype: str = "fp32",
                 output_dim: int | None = None) -> None:
        super().__init__()
        # not in the reference: the "bf16 towers" precision of BASELINE config C5 (see _bf16_linear)
        self.matmul_dtype = matmul_dtype
        self.embedding = embedding
        self.feature_encoder = feature_encoder
        self.fusion = "identity" if feature_encoder is None else fusion
        self.adaptive_mimic = gate
        self.num_embeddings = embedding.num_embeddings
        self.id_dim = embedding.embedding_dim
        self.output_dim = self.id_dim
        if self.fusion == "concat":  # encoders.py:211-216
            joint = self.id_dim + feature_encoder.output_dim
            self.projection = nn.Linear(joint, int(output_dim or joint))
            nn.init.xavier_uniform_(self.projection.weight)
            self.output_dim = self.projection.out_features


class OracleMimic(nn.Module):  # adaptive_mimic.py:20-38
    def __init__(self, num_users: int, num_items: int, embedding_dim: int, init_std: float = 0.02) -> None:
        super().__init__()
        if num_users <= 0 or num_items <= 0:
            raise ValueError("num_users and num_items must be positive.")
        self.embedding_dim = embedding_dim
        self.user_augmented = nn.Embedding(num_users, embedding_dim)
        self.item_augmented = nn.Embedding(num_items, embedding_dim)
        nn.init.normal_(self.user_augmented.weight, mean=0.0, std=init_std)
        nn.init.normal_(self.item_augmented.weight, mean=0.0, std=init_std)


class OracleModel(nn.Module):  # two_tower.py:19-38
    def __init__(self, user_encoder, item_encoder, adaptive_mimic=None) -> None:
        super().__init__()
        self.user_encoder = user_encoder
        self.item_encoder = item_encoder
        self.similarity = nn.CosineSimilarity(dim=-1)
        self.adaptive_mimic = adaptive_mimic


def _activation(name: str) -> nn.Module:  # encoders.py:68-78 _get_activation
    key = name.lower()
    if key == "relu":
        return nn.ReLU()
    if key == "gelu":
        return nn.GELU()
    if key == "tanh":
        return nn.Tanh()
    if key == "selu":
        return nn.SELU()
    raise ValueError(f"Unsupported activation '{name}'")


def build_tower(cfg: Mapping[str, Any], *, num_embeddings: int, feature_dim: int) -> OracleTower:
    """encoders.py:258-331 with the same parameter construction / init order."""
    id_cfg = cfg.get("id_embedding", {}) or {}
    params = id_cfg.get("params", {}) or {}
    if bool(params.get("sparse", False)) and params.get("max_norm") is not None:  # encoders.py:51-52
        raise ValueError("max_norm is not supported when using sparse embeddings.")
    emb = nn.Embedding(num_embeddings, int(params.get("embedding_dim", 64)), padding_idx=params.get("padding_idx"),
                       max_norm=params.get("max_norm"), sparse=bool(params.get("sparse", False)))
    init = id_cfg.get("init") or {"type": "normal", "std": 0.02}
    nn.init.normal_(emb.weight, mean=0.0, std=float(init.get("std", 0.02)))  # encoders.py:25-27
    fusion = str(cfg.get("fusion", "gated" if feature_dim > 0 else "identity")).lower()
    fe = None
    if feature_dim > 0:
        fcfg = dict(cfg.get("feature_encoder") or {})
        out = int(fcfg.get("output_dim") or emb.embedding_dim)
        kind = fcfg.get("type", "linear")
        if kind == "linear":  # encoders.py:121-124
            lin = nn.Linear(feature_dim, out)
            nn.init.xavier_uniform_(lin.weight)
            fe = FeatureEncoderWrapper(lin, out)
        elif kind == "identity":  # encoders.py:114-119
            if feature_dim != out:
                raise ValueError("Identity feature encoder requires input_dim == output_dim.")
            fe = FeatureEncoderWrapper(nn.Identity(), out)
        elif kind == "mlp":  # encoders.py:126-144
            mods: list[nn.Module] = []
            prev = feature_dim
            act = _activation(str(fcfg.get("activation", "relu")))  # encoders.py:68-78, one shared module
            for h in fcfg.get("hidden_dims") or []:
                lin = nn.Linear(prev, int(h))
                nn.init.xavier_uniform_(lin.weight)
                mods += [lin, act]
                if fcfg.get("dropout"):
                    mods.append(nn.Dropout(p=float(fcfg["dropout"])))
                prev = int(h)
            last = nn.Linear(prev, out)
            nn.init.xavier_uniform_(last.weight)
            mods.append(last)
            fe = FeatureEncoderWrapper(nn.Sequential(*mods), out)
        else:
            raise ValueError(f"oracle: unsupported feature encoder {kind}")
    gate = None
    if fusion in ("gated", "adaptive_mimic"):
        gate = FeatureFusionGate(emb.embedding_dim, (cfg.get("adaptive_mimic") or {}).get("hidden_dim"))
        fusion = "gated"
    mm = str(cfg.get("matmul_dtype", "fp32")).lower()
    return OracleTower(emb, fe, fusion, gate, "bf16" if mm in ("bf16", "bfloat16") else "fp32",
                       output_dim=cfg.get("output_dim"))


def build_model(
    tower_cfg: Mapping[str, Any], *, num_users: int, num_items: int, user_feature_dim: int, item_feature_dim: int,
    mimic: bool = True, init_std: float = 0.02,
) -> OracleModel:
    """training.py:1266-1301."""
    ue = build_tower(tower_cfg, num_embeddings=num_users, feature_dim=user_feature_dim)
    ie = build_tower(tower_cfg, num_embeddings=num_items, feature_dim=item_feature_dim)
    mm = OracleMimic(num_users, num_items, ue.output_dim, init_std) if mimic else None
    return OracleModel(ue, ie, mm)


# ---------------------------------------------------------------------------------------
# forward (encoders.py:221-255) with optional injected dropout keep-masks
# ---------------------------------------------------------------------------------------
def _dropout(x: torch.Tensor, p: float, keep: torch.Tensor | None, training: bool) -> torch.Tensor:
    if not training or p == 0.0:
        return x
    if keep is None:
        return F.dropout(x, p=p, training=True)
    noise = keep.to(torch.float32)
    noise.div_(1 - p)  # ATen _dropout_impl: noise.bernoulli_(1-p).div_(1-p); input * noise
    return x * noise


def _round_bf16(x: torch.Tensor) -> torch.Tensor:
    return x.to(torch.bfloat16).to(torch.float32)  # round to nearest even


class _BF16Linear(torch.autograd.Function):
    """nn.Linear with bf16 operands and fp32 accumulation — the definition of ttamm's
    matmul_dtype="bf16" (not reference behaviour; BASELINE config C5 "bf16 towers").  Every
    product of the forward and of both gradients rounds its two operands to bf16:
    y = bf(x) bf(W)^T + b,  dx = bf(dy) bf(W),  dW = bf(dy)^T bf(x),  db = sum bf(dy)."""

    @staticmethod
    def forward(ctx, x, w, b):
        xr, wr = _round_bf16(x), _round_bf16(w)
        ctx.save_for_backward(xr, wr)
        return xr @ wr.t() + b

    @staticmethod
    def backward(ctx, dy):
        xr, wr = ctx.saved_tensors
        dyr = _round_bf16(dy)
        return dyr @ wr, dyr.t() @ xr, dyr.sum(0)


def _linear(lin: nn.Linear, x: torch.Tensor, bf16: bool) -> torch.Tensor:
    return _BF16Linear.apply(x, lin.weight, lin.bias) if bf16 else lin(x)


def feature_forward(fe: FeatureEncoderWrapper, x: torch.Tensor, keep_masks: Sequence[torch.Tensor] | None,
                    training: bool, bf16: bool = False) -> torch.Tensor:
    net = fe.network
    if isinstance(net, nn.Linear):
        return _linear(net, x, bf16)
    if isinstance(net, nn.Identity):  # encoders.py:114-119
        return x
    hidden = 0
    for m in net:
        if isinstance(m, nn.Dropout):
            keep = keep_masks[hidden] if keep_masks is not None else None
            x = _dropout(x, m.p, keep, training)
            hidden += 1
        elif isinstance(m, nn.Linear):
            x = _linear(m, x, bf16)
        else:
            x = m(x)
    return x


def tower_forward(tower: OracleTower, idx: torch.Tensor, feats: torch.Tensor | None,
                  keep_masks: Sequence[torch.Tensor] | None = None, training: bool = True) -> torch.Tensor:
    e = tower.embedding(idx)  # encoders.py:223
    if tower.fusion == "identity" or tower.feature_encoder is None or feats is None:
        return e
    bf16 = tower.matmul_dtype == "bf16"
    f = feature_forward(tower.feature_encoder, feats, keep_masks, training, bf16)  # :233
    if tower.fusion == "sum":
        return e + f  # :240
    if tower.fusion == "concat":
        return _linear(tower.projection, torch.cat([e, f], dim=-1), bf16)  # :242-244
    g1, _, g2, _ = tower.adaptive_mimic.gate_network  # Linear, ReLU, Linear, Sigmoid (:157-162)
    ef = torch.cat([e, f], dim=-1)
    pre = _linear(g1, ef, bf16)
    hidden = torch.relu(pre) if GATE_HIDDEN_HOOK is None else GATE_HIDDEN_HOOK(tower, ef, pre)
    gate = torch.sigmoid(_linear(g2, hidden, bf16))  # :164-168
    return gate * e + (1.0 - gate) * f


# Test hook (tests/test_fullsize_parity_gpu.py, fp32 ReLU kinks): when set, the gate's hidden
# activation is GATE_HIDDEN_HOOK(tower, [e | f], pre-activation) instead of relu(pre-activation).
GATE_HIDDEN_HOOK = None


def gather_aug(table: nn.Embedding, idx: torch.Tensor, reference: torch.Tensor):
    """adaptive_mimic.py:88-105: (reference + table[idx], table[idx])."""
    if idx.dtype != torch.long:
        raise ValueError("Adaptive mimic indices must be torch.long tensors.")
    aug = table(idx.reshape(-1)).reshape(reference.shape)
    return reference + aug, aug


# ---------------------------------------------------------------------------------------
# sampler (samplers.py:11-85)
# ---------------------------------------------------------------------------------------
def sample_negative_items(users: torch.Tensor, *, num_items: int, positives: Mapping[int, set[int]],
                          num_negatives: int, generator: torch.Generator | None = None) -> torch.Tensor:
    if num_negatives <= 0:
        raise ValueError("num_negatives must be greater than zero.")
    if num_items <= 1:
        raise ValueError("num_items must be greater than one.")
    out = torch.empty((users.shape[0], num_negatives), dtype=torch.long)
    cache: dict[int, torch.Tensor] = {}
    for row, u in enumerate(users.tolist()):
        pos = positives.get(int(u), set())
        if len(pos) >= num_items:
            raise RuntimeError(f"User {int(u)} interacted with all items; cannot sample negatives.")
        pt = None
        if pos:
            pt = cache.get(int(u))
            if pt is None:
                pt = torch.tensor(sorted(pos), dtype=torch.long)
                cache[int(u)] = pt
        draw = torch.randint(0, num_items, (num_negatives,), dtype=torch.long, generator=generator)
        if pt is not None:
            bad = torch.isin(draw, pt)
            rounds = 0
            while bad.any():
                draw[bad] = torch.randint(0, num_items, (int(bad.sum().item()),), dtype=torch.long, generator=generator)
                bad = torch.isin(draw, pt)
                rounds += 1
                if rounds > 10:
                    raise RuntimeError("Exceeded resampling attempts while drawing negatives.")
        out[row] = draw
    return out


# ---------------------------------------------------------------------------------------
# optimizers (training.py:276-309, :1311-1350)
# ---------------------------------------------------------------------------------------
def parameter_groups(model: OracleModel) -> tuple[list, list]:
    dense, sparse, seen = [], [], set()

    def put(p, bucket):
        if id(p) not in seen:
            seen.add(id(p))
            bucket.append(p)

    for tower in (model.user_encoder, model.item_encoder):
        put(tower.embedding.weight, sparse if tower.embedding.sparse else dense)
        for name, p in tower.named_parameters():
            if name != "embedding.weight":
                put(p, dense)
    for p in model.parameters():
        put(p, dense)
    return dense, sparse


def build_optimizers(model: OracleModel, *, lr: float = 1e-3, weight_decay: float = 0.01, betas=(0.9, 0.999),
                     optimizer: str = "adamw", momentum: float = 0.0) -> list[torch.optim.Optimizer]:
    """training.py:1311-1350: the dense group under Adam / AdamW / SGD(momentum) by
    ``training.optimizer`` (the reference passes no betas to the dense Adam / AdamW; ``betas``
    here serves the parity tests' lr = 0 gradient export), the sparse ID tables under SparseAdam."""
    dense, sparse = parameter_groups(model)
    opts: list[torch.optim.Optimizer] = []
    name = optimizer.lower()
    if dense:
        if name in ("adam", "adamw"):  # :1316-1323
            cls = torch.optim.AdamW if name == "adamw" else torch.optim.Adam
            opts.append(cls(dense, lr=lr, weight_decay=weight_decay, betas=betas))
        elif name == "sgd":  # :1324-1330
            opts.append(torch.optim.SGD(dense, lr=lr, weight_decay=weight_decay, momentum=float(momentum)))
        else:
            raise ValueError(f"Unsupported optimizer: {optimizer}")  # :1331-1332
    if sparse:
        opts.append(torch.optim.SparseAdam(sparse, lr=lr, betas=betas))
    return opts


# ---------------------------------------------------------------------------------------
# category-alignment loss (training.py:530-579)
# ---------------------------------------------------------------------------------------
def compute_covariance(matrix: torch.Tensor) -> torch.Tensor:  # training.py:530-538
    if matrix.shape[0] <= 1:
        return torch.zeros((matrix.shape[1], matrix.shape[1]), device=matrix.device, dtype=matrix.dtype)
    centered = matrix - matrix.mean(dim=0, keepdim=True)
    return centered.T @ centered / (matrix.shape[0] - 1)


def category_alignment_loss(item_indices: torch.Tensor, item_embeddings: torch.Tensor, *,
                            category_tensor: torch.Tensor | None, major_category_id: int | None) -> torch.Tensor:
    """training.py:541-579: sum over non-major categories with >= 2 rows in the batch of
    ||cov_c - cov_major||_F^2, divided by the number compared (ascending category order)."""
    if category_tensor is None or major_category_id is None or item_indices.numel() == 0:
        return item_embeddings.new_zeros(())
    batch_categories = category_tensor.index_select(0, item_indices)
    unique_categories = batch_categories.unique()
    if unique_categories.numel() <= 1:
        return item_embeddings.new_zeros(())
    major_mask = batch_categories == major_category_id
    if major_mask.sum() < 2:
        return item_embeddings.new_zeros(())
    major_cov = compute_covariance(item_embeddings[major_mask])
    loss = item_embeddings.new_zeros(())
    compared = 0
    for cat_id in unique_categories.tolist():
        if cat_id == major_category_id:
            continue
        mask = batch_categories == cat_id
        if mask.sum() < 2:
            continue
        diff = compute_covariance(item_embeddings[mask]) - major_cov
        loss = loss + torch.sum(diff * diff)
        compared += 1
    if compared == 0:
        return item_embeddings.new_zeros(())
    return loss / compared


# ---------------------------------------------------------------------------------------
# one training step (training.py:726-831)
# ---------------------------------------------------------------------------------------
@dataclass
class StepResult:
    total: float
    bce: float
    mimic_user: float
    mimic_item: float
    category_alignment: float = 0.0


def train_step(
    model: OracleModel,
    optimizers: Sequence[torch.optim.Optimizer],
    users: torch.Tensor,
    pos_items: torch.Tensor,
    neg_items: torch.Tensor,
    *,
    user_features: torch.Tensor | None,
    item_features: torch.Tensor | None,
    loss_weights: Mapping[str, float] | None = None,
    user_keep_masks: Sequence[torch.Tensor] | None = None,
    item_keep_masks: Sequence[torch.Tensor] | None = None,
    item_category_tensor: torch.Tensor | None = None,
    major_category_id: int | None = None,
    in_batch: bool = False,
    gradient_clip_norm: float | None = None,
) -> StepResult:
    """One iteration of _train_one_epoch's body.  item_keep_masks rows are ordered
    [positives; negatives] (the two item_encoder calls, training.py:750 and :776).

    ``in_batch`` — NOT reference behaviour (the reference scores sampled negatives only,
    training.py:770-798); this is the definition of ttamm's in-batch mode (BASELINE configs C2/C4
    "in-batch negatives"): every user is scored against every positive of the batch,
    logits_ib = u @ p^T [B, B] with label 1 on the diagonal, followed by its own sampled negatives
    (``neg_items`` may have 0 columns); one BCEWithLogits mean over all B(B + N) logits.  Mimic
    losses and L_cal are unchanged (L_cal still over cat[positives; sampled negatives])."""
    model.train()
    lw = dict(loss_weights or {})
    lam_u = float(lw.get("mimic_user", 0.0))
    lam_i = float(lw.get("mimic_item", 0.0))
    mimic = model.adaptive_mimic
    B = users.shape[0]
    N = neg_items.shape[1] if neg_items.dim() == 2 else 0
    for opt in optimizers:  # :738-739
        opt.zero_grad()
    uf = user_features.index_select(0, users) if user_features is not None and user_features.numel() else None
    pf = item_features.index_select(0, pos_items) if item_features is not None and item_features.numel() else None
    pos_masks = [m[:B] for m in item_keep_masks] if item_keep_masks is not None else None
    neg_masks = [m[B:] for m in item_keep_masks] if item_keep_masks is not None else None
    t_u = tower_forward(model.user_encoder, users, uf, user_keep_masks)  # :749
    t_p = tower_forward(model.item_encoder, pos_items, pf, pos_masks)  # :750
    loss_u = loss_i = None
    if mimic is not None:  # :752-763 -> adaptive_mimic.py:40-68
        u, a_u = gather_aug(mimic.user_augmented, users, t_u)
        p, a_p = gather_aug(mimic.item_augmented, pos_items, t_p)
        loss_u = F.mse_loss(a_u, t_p.detach())
        loss_i = F.mse_loss(a_p, t_u.detach())
    else:
        u, p = t_u, t_p
    pos_logits = (u * p).sum(dim=-1)  # :770
    neg_flat = neg_items.reshape(-1)
    if N > 0:
        nf = item_features.index_select(0, neg_flat) if item_features is not None and item_features.numel() else None
        t_n = tower_forward(model.item_encoder, neg_flat, nf, neg_masks)  # :776
        n = gather_aug(mimic.item_augmented, neg_flat, t_n)[0] if mimic is not None else t_n
        n = n.view(-1, N, u.shape[-1])
        neg_logits = (u.unsqueeze(1) * n).sum(dim=-1)  # :786-787
    else:
        n = u.new_zeros((B, 0, u.shape[-1]))
        neg_logits = u.new_zeros((B, 0))
    if in_batch:
        ib = u @ p.t()
        logits = torch.cat([ib.reshape(-1), neg_logits.reshape(-1)], dim=0)
        labels = torch.cat([torch.eye(B, dtype=u.dtype).reshape(-1), torch.zeros_like(neg_logits.reshape(-1))], dim=0)
    else:
        logits = torch.cat([pos_logits, neg_logits.reshape(-1)], dim=0)
        labels = torch.cat([torch.ones_like(pos_logits), torch.zeros_like(neg_logits.reshape(-1))], dim=0)
    bce = nn.BCEWithLogitsLoss()(logits, labels)  # :798, criterion :1366
    total = bce
    if loss_u is not None and lam_u > 0:
        total = total + lam_u * loss_u
    if loss_i is not None and lam_i > 0:
        total = total + lam_i * loss_i
    lam_cal = float(lw.get("category_alignment", 0.0))
    cal = None
    if lam_cal > 0:  # :805-820
        cal = category_alignment_loss(torch.cat([pos_items, neg_flat], dim=0),
                                      torch.cat([p, n.reshape(-1, u.shape[-1])], dim=0),
                                      category_tensor=item_category_tensor, major_category_id=major_category_id)
        total = total + lam_cal * cal
    total.backward()  # :822
    if gradient_clip_norm is not None and gradient_clip_norm > 0:  # :824-825
        torch.nn.utils.clip_grad_norm_(model.parameters(), gradient_clip_norm)
    for opt in optimizers:  # :826-827
        opt.step()
    return StepResult(
        float(total.item()), float(bce.item()),
        float(loss_u.item()) if loss_u is not None else 0.0,
        float(loss_i.item()) if loss_i is not None else 0.0,
        float(cal.item()) if cal is not None else 0.0,
    )


def inbatch_bce_chunked(users: torch.Tensor, positives: torch.Tensor, *, row_base: int = 0,
                        inv_count: float | None = None, chunk: int = 1024,
                        dtype: torch.dtype = torch.float64) -> tuple[float, torch.Tensor, torch.Tensor]:
    """The in-batch block of train_step(in_batch=True) above (ib = u @ p^T, label 1 at
    (b, row_base + b); row_base = 0 and positives = p in one process, a rank's first global
    position and the all-gathered positives in the row-sharded step) evaluated in ``dtype``,
    ``chunk`` users at a time so a [8192 x 65536] score matrix is never held whole.  Returns
    (sum of the BCEWithLogits terms, dL/dusers, dL/dpositives) for L = inv_count * that sum
    (torch's BCE term max(x, 0) - x y + log1p(exp(-|x|)); dL/dS = (sigmoid(S) - Y) inv_count).
    Runs on whatever device the inputs are on (test infrastructure)."""
    u = users.to(dtype)
    p = positives.to(dtype)
    B, Bc = u.shape[0], p.shape[0]
    if inv_count is None:
        inv_count = 1.0 / (B * Bc)
    loss = 0.0
    du = torch.empty_like(u)
    dp = torch.zeros_like(p)
    for lo in range(0, B, chunk):
        hi = min(B, lo + chunk)
        s = u[lo:hi] @ p.t()
        y = torch.zeros_like(s)
        rows = torch.arange(hi - lo, device=s.device)
        y[rows, row_base + lo + rows] = 1.0
        loss += float((s.clamp_min(0) - s * y + torch.log1p(torch.exp(-s.abs()))).sum().item())
        ds = (torch.sigmoid(s) - y) * inv_count
        du[lo:hi] = ds @ p
        dp += ds.t() @ u[lo:hi]
    return loss, du, dp


def train_one_epoch(model, batches: Iterable, optimizers, *, negatives_per_positive: int, num_items: int,
                    positives: Mapping[int, set[int]], user_features, item_features,
                    loss_weights: Mapping[str, float] | None = None, max_steps: int | None = None,
                    item_category_tensor: torch.Tensor | None = None, major_category_id: int | None = None,
                    batch_hook=None, step_losses: list | None = None, in_batch: bool = False,
                    gradient_clip_norm: float | None = None) -> tuple[float, int, float]:
    """training.py:700-833 with the reference's per-row sampler; returns
    (mean loss, interactions, seconds).  ``batch_hook(step, users, pos) -> (negatives | None,
    {"user": masks, "item": masks} | None)`` injects the RNG streams (the same hook ttamm's
    train_one_epoch takes); ``step_losses`` collects each step's StepResult."""
    running, seen, steps = 0.0, 0, 0
    t0 = time.perf_counter()
    for users, pos in batches:
        neg, masks = batch_hook(steps, users, pos) if batch_hook is not None else (None, None)
        if neg is None and negatives_per_positive == 0:
            neg = torch.empty((users.shape[0], 0), dtype=torch.long)
        if neg is None:
            neg = sample_negative_items(users, num_items=num_items, positives=positives,
                                        num_negatives=negatives_per_positive)
        masks = masks or {}
        res = train_step(model, optimizers, users, pos, neg.reshape(users.shape[0], -1), user_features=user_features,
                         item_features=item_features, loss_weights=loss_weights,
                         user_keep_masks=masks.get("user"), item_keep_masks=masks.get("item"),
                         item_category_tensor=item_category_tensor, major_category_id=major_category_id,
                         in_batch=in_batch, gradient_clip_norm=gradient_clip_norm)
        if step_losses is not None:
            step_losses.append(res)
        running += res.total * users.shape[0]
        seen += users.shape[0]
        steps += 1
        if max_steps is not None and steps >= max_steps:
            break
    return running / max(seen, 1), seen, time.perf_counter() - t0


# ---------------------------------------------------------------------------------------
# ranking metrics (src/evaluation/metrics.py:22-116)
# ---------------------------------------------------------------------------------------
def _dcg(rels: Sequence[int]) -> float:
    return float(sum(r / np.log2(i + 2) for i, r in enumerate(rels)))


def user_metrics(predicted: Sequence[int], truth: set[int], ks: Iterable[int]) -> dict[str, float]:
    ks = sorted(ks)
    res: dict[str, float] = {}
    for k in ks:
        head = list(predicted[:k])
        hits = len(set(head) & truth)
        res[f"recall@{k}"] = hits / max(len(truth), 1)
        res[f"precision@{k}"] = hits / max(k, 1)
        res[f"hit_rate@{k}"] = 1.0 if hits else 0.0
        ideal = _dcg([1] * min(k, len(truth)))
        res[f"ndcg@{k}"] = _dcg([1 if x in truth else 0 for x in head]) / ideal if ideal else 0.0
        h, acc = 0, 0.0
        for i, x in enumerate(head, start=1):
            if x in truth:
                h += 1
                acc += h / i
        res[f"map@{k}"] = acc / min(len(truth), k) if truth else 0.0
    rr = 0.0
    for i, x in enumerate(predicted[: (ks[-1] if ks else len(predicted))], start=1):
        if x in truth:
            rr = 1.0 / i
            break
    res["mrr"] = rr
    return res


@dataclass(frozen=True)
class RankingMetrics:
    recall: dict
    precision: dict
    ndcg: dict
    hit_rate: dict
    map: dict
    mrr: float


def ranking_metrics(predictions: Mapping[int, Sequence[int]], truth: Mapping[int, set[int]], ks: Iterable[int]) -> RankingMetrics:
    ks = list(ks)
    acc = {name: {k: [] for k in ks} for name in ("recall", "precision", "ndcg", "hit_rate", "map")}
    mrr = []
    for u, pred in predictions.items():
        gt = truth.get(u, set())
        if not gt:
            continue
        m = user_metrics(pred, gt, ks)
        for name in acc:
            for k in ks:
                acc[name][k].append(m[f"{name}@{k}"])
        mrr.append(m["mrr"])

    def mean(v):
        return float(np.mean(v)) if v else 0.0

    return RankingMetrics(**{name: {k: mean(acc[name][k]) for k in ks} for name in acc}, mrr=mean(mrr))


# ---------------------------------------------------------------------------------------
# evaluation: exact-IP retrieval (training.py:613-679 encode + IndexFlatIP; :917-1043
# _evaluate_model, FAISS branch :944-970)
# ---------------------------------------------------------------------------------------
def encode_item_embeddings(model: OracleModel, *, num_items: int, item_features: torch.Tensor | None,
                           batch_size: int = 8192) -> torch.Tensor:
    """training.py:613-643 (eval mode, no grad; + augment_items when mimic is on)."""
    model.eval()
    out = []
    with torch.no_grad():
        for start in range(0, num_items, batch_size):
            idx = torch.arange(start, min(start + batch_size, num_items), dtype=torch.long)
            feats = item_features.index_select(0, idx) if item_features is not None else None
            emb = tower_forward(model.item_encoder, idx, feats, training=False)
            if model.adaptive_mimic is not None:
                emb = gather_aug(model.adaptive_mimic.item_augmented, idx, emb)[0]
            out.append(emb)
    return torch.cat(out) if out else torch.empty((0, 0))


def flat_ip_search(items: np.ndarray, queries: np.ndarray, k: int) -> tuple[np.ndarray, np.ndarray]:
    """faiss.IndexFlatIP.search: (scores, ids) of the k largest inner products per query, ids -1
    past the corpus size.  FAISS's tie order is unspecified; this restatement breaks ties by
    the lower item id (the order ttamm's kernel implements)."""
    scores = queries.astype(np.float32) @ items.astype(np.float32).T
    nq, ni = scores.shape
    ids = np.full((nq, k), -1, dtype=np.int64)
    out = np.full((nq, k), -np.inf, dtype=np.float32)
    for q in range(nq):
        order = np.lexsort((np.arange(ni), -scores[q]))[:k]  # score desc, then id asc
        ids[q, : order.size] = order
        out[q, : order.size] = scores[q, order]
    return out, ids


def normalize_l2(x: np.ndarray) -> np.ndarray:
    """faiss.normalize_L2 (called at training.py:670-672 on the index matrix and :954-955 on each
    query).  faiss is not installed here (third-party, unpinned by the reference); its published
    algorithm (faiss/utils/distances.cpp fvec_renorm_L2): per row nr = sum x^2 in fp32, and if
    nr > 0 every element is multiplied by the fp32 value of 1 / sqrt(nr).  Returns a new array."""
    x = np.array(x, dtype=np.float32, copy=True)
    nr = np.einsum("ij,ij->i", x.astype(np.float64), x.astype(np.float64)).astype(np.float32)
    root = np.sqrt(np.where(nr > 0, nr, np.float32(1.0)))  # sqrtf, fp32
    inv = np.where(nr > 0, (1.0 / root.astype(np.float64)).astype(np.float32), np.float32(1.0))  # 1.0 / sqrtf(nr)
    x *= inv[:, None]
    return x


def retrieve_with_faiss(items: np.ndarray, user_embedding: np.ndarray, blocked: set[int], ground_truth: set[int],
                        *, max_k: int, faiss_search_k: int) -> list[int]:
    """training.py:944-970 (_retrieve_with_faiss), dot-product index."""
    search_limit = max(max_k + len(ground_truth), 1)
    search_k = max(faiss_search_k, search_limit + len(blocked))
    _, idx = flat_ip_search(items, user_embedding[None, :], search_k)
    filtered: list[int] = []
    seen: set[int] = set()
    for item_id in idx[0].tolist():
        if item_id in blocked or item_id in seen or item_id < 0:
            continue
        filtered.append(int(item_id))
        seen.add(int(item_id))
        if len(filtered) >= search_limit:
            break
    for item_id in ground_truth:
        if item_id not in seen:
            filtered.append(item_id)
    return filtered[:max_k]


def evaluate_model(model: OracleModel, *, train_positive_map: Mapping[int, set[int]],
                   val_pairs: Sequence[tuple[int, int]], item_features: torch.Tensor | None,
                   user_features: torch.Tensor | None, num_items: int, k_values: Iterable[int],
                   faiss_search_k: int = 80, normalize: bool = False
                   ) -> tuple[dict[int, list[int]], dict[int, set[int]]]:
    """training.py:917-1043 with FAISS resources (exact IP over all items): per validation user,
    predictions exclude the user's train positives.  ``normalize``: the model's similarity is
    cosine, so the index and the queries are L2-normalised (:670-672, :954-955)."""
    max_k = max(k_values)
    items = encode_item_embeddings(model, num_items=num_items, item_features=item_features).numpy()
    if normalize:
        items = normalize_l2(items)
    groups: dict[int, list[int]] = {}
    for u, i in val_pairs:
        groups.setdefault(int(u), []).append(int(i))
    preds: dict[int, list[int]] = {}
    truth: dict[int, set[int]] = {}
    with torch.no_grad():
        for u in sorted(groups):  # DataFrame.groupby("user_idx") iterates users in sorted order
            gt = set(groups[u])
            if not gt:
                continue
            truth[u] = gt
            idx = torch.tensor([u], dtype=torch.long)
            feats = user_features.index_select(0, idx) if user_features is not None else None
            emb = tower_forward(model.user_encoder, idx, feats, training=False)
            if model.adaptive_mimic is not None:
                emb = gather_aug(model.adaptive_mimic.user_augmented, idx, emb)[0]
            query = normalize_l2(emb.numpy())[0] if normalize else emb[0].numpy()
            preds[u] = retrieve_with_faiss(items, query, set(train_positive_map.get(u, set())), gt,
                                           max_k=max_k, faiss_search_k=faiss_search_k)
    return preds, truth


def evaluate_model_sampled(model: OracleModel, *, train_positive_map: Mapping[int, set[int]],
                           val_pairs: Sequence[tuple[int, int]], item_features: torch.Tensor | None,
                           user_features: torch.Tensor | None, num_items: int, k_values: Iterable[int],
                           candidate_samples: int, rng: np.random.Generator, cosine: bool = True
                           ) -> tuple[dict[int, list[int]], dict[int, set[int]]]:
    """training.py:917-1043 without FAISS: _retrieve_with_sampling (:974-1009) per validation user,
    users ascending (DataFrame.groupby), the Python set / rng.choice calls as the reference makes
    them; scores by CosineSimilarity of F.normalize'd vectors (cosine model) or the dot product."""
    max_k = max(k_values)
    groups: dict[int, list[int]] = {}
    for u, i in val_pairs:
        groups.setdefault(int(u), []).append(int(i))
    preds: dict[int, list[int]] = {}
    truth: dict[int, set[int]] = {}
    model.eval()
    with torch.no_grad():
        for u in sorted(groups):
            gt = set(groups[u])
            if not gt:
                continue
            truth[u] = gt
            idx = torch.tensor([u], dtype=torch.long)
            feats = user_features.index_select(0, idx) if user_features is not None else None
            ue = tower_forward(model.user_encoder, idx, feats, training=False)
            if model.adaptive_mimic is not None:
                ue = gather_aug(model.adaptive_mimic.user_augmented, idx, ue)[0]
            blocked = set(train_positive_map.get(u, set()))
            candidates = set(gt)
            available = list(set(range(num_items)) - blocked)
            if available:
                budget = max(0, min(candidate_samples, len(available)))
                if budget > 0:
                    candidates.update(int(n) for n in rng.choice(available, size=budget, replace=False).tolist())
            cand = list(candidates)
            ct = torch.tensor(cand, dtype=torch.long)
            cf = item_features.index_select(0, ct) if item_features is not None else None
            ce = tower_forward(model.item_encoder, ct, cf, training=False)
            if model.adaptive_mimic is not None:
                ce = gather_aug(model.adaptive_mimic.item_augmented, ct, ce)[0]
            if cosine:
                scores = F.cosine_similarity(F.normalize(ue, dim=-1), F.normalize(ce, dim=-1), dim=-1)
            else:
                scores = (ue * ce).sum(dim=-1)
            top = torch.topk(scores.reshape(-1), k=min(max_k, len(cand)))
            preds[u] = [cand[i] for i in top.indices.tolist()]
    return preds, truth
