"""Shared builders for parity tests: the same model/optimizers/inputs on the CPU oracle and
on ttamm (MI355X)."""

from __future__ import annotations

import copy
from dataclasses import dataclass, field

import numpy as np
import torch

from oracle import cpu_reference as ref


@dataclass
class Shape:
    U: int = 64
    I: int = 256
    F: int = 12
    H: int = 16
    D: int = 8
    B: int = 32
    N: int = 5
    dropout: float = 0.15
    gate_hidden: int | None = None
    mimic: bool = True
    sparse: bool = True
    hidden_dims: tuple = (16,)
    matmul_dtype: str = "fp32"
    padding_idx: int | None = None  # nn.Embedding padding_idx of both ID tables (encoders.py:47)
    fusion: str = "gated"  # TowerEncoder fusion (encoders.py:203): gated / sum / concat
    max_norm: float | None = None  # nn.Embedding max_norm of both ID tables (dense only, encoders.py:48-52)
    activation: str = "relu"  # feature-MLP activation (encoders.py:68-78)
    feature_type: str = "mlp"  # feature encoder type (encoders.py:114-144): mlp / linear / identity (F == D)
    feature_out: int | None = None  # feature encoder output_dim (None: D)
    concat_out: int | None = -1  # concat output_dim: -1 = D, None = the reference default D + feature_out

    @property
    def P(self) -> int:
        """The tower output width (encoders.py:211-219): the mimic tables and scores are this wide."""
        if self.fusion != "concat":
            return self.D
        fo = self.feature_out or self.D
        return self.D + fo if self.concat_out is None else (self.D if self.concat_out == -1 else self.concat_out)

    def tower_cfg(self) -> dict:
        params = {"embedding_dim": self.D, "sparse": self.sparse}
        if self.padding_idx is not None:
            params["padding_idx"] = self.padding_idx
        if self.max_norm is not None:
            params["max_norm"] = self.max_norm
        return {
            "type": "tower",
            "matmul_dtype": self.matmul_dtype,
            "id_embedding": {"params": params, "init": {"type": "normal", "std": 0.02}},
            "feature_encoder": {"type": self.feature_type, "hidden_dims": list(self.hidden_dims),
                                "activation": self.activation, "output_dim": self.feature_out or self.D,
                                "dropout": self.dropout},
            "fusion": self.fusion,
            # the concat projection's width (encoders.py:211-212; None = embedding + feature width)
            "output_dim": self.D if self.concat_out == -1 else self.concat_out,
            "adaptive_mimic": {"hidden_dim": self.gate_hidden} if self.gate_hidden else {},
        }


LOSS_WEIGHTS = {"mimic_user": 0.15, "mimic_item": 0.15, "category_alignment": 0.01}


def synthetic_features(n: int, F: int, gen: torch.Generator) -> torch.Tensor:
    """Item-feature rows shaped like features.py:195-266: category weights {1, .5, .333},
    one author one-hot, and N(0,1) numeric columns."""
    x = torch.zeros((n, F), dtype=torch.float32)
    ncat = max(1, (F - 5) // 2)
    nauth = max(1, F - 5 - ncat)
    for w in (1.0, 0.5, 1.0 / 3.0):
        cols = torch.randint(0, ncat, (n,), generator=gen)
        x[torch.arange(n), cols] = torch.maximum(x[torch.arange(n), cols], torch.tensor(w))
    a = torch.randint(0, nauth, (n,), generator=gen)
    x[torch.arange(n), ncat + a] = 1.0
    x[:, ncat + nauth:] = torch.randn((n, F - ncat - nauth), generator=gen)
    return x


@dataclass
class Problem:
    shape: Shape
    model: ref.OracleModel
    user_features: torch.Tensor
    item_features: torch.Tensor
    positives: dict
    batches: list = field(default_factory=list)  # (users, pos, neg, user_masks, item_masks)


def make_problem(shape: Shape, *, seed: int = 1234, steps: int = 1, positives_per_user: int = 4) -> Problem:
    torch.manual_seed(seed)
    gen = torch.Generator().manual_seed(seed + 1)
    item_features = synthetic_features(shape.I, shape.F, gen)
    positives: dict[int, set[int]] = {}
    for u in range(shape.U):
        positives[u] = set(torch.randint(0, shape.I, (positives_per_user,), generator=gen).tolist())
    user_features = torch.zeros((shape.U, shape.F), dtype=torch.float32)
    for u, items in positives.items():
        user_features[u] = item_features[sorted(items)].mean(dim=0)
    model = ref.build_model(shape.tower_cfg(), num_users=shape.U, num_items=shape.I,
                            user_feature_dim=shape.F, item_feature_dim=shape.F, mimic=shape.mimic)
    prob = Problem(shape, model, user_features, item_features, positives)
    for _ in range(steps):
        users = torch.randint(0, shape.U, (shape.B,), generator=gen)
        pos = torch.tensor([sorted(positives[int(u)])[0] for u in users], dtype=torch.long)
        neg = torch.randint(0, shape.I, (shape.B, shape.N), generator=gen)
        if shape.padding_idx is not None:  # the padding id occurs among users, positives and negatives
            users[:3] = shape.padding_idx
            pos[3] = shape.padding_idx
            neg[:2, :2] = shape.padding_idx
        nh = len(shape.hidden_dims) if shape.feature_type == "mlp" else 0
        um = [(torch.rand((shape.B, h), generator=gen) >= shape.dropout).to(torch.uint8) for h in shape.hidden_dims][:nh]
        im = [(torch.rand((shape.B * (1 + shape.N), h), generator=gen) >= shape.dropout).to(torch.uint8)
              for h in shape.hidden_dims][:nh]
        prob.batches.append((users, pos, neg, um, im))
    return prob


def clone_model(model):
    return copy.deepcopy(model)


def run_oracle(prob: Problem, *, lr=1e-3, betas=(0.9, 0.999), weight_decay=0.01, steps=None, model=None,
               gradient_clip_norm=None, optimizer="adamw", momentum=0.0):
    model = model if model is not None else clone_model(prob.model)
    opts = ref.build_optimizers(model, lr=lr or 1e-3, betas=betas, weight_decay=weight_decay, optimizer=optimizer,
                                momentum=momentum)
    set_lr(opts, lr)
    results = []
    for (users, pos, neg, um, im) in prob.batches[: steps or len(prob.batches)]:
        results.append(ref.train_step(model, opts, users, pos, neg, user_features=prob.user_features,
                                      item_features=prob.item_features, loss_weights=LOSS_WEIGHTS,
                                      user_keep_masks=um, item_keep_masks=im, gradient_clip_norm=gradient_clip_norm))
    return model, opts, results


def set_lr(opts, lr: float) -> None:
    """SparseAdam rejects lr = 0 at construction; the grad-export tests set it afterwards."""
    for opt in opts:
        for g in opt.param_groups:
            g["lr"] = lr


def named_optimizer_state(model, opts) -> dict[str, dict[str, torch.Tensor]]:
    """{param name: {exp_avg, exp_avg_sq}} across the optimizers."""
    by_id = {id(p): n for n, p in model.named_parameters()}
    out = {}
    for opt in opts:
        for p, st in opt.state.items():
            out[by_id[id(p)]] = {k: (v.detach().cpu().clone() if torch.is_tensor(v) else v) for k, v in st.items()}
    return out


def rel_err(a: torch.Tensor, b: torch.Tensor) -> float:
    """Norm-wise relative error max|a-b| / max|b| (the tolerance definition used by the
    parity tests; 0 when both are zero)."""
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    den = b.abs().max().item()
    num = (a - b).abs().max().item()
    if den == 0:
        return num
    return num / den
