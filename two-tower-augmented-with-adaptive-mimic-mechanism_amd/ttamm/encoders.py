"""Tower encoders — drop-in for the reference's ``src/models/encoders.py``.

Module layout, constructor signatures, parameter initialisation and ``state_dict`` keys
match the reference (encoders.py:19-331) so configs and checkpoints carry over:

    embedding.weight                                   (nn.Embedding, encoders.py:39-65)
    feature_encoder.network.{i}.{weight,bias}          (nn.Sequential MLP, encoders.py:102-146)
    adaptive_mimic.gate_network.{0,2}.{weight,bias}    (FeatureFusionGate, encoders.py:149-168)

``TowerEncoder.forward`` executes on the MI355X through libttamm: in eval mode / under no_grad
``ttamm_tower_forward`` (ID-row gather, MFMA feature MLP and the fusion in fused gfx950 kernels);
under autograd ``ttamm_tower_train_forward`` / ``_backward`` wrapped in a torch.autograd.Function
(ttamm/autograd.py), so the reference's own loop body can call the modules and ``backward()``.
The fast training path is the fused step (``ttamm.training.train_one_epoch``).
"""

from __future__ import annotations

import ctypes
import warnings
from dataclasses import dataclass
from typing import Any, Iterable, Mapping

import torch
from torch import nn

from . import _lib

_FUSIONS = ("identity", "sum", "concat", "gated")
_ACTIVATIONS = {"relu": nn.ReLU, "gelu": nn.GELU, "tanh": nn.Tanh, "selu": nn.SELU}


def _init_embedding(embedding: nn.Embedding, init_config: Mapping[str, Any] | None = None) -> None:
    """Weight init of an ID table (encoders.py:19-36); default N(0, 0.02)."""
    cfg = dict(init_config or {"type": "normal", "std": 0.02})
    kind = str(cfg.get("type", "normal")).lower()
    weight = embedding.weight
    if kind == "normal":
        nn.init.normal_(weight, mean=0.0, std=float(cfg.get("std", 0.02)))
    elif kind == "uniform":
        bound = float(cfg.get("bound", 0.1))
        nn.init.uniform_(weight, -bound, bound)
    elif kind == "xavier_normal":
        nn.init.xavier_normal_(weight)
    elif kind == "xavier_uniform":
        nn.init.xavier_uniform_(weight)
    else:
        raise ValueError(f"Unsupported embedding init type: {kind}")


def build_id_embedding(
    config: Mapping[str, Any],
    *,
    num_embeddings: int,
    device: torch.device | None = None,
) -> nn.Embedding:
    """nn.Embedding from ``{"params": {...}, "init": {...}}`` (encoders.py:39-65)."""
    params = dict(config.get("params", {}) or {})
    sparse = bool(params.get("sparse", False))
    max_norm = params.get("max_norm")
    if sparse and max_norm is not None:
        raise ValueError("max_norm is not supported when using sparse embeddings.")
    table = nn.Embedding(
        num_embeddings=num_embeddings,
        embedding_dim=int(params.get("embedding_dim", 64)),
        padding_idx=params.get("padding_idx"),
        max_norm=max_norm,
        sparse=sparse,
    )
    _init_embedding(table, config.get("init"))
    return table.to(device) if device is not None else table


def _get_activation(name: str) -> nn.Module:
    try:
        return _ACTIVATIONS[name.lower()]()
    except KeyError:
        raise ValueError(f"Unsupported activation '{name}'") from None


class FeatureEncoderWrapper(nn.Module):
    """Projection network plus its output width (encoders.py:81-90)."""

    def __init__(self, network: nn.Module, output_dim: int) -> None:
        super().__init__()
        self.network = network
        self.output_dim = output_dim

    def forward(self, inputs: torch.Tensor) -> torch.Tensor:
        return self.network(inputs)


@dataclass(frozen=True)
class FeatureEncoderConfig:
    type: str = "linear"
    output_dim: int | None = None
    hidden_dims: Iterable[int] | None = None
    activation: str = "relu"
    dropout: float = 0.0


def _xavier_linear(fan_in: int, fan_out: int) -> nn.Linear:
    layer = nn.Linear(fan_in, fan_out)
    nn.init.xavier_uniform_(layer.weight)
    return layer


def build_feature_encoder(
    config: Mapping[str, Any] | None,
    *,
    input_dim: int,
    fallback_output_dim: int,
) -> FeatureEncoderWrapper | None:
    """Feature projection (encoders.py:102-146): identity, linear, or MLP with
    [Linear, activation, (Dropout)] per hidden layer followed by a final Linear."""
    if input_dim == 0:
        return None
    cfg = FeatureEncoderConfig(**(config or {}))
    out_dim = int(cfg.output_dim or fallback_output_dim)
    if cfg.type == "identity":
        if input_dim != out_dim:
            raise ValueError("Identity feature encoder requires input_dim == output_dim.")
        return FeatureEncoderWrapper(nn.Identity(), out_dim)
    if cfg.type == "linear":
        return FeatureEncoderWrapper(_xavier_linear(input_dim, out_dim), out_dim)
    if cfg.type == "mlp":
        activation = _get_activation(cfg.activation)
        modules: list[nn.Module] = []
        width = input_dim
        for hidden in (int(h) for h in (cfg.hidden_dims or [])):
            modules.append(_xavier_linear(width, hidden))
            modules.append(activation)  # one shared activation module, as in the reference
            if cfg.dropout:
                modules.append(nn.Dropout(p=cfg.dropout))
            width = hidden
        modules.append(_xavier_linear(width, out_dim))
        return FeatureEncoderWrapper(nn.Sequential(*modules), out_dim)
    raise ValueError(f"Unsupported feature encoder type: {cfg.type}")


class FeatureFusionGate(nn.Module):
    """g = sigmoid(W2 relu(W1 [e; f] + b1) + b2); out = g*e + (1-g)*f (encoders.py:149-168)."""

    def __init__(self, dim: int, hidden_dim: int | None = None) -> None:
        super().__init__()
        width = hidden_dim or dim
        self.gate_network = nn.Sequential(
            nn.Linear(dim * 2, width),
            nn.ReLU(),
            nn.Linear(width, dim),
            nn.Sigmoid(),
        )

    def forward(self, id_repr: torch.Tensor, feature_repr: torch.Tensor) -> torch.Tensor:
        """gate * id + (1 - gate) * feature (encoders.py:164-168) on the fused gate kernels, with
        autograd to both inputs and the gate's parameters (ttamm/autograd.py gate_forward)."""
        from .autograd import gate_forward

        _lib.require_rocm(id_repr, "FeatureFusionGate")
        shape = id_repr.shape
        out = gate_forward(self, id_repr.reshape(-1, shape[-1]), feature_repr.reshape(-1, shape[-1]))
        return out.reshape(shape)


class TowerEncoder(nn.Module):
    """ID embedding + optional feature encoder + fusion (encoders.py:171-255)."""

    def __init__(
        self,
        *,
        embedding: nn.Embedding,
        feature_encoder: FeatureEncoderWrapper | None,
        fusion: str,
        output_dim: int | None,
        adaptive_mimic: FeatureFusionGate | None,
        matmul_dtype: str = "fp32",
    ) -> None:
        super().__init__()
        self.embedding = embedding
        # ttamm extension (BASELINE config C5, "bf16 towers"): the precision of the
        # feature-MLP / gate GEMMs — "fp32" (the reference) or "bf16" (operands rounded to
        # bf16, fp32 accumulation; ttamm.h ttamm_tower.matmul_bf16)
        self.matmul_dtype = _matmul_dtype(matmul_dtype)
        self.feature_encoder = feature_encoder
        self.adaptive_mimic = adaptive_mimic
        self.num_embeddings = embedding.num_embeddings
        self.id_dim = embedding.embedding_dim
        mode = fusion
        if mode == "adaptive_mimic":
            warnings.warn(
                "TowerEncoder fusion='adaptive_mimic' is deprecated; use fusion='gated' instead.",
                DeprecationWarning,
                stacklevel=2,
            )
            mode = "gated"
        if mode not in _FUSIONS:
            raise ValueError(f"Unsupported fusion strategy: {fusion}")
        self.fusion = "identity" if feature_encoder is None else mode
        self.output_dim = self.id_dim
        if self.fusion == "concat":
            joint = self.id_dim + feature_encoder.output_dim
            self.output_dim = int(output_dim or joint)
            self.projection = _xavier_linear(joint, self.output_dim)

    # -- HIP execution -------------------------------------------------------------------
    def tower_struct(self, features: torch.Tensor | None, feat_ld: int | None = None) -> _lib.Tower:
        """Describe this tower to libttamm (parameters only; see training.py for the
        optimizer-state variant)."""
        return describe_tower(self, features=features, feat_ld=feat_ld)

    def forward(self, inputs: Mapping[str, torch.Tensor]) -> torch.Tensor:
        indices = inputs["indices"]
        features = inputs.get("features")
        return tower_forward(self, indices, features=features)


def build_tower_encoder(
    config: Mapping[str, Any] | None,
    *,
    num_embeddings: int,
    feature_dim: int,
    device: torch.device | None = None,
) -> TowerEncoder:
    """Factory matching encoders.py:258-331 (``type: tower`` or ``type: embedding``)."""
    cfg = dict(config or {})
    kind = str(cfg.get("type", "tower")).lower()
    if kind not in ("tower", "embedding"):
        raise ValueError(f"Unsupported encoder type: {kind}")
    if kind == "embedding":
        table = build_id_embedding(
            {"params": cfg.get("params", {}), "init": cfg.get("init")},
            num_embeddings=num_embeddings,
            device=device,
        )
        return TowerEncoder(
            embedding=table, feature_encoder=None, fusion="identity", output_dim=None, adaptive_mimic=None
        ).to(device)

    id_cfg = cfg.get("id_embedding", {}) or {}
    table = build_id_embedding(
        {"params": id_cfg.get("params", {}), "init": id_cfg.get("init")},
        num_embeddings=num_embeddings,
        device=device,
    )
    fusion = str(cfg.get("fusion", "gated" if feature_dim > 0 else "identity")).lower()
    feature_encoder = build_feature_encoder(
        cfg.get("feature_encoder"), input_dim=feature_dim, fallback_output_dim=table.embedding_dim
    )
    if fusion in ("sum", "adaptive_mimic", "gated") and feature_encoder is not None:
        if feature_encoder.output_dim != table.embedding_dim:
            raise ValueError(
                "Feature encoder output dimension must equal embedding dimension for 'sum' or 'gated' fusion."
            )
    gate = None
    if fusion in ("adaptive_mimic", "gated"):
        gate = FeatureFusionGate(dim=table.embedding_dim, hidden_dim=(cfg.get("adaptive_mimic", {}) or {}).get("hidden_dim"))
    tower = TowerEncoder(
        embedding=table,
        feature_encoder=feature_encoder,
        fusion=fusion,
        output_dim=cfg.get("output_dim"),
        adaptive_mimic=gate,
        matmul_dtype=str(cfg.get("matmul_dtype", "fp32")),
    )
    return tower.to(device) if device is not None else tower


# ---------------------------------------------------------------------------------------
# Mapping of a TowerEncoder onto the libttamm tower descriptor
# ---------------------------------------------------------------------------------------
_FUSION_CODE = {"identity": _lib.FUSION_IDENTITY, "sum": _lib.FUSION_SUM, "gated": _lib.FUSION_GATED,
                "concat": _lib.FUSION_CONCAT}


def _matmul_dtype(name: str) -> str:
    key = str(name).lower()
    if key in ("fp32", "float32", "float"):
        return "fp32"
    if key in ("bf16", "bfloat16"):
        return "bf16"
    raise ValueError(f"Unsupported matmul_dtype: {name} (fp32 or bf16)")


_ACT_CODE = {nn.ReLU: _lib.ACT_RELU, nn.GELU: _lib.ACT_GELU, nn.Tanh: _lib.ACT_TANH, nn.SELU: _lib.ACT_SELU}


def feature_layers(tower: TowerEncoder) -> tuple[list[nn.Linear], float]:
    """The Linear layers of the feature encoder (none for the identity encoder) and its
    dropout p (encoders.py:102-146)."""
    return _feature_net(tower)[:2]


def feature_activation(tower: TowerEncoder) -> int:
    """ttamm.h TTAMM_ACT_* of the feature MLP's hidden layers (encoders.py:68-78, :130)."""
    return _feature_net(tower)[2]


def _feature_net(tower: TowerEncoder) -> tuple[list[nn.Linear], float, int]:
    if tower.feature_encoder is None or tower.fusion == "identity":
        return [], 0.0, _lib.ACT_RELU
    net = tower.feature_encoder.network
    if isinstance(net, nn.Linear):
        return [net], 0.0, _lib.ACT_RELU
    if isinstance(net, nn.Identity):  # encoders.py:114-119: f = the feature row
        return [], 0.0, _lib.ACT_RELU
    if not isinstance(net, nn.Sequential):
        raise NotImplementedError(f"ttamm: feature encoder {type(net).__name__} is not implemented")
    linears: list[nn.Linear] = []
    p = 0.0
    act = _lib.ACT_RELU
    for m in net:
        if isinstance(m, nn.Linear):
            linears.append(m)
        elif isinstance(m, nn.Dropout):
            p = float(m.p)
        elif type(m) in _ACT_CODE:
            if isinstance(m, nn.GELU) and m.approximate != "none":
                raise NotImplementedError("ttamm: GELU(approximate='tanh') is not implemented")
            act = _ACT_CODE[type(m)]
        else:
            raise NotImplementedError(f"ttamm: activation {type(m).__name__} is not implemented")
    if len(linears) > _lib.MAX_LINEAR:
        raise NotImplementedError(f"ttamm: at most {_lib.MAX_LINEAR} feature-encoder layers")
    return linears, p, act


def _linear_struct(layer: nn.Linear, state: Mapping[int, Mapping[str, torch.Tensor]] | None = None) -> _lib.Linear:
    s = _lib.Linear()
    s.weight = layer.weight.data_ptr()
    s.bias = layer.bias.data_ptr()
    s.in_features = layer.in_features
    s.out_features = layer.out_features
    if state is not None:
        sw, sb = state[id(layer.weight)], state[id(layer.bias)]
        s.weight_exp_avg = sw["exp_avg"].data_ptr()
        s.weight_exp_avg_sq = sw["exp_avg_sq"].data_ptr()
        s.bias_exp_avg = sb["exp_avg"].data_ptr()
        s.bias_exp_avg_sq = sb["exp_avg_sq"].data_ptr()
    return s


def describe_tower(
    tower: TowerEncoder,
    *,
    features: torch.Tensor | None,
    feat_ld: int | None = None,
    mimic_table: torch.Tensor | None = None,
    state: Mapping[int, Mapping[str, torch.Tensor]] | None = None,
    id_optimizer: int = _lib.OPT_SPARSE_ADAM,
) -> _lib.Tower:
    if tower.embedding.max_norm is not None and float(tower.embedding.norm_type) != 2.0:
        raise NotImplementedError("ttamm: max_norm embeddings with norm_type != 2")
    s = _lib.Tower()
    emb = tower.embedding.weight
    s.id.weight = emb.data_ptr()
    s.id.rows = emb.shape[0]
    s.id.dim = emb.shape[1]
    s.id.optimizer = id_optimizer
    if tower.embedding.padding_idx is not None:  # nn.Embedding normalises it to [0, rows)
        s.id.has_padding_idx = 1
        s.id.padding_idx = int(tower.embedding.padding_idx)
    if tower.embedding.max_norm is not None:  # renorm of looked-up rows (embedding_renorm_)
        s.id.max_norm = float(tower.embedding.max_norm)
    if state is not None:
        st = state[id(emb)]
        s.id.exp_avg = st["exp_avg"].data_ptr()
        s.id.exp_avg_sq = st["exp_avg_sq"].data_ptr()
    if mimic_table is not None:
        s.mimic.weight = mimic_table.data_ptr()
        s.mimic.rows = mimic_table.shape[0]
        s.mimic.dim = mimic_table.shape[1]
        s.mimic.optimizer = _lib.OPT_DENSE
        if state is not None:
            st = state[id(mimic_table)]
            s.mimic.exp_avg = st["exp_avg"].data_ptr()
            s.mimic.exp_avg_sq = st["exp_avg_sq"].data_ptr()
    s.fusion = _FUSION_CODE[tower.fusion]
    s.matmul_bf16 = 1 if getattr(tower, "matmul_dtype", "fp32") == "bf16" else 0
    linears, p, act = _feature_net(tower)
    if s.fusion != _lib.FUSION_IDENTITY:
        if features is None:
            raise ValueError("ttamm: this tower fuses feature rows; features are required")
        if features.dtype != torch.float32 or features.stride(-1) != 1:
            raise ValueError("ttamm: feature rows must be fp32 with unit column stride")
        s.features = features.data_ptr()
        s.feat_ld = int(feat_ld if feat_ld is not None else features.stride(0))
        s.feat_dim = features.shape[1]
        s.dropout = p
        s.activation = act
        s.n_linear = len(linears)
        for i, layer in enumerate(linears):
            s.linear[i] = _linear_struct(layer, state)
        if tower.fusion == "gated":
            g = tower.adaptive_mimic.gate_network
            s.gate[0] = _linear_struct(g[0], state)
            s.gate[1] = _linear_struct(g[2], state)
        elif tower.fusion == "concat":  # the projection rides in gate[0] (ttamm.h TTAMM_FUSION_CONCAT)
            s.gate[0] = _linear_struct(tower.projection, state)
    return s


def tower_forward(
    tower: TowerEncoder,
    indices: torch.Tensor,
    *,
    features: torch.Tensor | None,
    mimic_table: torch.Tensor | None = None,
) -> torch.Tensor:
    """TowerEncoder.forward on the MI355X (encoders.py:221-255); optionally adds the mimic rows
    (AdaptiveMimicMechanism._apply_aug, adaptive_mimic.py:88-95).  Under autograd (a parameter
    requires grad) or in train mode with dropout, the training forward runs (ttamm/autograd.py:
    activations kept for the backward, the mimic rows added with their table gradient)."""
    _lib.require_rocm(indices, "TowerEncoder.forward")
    if indices.dtype != torch.long:
        raise ValueError("ttamm: indices must be torch.long")
    if features is not None and tower.fusion == "identity":
        features = None
    use_features = tower.fusion != "identity" and features is not None
    idx = indices.reshape(-1).contiguous()
    _lib.check_index_range(idx, tower.num_embeddings)
    n = idx.numel()
    train = (torch.is_grad_enabled() and any(p.requires_grad for p in tower.parameters())) or \
        (tower.training and feature_layers(tower)[1] > 0)
    if train:
        from .autograd import ApplyAugFunction, tower_train_forward

        feats = None
        if use_features:
            feats = features.reshape(-1, features.shape[-1])
            if feats.shape[0] != n:
                raise ValueError("ttamm: features must have one row per index")
        out = tower_train_forward(tower, idx, feats)
        if mimic_table is not None:  # + table[idx] with the table's gradient (adaptive_mimic.py:88-95)
            if mimic_table.shape[1] != out.shape[-1]:
                raise ValueError("Adaptive mimic requires user and item embedding dimensions to match.")
            out, _ = ApplyAugFunction.apply(mimic_table, idx, out.contiguous())
        return out.reshape(*indices.shape, out.shape[-1])
    out = torch.empty((n, tower.output_dim if use_features else tower.id_dim), dtype=torch.float32, device=idx.device)
    if not use_features and tower.fusion != "identity":
        # the reference falls back to the ID embedding when features are absent (encoders.py:228-231)
        lib = _lib.load()
        _lib.check(
            lib.ttamm_gather_rows(
                tower.embedding.weight.data_ptr(), tower.num_embeddings, tower.id_dim, idx.data_ptr(), n,
                out.data_ptr(), tower.id_dim, _lib.stream_handle(idx.device),
            )
        )
        if mimic_table is not None:
            _lib.check(
                lib.ttamm_mimic_augment(
                    mimic_table.data_ptr(), mimic_table.shape[0], tower.id_dim, idx.data_ptr(), n, out.data_ptr(),
                    out.data_ptr(), None, _lib.stream_handle(idx.device),
                )
            )
        return out.reshape(*indices.shape, tower.id_dim)
    feats = None
    if use_features:
        feats = features.reshape(-1, features.shape[-1])
        if feats.dtype != torch.float32:
            raise ValueError("ttamm: features must be float32")
        if feats.stride(-1) != 1 or feats.stride(0) % 4 or feats.data_ptr() % 16:
            width = feats.shape[1]
            padded = torch.zeros((feats.shape[0], (width + 3) // 4 * 4), dtype=torch.float32, device=feats.device)
            padded[:, :width].copy_(feats)
            feats = padded[:, :width]
        if feats.shape[0] != n:
            raise ValueError("ttamm: features must have one row per index")
    desc = describe_tower(tower, features=feats, mimic_table=mimic_table)
    lib = _lib.load()
    ws_bytes = lib.ttamm_tower_forward_workspace_size(ctypes.byref(desc), n)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=idx.device)
    _lib.check(
        lib.ttamm_tower_forward(
            ctypes.byref(desc), idx.data_ptr(), None, n, 1 if mimic_table is not None else 0, out.data_ptr(),
            ws.data_ptr(), ws_bytes, _lib.stream_handle(idx.device),
        )
    )
    return out.reshape(*indices.shape, out.shape[-1])
