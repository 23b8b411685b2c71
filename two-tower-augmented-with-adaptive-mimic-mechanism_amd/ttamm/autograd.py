"""Module-level autograd for the drop-in classes (SURVEY.md §8 b: "torch.autograd.Function per
op, for module-level parity").

With these, the reference's own loop body (training.py:741-827) runs unchanged on ttamm's
modules — ``model.user_encoder(...)``, ``model.adaptive_mimic(...)``, ``loss.backward()``, the
caller's torch optimizers — and every forward and backward of the towers and the mimic tables
executes in libttamm's gfx950 kernels:

  * ``TowerFunction``: TowerEncoder.forward in training mode (encoders.py:221-255).  Forward:
    ``ttamm_tower_train_forward`` (ID-row gather, MFMA feature MLP with its activation and
    dropout, fusion), keeping the activations in a workspace tensor held by the autograd graph.
    Backward: ``ttamm_tower_train_backward`` (gate / projection, dgrad chain, one grouped
    weight-gradient launch) into a gradient arena whose pieces are returned as the Linear
    layers' ``.grad``; the ID table's gradient is nn.Embedding's — a sparse COO tensor of the
    per-position rows (sparse=True; the padding row dropped) or their dense sum (sparse=False,
    ``ttamm_scatter_add_rows``).
  * ``ApplyAugFunction``: AdaptiveMimicMechanism._apply_aug (adaptive_mimic.py:88-105):
    (base + table[idx], table[idx]); the dense table gradient is the scatter-add of both outputs'
    gradients (the table is a dense nn.Embedding in the AdamW group, training.py:306-307).
  * ``MSEFunction``: F.mse_loss(rows, target.detach()) (adaptive_mimic.py:66-67).

The fused step (``ttamm.train_one_epoch`` / ``FusedTrainStep``) remains the fast path: it never
materialises ``.grad`` or a dense table gradient.  This path exists so code written against the
reference's modules trains on the MI355X as written."""

from __future__ import annotations

import ctypes
from typing import Sequence

import torch
from torch import nn

from . import _lib


def _ptr(t: torch.Tensor | None):
    return ctypes.c_void_p(t.data_ptr()) if t is not None and t.numel() else None


def _padded_rows(feats: torch.Tensor) -> torch.Tensor:
    """fp32 rows with a 16-byte aligned row stride (a copy only when needed)."""
    if feats.dtype != torch.float32:
        raise ValueError("ttamm: features must be float32")
    if feats.stride(-1) == 1 and feats.stride(0) % 4 == 0 and feats.data_ptr() % 16 == 0:
        return feats
    width = feats.shape[1]
    padded = torch.zeros((feats.shape[0], (width + 3) // 4 * 4), dtype=torch.float32, device=feats.device)
    padded[:, :width].copy_(feats)
    return padded[:, :width]


def tower_params(tower) -> list[nn.Parameter]:
    """The parameters a tower's training forward reads, in the gradient arena's order after the
    ID table: each feature Linear's weight and bias, then the gate's two Linear (or the concat
    projection)."""
    from .encoders import feature_layers

    out: list[nn.Parameter] = [tower.embedding.weight]
    if tower.fusion == "identity":
        return out
    for layer in feature_layers(tower)[0]:
        out += [layer.weight, layer.bias]
    if tower.fusion == "gated":
        g = tower.adaptive_mimic.gate_network
        out += [g[0].weight, g[0].bias, g[2].weight, g[2].bias]
    elif tower.fusion == "concat":
        out += [tower.projection.weight, tower.projection.bias]
    return out


class _TowerRun:
    """One training forward of a tower: its descriptor, rows, workspace and dropout stream."""

    def __init__(self, tower, idx: torch.Tensor, feats: torch.Tensor | None, seed: int, counter: int,
                 keep_masks: Sequence[torch.Tensor] | None, feature_grad: bool = False) -> None:
        from .encoders import describe_tower

        self.tower = tower
        self.idx = idx
        self.feats = feats
        self.desc = describe_tower(tower, features=feats)
        self.lib = _lib.load()
        n = idx.numel()
        self.n = n
        self.ws = torch.empty(max(1, int(self.lib.ttamm_tower_train_workspace_size(ctypes.byref(self.desc), n))),
                              dtype=torch.uint8, device=idx.device)
        self.masks = list(keep_masks or [])
        arr = (ctypes.c_void_p * max(1, _lib.MAX_LINEAR))()
        for i, m in enumerate(self.masks[: _lib.MAX_LINEAR]):
            arr[i] = m.data_ptr() if m is not None else None
        self._mask_keep = arr
        self.mask_arr = ctypes.cast(arr, ctypes.c_void_p) if self.masks else None
        self.seed, self.counter = seed, counter
        self.feature_grad = feature_grad

    def forward(self) -> torch.Tensor:
        D = getattr(self.tower, "output_dim", self.tower.id_dim)  # concat: the projection's width
        out = torch.empty((self.n, D), dtype=torch.float32, device=self.idx.device)
        _lib.check(self.lib.ttamm_tower_train_forward(
            ctypes.byref(self.desc), _ptr(self.idx), None, self.n, self.mask_arr, self.seed, self.counter,
            _ptr(out), _ptr(self.ws), self.ws.numel(), _lib.stream_handle(self.idx.device)))
        return out

    def backward(self, d_out: torch.Tensor) -> tuple[torch.Tensor | None, ...]:
        tower = self.tower
        D = tower.id_dim
        fo = self.feats.shape[1] if self.feature_grad else 0  # identity feature encoder: F wide
        dev = self.idx.device
        params = tower_params(tower)
        n_arena = int(self.lib.ttamm_tower_grad_floats(ctypes.byref(self.desc)))
        arena = torch.empty(max(1, n_arena), dtype=torch.float32, device=dev)
        d_rows = torch.empty((self.n, D), dtype=torch.float32, device=dev)
        d_feat = torch.empty((self.n, fo), dtype=torch.float32, device=dev) if self.feature_grad else None
        _lib.check(self.lib.ttamm_tower_train_backward(
            ctypes.byref(self.desc), _ptr(self.idx), None, self.n, self.mask_arr, _ptr(d_out), _ptr(arena),
            _ptr(d_rows), _ptr(d_feat), _ptr(self.ws), self.ws.numel(), _lib.stream_handle(dev)))
        grads: list[torch.Tensor | None] = [self._id_grad(d_rows)]
        off = 0
        for p in params[1:]:  # arena pieces start at multiples of 64 floats (ttamm.h)
            k = p.numel()
            grads.append(arena[off:off + k].view_as(p))
            off += (k + 63) // 64 * 64
        self.d_feat = d_feat
        return tuple(grads)

    def _id_grad(self, d_rows: torch.Tensor) -> torch.Tensor:
        emb = self.tower.embedding
        pad = emb.padding_idx
        if emb.sparse:  # torch embedding_sparse_backward: uncoalesced rows, the padding row dropped
            idx, vals = self.idx, d_rows
            if pad is not None:
                keep = idx != pad
                idx, vals = idx[keep], vals[keep]
            return torch.sparse_coo_tensor(idx.unsqueeze(0), vals, emb.weight.shape)
        grad = torch.zeros_like(emb.weight)
        _lib.check(self.lib.ttamm_scatter_add_rows(
            _ptr(grad), grad.shape[0], grad.shape[1], _ptr(self.idx), self.n, _ptr(d_rows), d_rows.shape[1], None, 0,
            None, 1.0, int(pad) if pad is not None else -1, _lib.stream_handle(grad.device)))
        return grad


class TowerFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, run: _TowerRun, *params: torch.Tensor) -> torch.Tensor:  # noqa: D401
        ctx.run = run
        return run.forward()

    @staticmethod
    def backward(ctx, d_out: torch.Tensor):
        grads = ctx.run.backward(d_out.contiguous())
        ctx.run = None  # the workspace goes with the graph
        return (None, *grads)


def tower_train_forward(tower, idx: torch.Tensor, features: torch.Tensor | None, *,
                        keep_masks: Sequence[torch.Tensor] | None = None) -> torch.Tensor:
    """TowerEncoder.forward in training mode with autograd (encoders.py:221-255).  Dropout draws
    from a Philox stream keyed by a seed from torch's global generator (reproducible under
    torch.manual_seed); ``keep_masks`` (uint8 [n, out] per hidden layer)
    injects them instead (parity tests)."""
    from .samplers import draw_seed
    from .training import _IdentityView

    view = tower
    if tower.fusion == "identity" or features is None:  # the ID lookup only (encoders.py:225-231)
        view, features = _IdentityView(tower), None
    elif not tower.training or feature_dropout(tower) == 0.0:
        keep_masks = None
    if features is not None:
        features = _padded_rows(features)
    drop = tower.training and features is not None and feature_dropout(tower) > 0
    # every call draws a fresh seed, so the Philox counter stays 0: the stream is then a pure
    # function of torch's seeded generator (two runs under one manual_seed agree bit for bit)
    seed = draw_seed() if drop and not keep_masks else 0
    run = _TowerRun(view, idx, features, seed, 0, keep_masks)
    if not drop:  # eval mode: nn.Dropout is the identity
        run.desc.dropout = 0.0
    return TowerFunction.apply(run, *tower_params(view))


def feature_dropout(tower) -> float:
    from .encoders import feature_layers

    return feature_layers(tower)[1]


class _GateRun(_TowerRun):
    """FeatureFusionGate.forward on given rows: a gated tower whose "ID table" is id_repr and
    whose identity feature encoder reads feature_repr (the rows' own positions)."""

    def __init__(self, gate, id_repr: torch.Tensor, feature_repr: torch.Tensor) -> None:
        from .encoders import FeatureEncoderWrapper, TowerEncoder

        n, D = id_repr.shape
        emb = nn.Embedding(n, D, _weight=id_repr.detach(), _freeze=True)
        view = TowerEncoder(embedding=emb, feature_encoder=FeatureEncoderWrapper(nn.Identity(), D), fusion="gated",
                            output_dim=None, adaptive_mimic=gate)
        idx = torch.arange(n, device=id_repr.device)
        super().__init__(view, idx, _padded_rows(feature_repr.detach()), 0, 0, None, feature_grad=True)


class GateFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, run: _GateRun, id_repr, feature_repr, *gate_params):  # noqa: D401
        ctx.run = run
        return run.forward()

    @staticmethod
    def backward(ctx, d_out: torch.Tensor):
        run = ctx.run
        grads = run.backward(d_out.contiguous())
        ctx.run = None
        # grads[0] is the "ID table" gradient: with one position per row it is d(id_repr) itself
        d_id = grads[0].to_dense() if grads[0].is_sparse else grads[0]
        return (None, d_id, run.d_feat, *grads[1:])


def gate_forward(gate, id_repr: torch.Tensor, feature_repr: torch.Tensor) -> torch.Tensor:
    """FeatureFusionGate.forward (encoders.py:164-168) through the fused gate kernels."""
    if id_repr.shape != feature_repr.shape or id_repr.dim() != 2:
        raise ValueError("ttamm: FeatureFusionGate takes two [n, dim] tensors of the same shape")
    run = _GateRun(gate, id_repr.contiguous(), feature_repr)
    g = gate.gate_network
    return GateFunction.apply(run, id_repr, feature_repr, g[0].weight, g[0].bias, g[2].weight, g[2].bias)


# ---- adaptive mimic (adaptive_mimic.py:88-105, :66-67) -------------------------------------
class ApplyAugFunction(torch.autograd.Function):
    """(base + table[idx], table[idx]) with the dense table gradient."""

    @staticmethod
    def forward(ctx, table: torch.Tensor, idx: torch.Tensor, base: torch.Tensor):  # noqa: D401
        out = torch.empty_like(base)
        rows = torch.empty_like(base)
        lib = _lib.load()
        _lib.check(lib.ttamm_mimic_augment(_ptr(table), table.shape[0], table.shape[1], _ptr(idx), idx.numel(),
                                           _ptr(base), _ptr(out), _ptr(rows), _lib.stream_handle(base.device)))
        ctx.save_for_backward(idx)
        ctx.table_shape = table.shape
        return out, rows

    @staticmethod
    def backward(ctx, d_out: torch.Tensor | None, d_rows: torch.Tensor | None):
        (idx,) = ctx.saved_tensors
        lib = _lib.load()
        d_table = None
        if ctx.needs_input_grad[0]:
            ref = d_out if d_out is not None else d_rows
            d_table = torch.zeros(ctx.table_shape, dtype=torch.float32, device=ref.device)
            for g in (d_out, d_rows):
                if g is None:
                    continue
                g = g.contiguous()
                _lib.check(lib.ttamm_scatter_add_rows(_ptr(d_table), d_table.shape[0], d_table.shape[1], _ptr(idx),
                                                      idx.numel(), _ptr(g), g.shape[1], None, 0, None, 1.0, -1,
                                                      _lib.stream_handle(g.device)))
        return d_table, None, d_out


class MSEFunction(torch.autograd.Function):
    """F.mse_loss(x, target) (reduction 'mean').  The reference detaches the target
    (adaptive_mimic.py:66-67); a target that requires grad gets -dx, as F.mse_loss gives it."""

    @staticmethod
    def forward(ctx, x: torch.Tensor, target: torch.Tensor):  # noqa: D401
        out = torch.empty((), dtype=torch.float32, device=x.device)
        _lib.check(_lib.load().ttamm_mse_loss(_ptr(x), _ptr(target), x.numel(), _ptr(out),
                                              _lib.stream_handle(x.device)))
        ctx.save_for_backward(x, target)
        return out

    @staticmethod
    def backward(ctx, d_loss: torch.Tensor):
        x, target = ctx.saved_tensors
        n, D = x.shape
        dx = torch.zeros_like(x)
        dl = d_loss.contiguous()
        # dx = 2 / numel * (x - target) * dL (idx = NULL: row r into row r)
        _lib.check(_lib.load().ttamm_scatter_add_rows(_ptr(dx), n, D, None, n, _ptr(x), D, _ptr(target), D, _ptr(dl),
                                                      2.0 / x.numel(), -1, _lib.stream_handle(x.device)))
        return (dx if ctx.needs_input_grad[0] else None), (-dx if ctx.needs_input_grad[1] else None)
