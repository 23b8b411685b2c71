"""Adaptive mimic mechanism — drop-in for ``src/models/adaptive_mimic.py``.

Same parameters (``user_augmented.weight``, ``item_augmented.weight``), same init and the
same error conventions (adaptive_mimic.py:20-105).  The row gathers, the augmentation add
and the MSE reductions run on the MI355X through libttamm, with autograd (ttamm/autograd.py:
the dense table gradients by ttamm_scatter_add_rows) when the reference's own loop calls the
module.  Inside ``ttamm.train_one_epoch`` the whole mechanism (gather, add, stop-grad MSE,
gradients, full-table AdamW) is fused into the step instead (``ttamm_train_step``).
"""

from __future__ import annotations

from typing import Optional, Tuple

import torch
from torch import nn

from . import _lib


class AdaptiveMimicMechanism(nn.Module):
    """Per-user / per-item augmentation tables nudged toward the opposite tower."""

    def __init__(self, *, num_users: int, num_items: int, embedding_dim: int, init_std: float = 0.02) -> None:
        super().__init__()
        if num_users <= 0 or num_items <= 0:
            raise ValueError("num_users and num_items must be positive.")
        self.embedding_dim = int(embedding_dim)
        self.user_augmented = nn.Embedding(num_users, self.embedding_dim)
        self.item_augmented = nn.Embedding(num_items, self.embedding_dim)
        for table in (self.user_augmented, self.item_augmented):
            nn.init.normal_(table.weight, mean=0.0, std=init_std)

    def forward(
        self,
        *,
        user_indices: torch.Tensor | None,
        item_indices: torch.Tensor | None,
        user_embedding: torch.Tensor,
        item_embedding: torch.Tensor,
    ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor | None, torch.Tensor | None]:
        """(augmented_user, augmented_item, mimic_user_loss, mimic_item_loss) — adaptive_mimic.py:40-68."""
        if user_indices is None or item_indices is None:
            raise ValueError("user_indices and item_indices are required for mimic.")
        aug_user, user_rows = self._apply_aug(self.user_augmented, user_indices, user_embedding)
        aug_item, item_rows = self._apply_aug(self.item_augmented, item_indices, item_embedding)
        loss_u = _mse(user_rows, item_embedding.detach())
        loss_i = _mse(item_rows, user_embedding.detach())
        return aug_user, aug_item, loss_u, loss_i

    def augment_users(self, indices: Optional[torch.Tensor], base_embedding: torch.Tensor) -> torch.Tensor:
        if indices is None:
            return base_embedding
        return self._apply_aug(self.user_augmented, indices, base_embedding)[0]

    def augment_items(self, indices: Optional[torch.Tensor], base_embedding: torch.Tensor) -> torch.Tensor:
        if indices is None:
            return base_embedding
        return self._apply_aug(self.item_augmented, indices, base_embedding)[0]

    def _apply_aug(
        self, table: nn.Embedding, indices: torch.Tensor, reference: torch.Tensor
    ) -> Tuple[torch.Tensor, torch.Tensor]:
        """(reference + table[indices], table[indices]) — adaptive_mimic.py:88-105."""
        if indices.dtype != torch.long:
            raise ValueError("Adaptive mimic indices must be torch.long tensors.")
        _lib.require_rocm(reference, "AdaptiveMimicMechanism")
        flat = indices.reshape(-1).contiguous()
        _lib.check_index_range(flat, table.num_embeddings)
        base = reference.reshape(flat.numel(), -1)
        if base.shape[1] != self.embedding_dim:
            raise ValueError("Adaptive mimic: embedding width does not match the augmentation tables.")
        base = base.contiguous()
        if torch.is_grad_enabled() and (table.weight.requires_grad or reference.requires_grad):
            from .autograd import ApplyAugFunction

            out, rows = ApplyAugFunction.apply(table.weight, flat, base)
            return out.reshape(reference.shape), rows.reshape(reference.shape)
        out = torch.empty_like(base)
        rows = torch.empty_like(base)
        lib = _lib.load()
        _lib.check(
            lib.ttamm_mimic_augment(
                table.weight.data_ptr(), table.num_embeddings, self.embedding_dim, flat.data_ptr(), flat.numel(),
                base.data_ptr(), out.data_ptr(), rows.data_ptr(), _lib.stream_handle(base.device),
            )
        )
        return out.reshape(reference.shape), rows.reshape(reference.shape)


def _mse(x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """F.mse_loss(x, y), reduction 'mean' (y is detached by the callers, adaptive_mimic.py:66-67;
    a y that requires grad gets its gradient as in F.mse_loss)."""
    xs, ys = x.contiguous(), y.contiguous()
    if xs.shape != ys.shape:
        raise ValueError("ttamm: mse_loss input and target shapes differ")
    if torch.is_grad_enabled() and (xs.requires_grad or ys.requires_grad):
        from .autograd import MSEFunction

        return MSEFunction.apply(xs.reshape(xs.shape[0], -1), ys.reshape(ys.shape[0], -1))
    out = torch.empty((), dtype=torch.float32, device=x.device)
    _lib.check(_lib.load().ttamm_mse_loss(xs.data_ptr(), ys.data_ptr(), xs.numel(), out.data_ptr(),
                                          _lib.stream_handle(x.device)))
    return out
