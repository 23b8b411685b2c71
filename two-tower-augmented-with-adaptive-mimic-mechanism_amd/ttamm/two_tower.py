"""Two-tower container — drop-in for ``src/models/two_tower.py`` (two_tower.py:19-95)."""

from __future__ import annotations

from typing import Any

import torch
from torch import nn

from .adaptive_mimic import AdaptiveMimicMechanism


class TwoTowerModel(nn.Module):
    """Holds the user/item towers, the similarity module and the mimic module.  Parameter
    names (``user_encoder.*``, ``item_encoder.*``, ``adaptive_mimic.*``) match the reference."""

    def __init__(
        self,
        user_encoder: nn.Module,
        item_encoder: nn.Module,
        similarity: nn.Module | None = None,
        adaptive_mimic: AdaptiveMimicMechanism | None = None,
    ) -> None:
        super().__init__()
        self.user_encoder = user_encoder
        self.item_encoder = item_encoder
        self.similarity = similarity or nn.CosineSimilarity(dim=-1)
        self.adaptive_mimic = adaptive_mimic

    def forward(self, user_inputs: Any, item_inputs: Any, *, return_embeddings: bool = False) -> dict[str, torch.Tensor]:
        users = self.user_encoder(user_inputs)
        items = self.item_encoder(item_inputs)
        out: dict[str, torch.Tensor] = {}
        if self.adaptive_mimic is not None:
            users, items, loss_u, loss_i = self.adaptive_mimic(
                user_indices=_extract_indices(user_inputs),
                item_indices=_extract_indices(item_inputs),
                user_embedding=users,
                item_embedding=items,
            )
            if loss_u is not None:
                out["mimic_user_loss"] = loss_u
            if loss_i is not None:
                out["mimic_item_loss"] = loss_i
        if return_embeddings:
            out["user_embedding"] = users
            out["item_embedding"] = items
        out["score"] = self.similarity(users, items)
        return out


def _extract_indices(inputs: Any) -> torch.Tensor | None:
    if isinstance(inputs, torch.Tensor):
        return inputs
    if isinstance(inputs, dict) and isinstance(inputs.get("indices"), torch.Tensor):
        return inputs["indices"]
    return None
