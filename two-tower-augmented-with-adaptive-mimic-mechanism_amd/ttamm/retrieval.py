"""Exact inner-product retrieval on the MI355X — drop-in for the FAISS branch of
the reference's evaluation: ``_encode_item_embeddings`` (training.py:613-643), the
``IndexFlatIP`` index (:645-679) and ``_evaluate_model``'s search + filter (:917-1043,
:944-970).

The item matrix stays in HBM; ``retrieve_topk`` runs ``ttamm_retrieval_topk`` (fp32 MFMA scores
fused with a per-query top-k that skips each user's blocked train positives), so there is no
per-user search call and no host round trip per user.
"""

from __future__ import annotations

import ctypes
from typing import Any, Iterable, Mapping, Sequence

import torch
from torch import nn

from . import _lib
from .encoders import TowerEncoder, describe_tower
from .training import _pad_features


def _encode(tower: TowerEncoder, mimic_table: torch.Tensor | None, rows: torch.Tensor,
            features: torch.Tensor | None, chunk: int) -> torch.Tensor:
    """TowerEncoder.forward (eval) + augment for `rows`, reading feature row r of the FULL
    feature matrix by index (no gathered copy)."""
    lib = _lib.load()
    dev = rows.device
    n = rows.numel()
    D = tower.id_dim
    out = torch.empty((n, D), dtype=torch.float32, device=dev)
    if n == 0:
        return out
    _lib.check_index_range(rows, tower.num_embeddings)
    feats = _pad_features(features) if tower.fusion != "identity" else None
    if tower.fusion != "identity" and feats is None:
        # no features: the reference falls back to the ID embedding (encoders.py:228-231)
        _lib.check(lib.ttamm_gather_rows(tower.embedding.weight.data_ptr(), tower.num_embeddings, D, rows.data_ptr(),
                                         n, out.data_ptr(), D, _lib.stream_handle(dev)))
        if mimic_table is not None:
            _lib.check(lib.ttamm_mimic_augment(mimic_table.data_ptr(), mimic_table.shape[0], D, rows.data_ptr(), n,
                                               out.data_ptr(), out.data_ptr(), None, _lib.stream_handle(dev)))
        return out
    view = tower if feats is not None else _NoFeatures(tower)
    desc = describe_tower(view, features=feats, mimic_table=mimic_table)
    ws_bytes = int(lib.ttamm_tower_forward_workspace_size(ctypes.byref(desc), min(n, chunk)))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    for lo in range(0, n, chunk):
        m = min(chunk, n - lo)
        r = rows[lo:lo + m]
        _lib.check(lib.ttamm_tower_forward(ctypes.byref(desc), r.data_ptr(), r.data_ptr() if feats is not None else None,
                                           m, 1 if mimic_table is not None else 0, out[lo:lo + m].data_ptr(),
                                           ws.data_ptr(), ws_bytes, _lib.stream_handle(dev)))
    return out


class _NoFeatures(nn.Module):
    def __init__(self, tower: TowerEncoder) -> None:
        super().__init__()
        object.__setattr__(self, "_t", tower)
        self.fusion = "identity"
        self.feature_encoder = None
        self.embedding = tower.embedding


def _uses_cosine(model: nn.Module) -> bool:
    """training.py:670 / :942: the FAISS index and the queries are L2-normalised when the model's
    similarity module is nn.CosineSimilarity (the default, configs/default.yaml:59)."""
    return isinstance(getattr(model, "similarity", None), nn.CosineSimilarity)


def normalize_rows(x: torch.Tensor) -> torch.Tensor:
    """faiss.normalize_L2 (training.py:670-672, :954-955) on a device matrix, in place: each row
    scaled by 1 / sqrt(sum of squares); all-zero rows unchanged.  Returns ``x``."""
    _lib.require_rocm(x, "normalize_rows")
    if x.dtype != torch.float32 or x.dim() != 2 or x.stride(1) != 1:
        raise ValueError("ttamm normalize_rows: a float32 [n, dim] matrix with unit column stride is required")
    if x.numel():
        _lib.check(_lib.load().ttamm_normalize_rows(x.data_ptr(), x.shape[0], x.shape[1], x.stride(0),
                                                     _lib.stream_handle(x.device)))
    return x


def encode_item_embeddings(model, *, num_items: int, item_features: torch.Tensor | None, device: torch.device,
                           batch_size: int = 262_144) -> torch.Tensor:
    """_encode_item_embeddings (training.py:613-643): [num_items, D] item-tower outputs (eval
    mode) plus the item mimic rows — kept in HBM (the reference copies them to the host)."""
    mimic = getattr(model, "adaptive_mimic", None)
    rows = torch.arange(num_items, dtype=torch.long, device=device)
    with torch.no_grad():
        return _encode(model.item_encoder, mimic.item_augmented.weight if mimic is not None else None, rows,
                       item_features, batch_size)


def encode_user_embeddings(model, users: torch.Tensor, *, user_features: torch.Tensor | None,
                           batch_size: int = 262_144) -> torch.Tensor:
    """The query side of _evaluate_model (training.py:1003-1011): user tower (eval) + augment_users."""
    mimic = getattr(model, "adaptive_mimic", None)
    with torch.no_grad():
        return _encode(model.user_encoder, mimic.user_augmented.weight if mimic is not None else None,
                       users.to(torch.long).contiguous(), user_features, batch_size)


def blocked_csr(users: Sequence[int], blocked: Mapping[int, Iterable[int]], device: torch.device
                ) -> tuple[torch.Tensor, torch.Tensor]:
    """Per-query blocked items as CSR (offsets [len(users)+1], values sorted per query)."""
    offsets = [0]
    values: list[int] = []
    for u in users:
        vals = sorted(int(i) for i in blocked.get(int(u), ()))
        values.extend(vals)
        offsets.append(len(values))
    return (torch.tensor(offsets, dtype=torch.long, device=device),
            torch.tensor(values, dtype=torch.long, device=device))


def retrieve_topk(queries: torch.Tensor, items: torch.Tensor, k: int, *,
                  blocked_offsets: torch.Tensor | None = None,
                  blocked_values: torch.Tensor | None = None) -> tuple[torch.Tensor, torch.Tensor]:
    """(scores [nq, k], ids [nq, k]): per query the k best items by inner product that are not
    blocked, best first, ties by item id; -inf / -1 where fewer than k items qualify."""
    _lib.require_rocm(queries, "retrieve_topk")
    if queries.dtype != torch.float32 or items.dtype != torch.float32:
        raise ValueError("ttamm retrieval: float32 embeddings required")
    if queries.dim() != 2 or items.dim() != 2 or queries.shape[1] != items.shape[1]:
        raise ValueError("ttamm retrieval: queries [nq, D] and items [ni, D] with the same D")
    q = _pad_features(queries) if queries.numel() else queries
    x = _pad_features(items) if items.numel() else items
    nq, D = queries.shape
    ni = items.shape[0]
    if (blocked_offsets is None) != (blocked_values is None):
        raise ValueError("ttamm retrieval: blocked_offsets and blocked_values go together")
    if blocked_offsets is not None and blocked_offsets.numel() != nq + 1:
        raise ValueError("ttamm retrieval: blocked_offsets must have n_queries + 1 entries")
    scores = torch.empty((nq, k), dtype=torch.float32, device=queries.device)
    ids = torch.empty((nq, k), dtype=torch.long, device=queries.device)
    lib = _lib.load()
    ws_bytes = int(lib.ttamm_retrieval_topk_workspace_size(nq, ni, D, k))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=queries.device)
    bv = blocked_values if blocked_values is not None and blocked_values.numel() else None
    _lib.check(lib.ttamm_retrieval_topk(
        q.data_ptr() if nq else None, nq, q.stride(0) if nq else D, x.data_ptr() if ni else None, ni,
        x.stride(0) if ni else D, D,
        blocked_offsets.data_ptr() if bv is not None else None, bv.data_ptr() if bv is not None else None,
        k, scores.data_ptr(), ids.data_ptr(), ws.data_ptr(), ws_bytes, _lib.stream_handle(queries.device)))
    return scores, ids


def _group_pairs(val_interactions: Any) -> dict[int, list[int]]:
    groups: dict[int, list[int]] = {}
    if hasattr(val_interactions, "groupby"):  # pandas DataFrame (training.py:999)
        for u, g in val_interactions.groupby("user_idx"):
            groups[int(u)] = [int(i) for i in g["item_idx"].tolist()]
        return groups
    for u, i in val_interactions:
        groups.setdefault(int(u), []).append(int(i))
    return dict(sorted(groups.items()))


def evaluate_model(
    model,
    *,
    train_positive_map: Mapping[int, set[int]],
    val_interactions: Any,
    item_feature_tensor: torch.Tensor | None,
    user_feature_tensor: torch.Tensor | None,
    device: torch.device,
    num_items: int,
    candidate_samples: int = 0,
    k_values: Iterable[int] = (20,),
    rng: Any = None,
    faiss_resources: Any = None,
    faiss_search_k: int = 0,
    item_embeddings: torch.Tensor | None = None,
) -> tuple[dict[int, list[int]], dict[int, set[int]]]:
    """_evaluate_model (training.py:917-1043), exact inner-product branch (cosine models: on
    L2-normalised items and queries, as the FAISS index is built), for every validation user at
    once.  ``val_interactions``: a DataFrame with user_idx / item_idx columns or an
    iterable of (user, item) pairs.  ``candidate_samples`` / ``rng`` / ``faiss_resources`` are
    accepted for signature compatibility; retrieval is always the exact full-corpus search
    (the FAISS branch).

    Semantics kept from :944-970: a user's train positives are never returned; predictions are
    the best max(k_values) remaining items; if fewer exist, the user's ground-truth items not
    already listed are appended (set iteration order) and the list is cut to max_k."""
    groups = _group_pairs(val_interactions)
    if not groups:
        return {}, {}
    model.eval()
    max_k = max(k_values)
    users = [u for u, items in groups.items() if items]
    truth = {u: set(groups[u]) for u in users}
    if item_embeddings is None:
        item_embeddings = encode_item_embeddings(model, num_items=num_items, item_features=item_feature_tensor,
                                                 device=device)
    q = encode_user_embeddings(model, torch.tensor(users, dtype=torch.long, device=device),
                               user_features=user_feature_tensor)
    if _uses_cosine(model):  # normalize_L2 on the index (:670-672) and on every query (:954-955)
        item_embeddings = normalize_rows(item_embeddings.clone())
        normalize_rows(q)
    boff, bval = blocked_csr(users, train_positive_map, device)
    _, ids = retrieve_topk(q, item_embeddings, max_k, blocked_offsets=boff, blocked_values=bval)
    preds: dict[int, list[int]] = {}
    for u, row in zip(users, ids.cpu().tolist()):
        got = [i for i in row if i >= 0]
        if len(got) < max_k:
            seen = set(got)
            got.extend(i for i in truth[u] if i not in seen)
        preds[u] = got[:max_k]
    return preds, truth
