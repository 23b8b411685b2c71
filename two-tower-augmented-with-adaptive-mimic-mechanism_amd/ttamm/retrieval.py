"""Exact inner-product retrieval on the MI355X — drop-in for the FAISS branch of
the reference's evaluation: ``_encode_item_embeddings`` (training.py:613-643), the
``IndexFlatIP`` index (:645-679) and ``_evaluate_model``'s search + filter (:917-1043,
:944-970).

The item matrix stays in HBM; ``retrieve_topk`` runs ``ttamm_retrieval_topk`` (fp32-accurate
scores on the bf16 matrix cores — each operand split into three bf16 planes, six MFMA products
per fp32 product, D <= 128; fp32 MFMA for wider rows or with TTAMM_RETRIEVAL_FP32=1 — fused with
a per-query top-k that skips each user's blocked train positives), so there is no per-user search
call and no host round trip per user.  Scores agree with faiss IndexFlatIP's fp32 inner products
to ~1e-7 relative, not bit for bit: near-tied items can swap.
"""

from __future__ import annotations

import ctypes
from typing import Any, Iterable, Mapping, Sequence

import numpy as np
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
    feats = _pad_features(features) if tower.fusion != "identity" else None
    out = torch.empty((n, tower.output_dim if feats is not None else D), dtype=torch.float32, device=dev)
    if n == 0:
        return out
    _lib.check_index_range(rows, tower.num_embeddings)
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
    if queries.shape[1] % 8:
        # the kernel takes D % 8 == 0: zero columns leave every inner product unchanged (any D
        # trains, and FAISS IndexFlatIP takes any D)
        D8 = (queries.shape[1] + 7) // 8 * 8
        queries = torch.nn.functional.pad(queries, (0, D8 - queries.shape[1]))
        items = torch.nn.functional.pad(items, (0, D8 - items.shape[1]))
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


def prepare_faiss_resources(model, *, num_items: int, item_features: torch.Tensor | None, device: torch.device,
                            similarity_module: nn.Module | None = None, batch_size: int = 262_144,
                            retain_embeddings: bool = False) -> dict[str, Any] | None:
    """_prepare_faiss_resources (training.py:646-679): the item matrix of the exact inner-product
    index — kept in HBM instead of a faiss.IndexFlatIP — L2-normalised when the similarity is
    cosine.  Pass the result as ``faiss_resources`` to evaluate_model."""
    if num_items == 0:
        return None
    emb = encode_item_embeddings(model, num_items=num_items, item_features=item_features, device=device,
                                 batch_size=batch_size)
    sim = similarity_module if similarity_module is not None else getattr(model, "similarity", None)
    normalize = isinstance(sim, nn.CosineSimilarity)
    if normalize:
        normalize_rows(emb)
    out: dict[str, Any] = {"index": emb, "normalize": normalize}
    if retain_embeddings:
        out["embeddings"] = emb
    return out


def sampled_candidates(users: Sequence[int], truth: Mapping[int, set[int]], blocked: Mapping[int, Iterable[int]],
                       *, num_items: int, candidate_samples: int, rng: np.random.Generator) -> list[list[int]]:
    """Candidate lists of _retrieve_with_sampling (training.py:979-987), drawing from ``rng`` in
    the reference's order (one rng.choice per user, users ascending as DataFrame.groupby yields
    them): the user's ground truth plus up to ``candidate_samples`` distinct unblocked items.
    The reference draws from ``list(set(range(n)) - blocked)``, whose order is CPython's: when
    len(blocked) < n / 4 (set_difference's copy-and-discard path, (n >> 2) > len(blocked)) it is
    ascending (small ints sit at their own hash slot of a table larger than n), so the sorted
    setdiff is the same array and rng.choice picks the same items; otherwise CPython builds a new,
    smaller table whose order is not ascending, and the reference's expression itself is
    evaluated.  The list order is the reference's set order."""
    everything = np.arange(num_items, dtype=np.int64)
    lists: list[list[int]] = []
    for u in users:
        cands = set(truth[u])
        b = set(blocked.get(int(u), ()))
        if not b:
            avail = everything
        elif (num_items >> 2) > len(b):
            avail = np.setdiff1d(everything, np.fromiter(b, dtype=np.int64), assume_unique=False)
        else:  # CPython's new-set path: the reference's own expression, in its iteration order
            avail = np.fromiter(set(range(num_items)) - b, dtype=np.int64)
        if avail.size:
            budget = max(0, min(int(candidate_samples), int(avail.size)))
            if budget > 0:
                cands.update(int(n) for n in rng.choice(avail, size=budget, replace=False).tolist())
        lists.append(list(cands))
    return lists


def _evaluate_sampled(model, users: list[int], truth: dict[int, set[int]], blocked: Mapping[int, Iterable[int]], *,
                      item_features, user_features, device, num_items: int, candidate_samples: int, max_k: int,
                      rng: np.random.Generator) -> dict[int, list[int]]:
    """_retrieve_with_sampling for every user in one launch (ttamm_candidate_topk)."""
    lists = sampled_candidates(users, truth, blocked, num_items=num_items, candidate_samples=candidate_samples, rng=rng)
    flat = np.fromiter((i for c in lists for i in c), dtype=np.int64)
    offsets = np.zeros(len(lists) + 1, dtype=np.int64)
    np.cumsum([len(c) for c in lists], out=offsets[1:])
    most = max((len(c) for c in lists), default=0)
    uniq, rows = np.unique(flat, return_inverse=True)
    mimic = getattr(model, "adaptive_mimic", None)
    with torch.no_grad():
        items = _encode(model.item_encoder, mimic.item_augmented.weight if mimic is not None else None,
                        torch.from_numpy(uniq).to(device), item_features, 262_144)
        q = encode_user_embeddings(model, torch.tensor(users, dtype=torch.long, device=device), user_features=user_features)
    k = max(1, max_k)
    scores = torch.empty((len(users), k), dtype=torch.float32, device=device)
    pos = torch.empty((len(users), k), dtype=torch.long, device=device)
    off_d = torch.from_numpy(offsets).to(device)
    rows_d = torch.from_numpy(rows.astype(np.int64)).to(device)
    cosine = 1 if isinstance(getattr(model, "similarity", None), nn.CosineSimilarity) else 0
    _lib.check(_lib.load().ttamm_candidate_topk(
        q.data_ptr(), len(users), q.stride(0), items.data_ptr() if items.numel() else None, items.shape[0],
        items.stride(0) if items.numel() else q.shape[1], q.shape[1], off_d.data_ptr(),
        rows_d.data_ptr() if rows_d.numel() else None, most, cosine, k, scores.data_ptr(), pos.data_ptr(),
        _lib.stream_handle(device)))
    preds: dict[int, list[int]] = {}
    for u, cand, prow in zip(users, lists, pos.cpu().tolist()):
        preds[u] = [cand[p] for p in prow[: min(max_k, len(cand))]]
    return preds


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
    """_evaluate_model (training.py:917-1043) for every validation user at once.
    ``val_interactions``: a DataFrame with user_idx / item_idx columns or an iterable of
    (user, item) pairs.  Branches, as the reference picks them (:940, :1029-1040):

      * ``faiss_resources`` given (``prepare_faiss_resources``: the HBM item matrix standing in
        for faiss.IndexFlatIP) — exact inner-product search, on L2-normalised items and queries
        for a cosine model.  A user's train positives are never returned; predictions are the
        best max(k_values) remaining items; if fewer exist, the user's ground-truth items not
        already listed are appended (set iteration order) and the list is cut to max_k (:944-972);
      * no ``faiss_resources`` and an ``rng`` — the sampled-candidate branch the reference takes
        without faiss (:974-1009): ground truth + ``candidate_samples`` random unblocked items
        per user drawn from ``rng`` in the reference's order, ranked by the model's similarity;
      * neither — the exact search (the item matrix is built here)."""
    groups = _group_pairs(val_interactions)
    if not groups:
        return {}, {}
    model.eval()
    max_k = max(k_values)
    users = [u for u, items in groups.items() if items]
    truth = {u: set(groups[u]) for u in users}
    if faiss_resources is None and rng is not None and item_embeddings is None:
        return _evaluate_sampled(model, users, truth, train_positive_map, item_features=item_feature_tensor,
                                 user_features=user_feature_tensor, device=device, num_items=num_items,
                                 candidate_samples=candidate_samples, max_k=max_k, rng=rng), truth
    if faiss_resources is not None and item_embeddings is None:
        item_embeddings = faiss_resources["index"]
        if faiss_resources.get("normalize"):  # already normalised; the queries still need it
            q = encode_user_embeddings(model, torch.tensor(users, dtype=torch.long, device=device),
                                       user_features=user_feature_tensor)
            normalize_rows(q)
            return _exact(users, truth, q, item_embeddings, train_positive_map, max_k, device), truth
    if item_embeddings is None:
        item_embeddings = encode_item_embeddings(model, num_items=num_items, item_features=item_feature_tensor,
                                                 device=device)
    q = encode_user_embeddings(model, torch.tensor(users, dtype=torch.long, device=device),
                               user_features=user_feature_tensor)
    if _uses_cosine(model):  # normalize_L2 on the index (:670-672) and on every query (:954-955)
        item_embeddings = normalize_rows(item_embeddings.clone())
        normalize_rows(q)
    return _exact(users, truth, q, item_embeddings, train_positive_map, max_k, device), truth


def _exact(users, truth, q, item_embeddings, train_positive_map, max_k, device) -> dict[int, list[int]]:
    boff, bval = blocked_csr(users, train_positive_map, device)
    _, ids = retrieve_topk(q, item_embeddings, max_k, blocked_offsets=boff, blocked_values=bval)
    preds: dict[int, list[int]] = {}
    for u, row in zip(users, ids.cpu().tolist()):
        got = [i for i in row if i >= 0]
        if len(got) < max_k:
            seen = set(got)
            got.extend(i for i in truth[u] if i not in seen)
        preds[u] = got[:max_k]
    return preds
