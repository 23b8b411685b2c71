"""CPU restatement of the reference's data preparation — TEST INFRASTRUCTURE ONLY.

Turns CSVs in the reference schema (books: title, author, average_rating, rating_number, price,
categories, parent_asin; interactions: parent_asin, userId, timestamp) into what the training
step consumes, following the reference function by function:

  load_dataset                      src/data/loaders.py:32-118
  build_training_dataset            src/data/preprocessing.py:42-166
  build_item/user_feature_matrix    src/data/features.py:129-315 (parse_category_tokens :58-126)
  build_index_mapping               src/data/indexers.py:38-55
  split_train_validation_test       src/pipelines/training.py:193-257
  item_category_tensor              src/pipelines/training.py:582-610

It exists to build the joinable trimmed-scale fixture of the Recall@20 parity test (the
shipped trimmed CSVs share no parent_asin), so both the oracle and ttamm train on
the exact inputs the reference would derive.  Only tests/ import it.
"""

from __future__ import annotations

import ast
from collections import Counter
from dataclasses import dataclass
from pathlib import Path
from typing import Any, Mapping

import numpy as np
import pandas as pd
import torch


# ---------------------------------------------------------------------------------------
# loaders.py:32-118
# ---------------------------------------------------------------------------------------
def load_dataset(data_dir: Path, *, books_file: str, interactions_file: str,
                 books_limit: int | None = None, interactions_limit: int | None = None):
    data_dir = Path(data_dir)
    for f in (books_file, interactions_file):
        if not (data_dir / f).exists():
            raise FileNotFoundError(f"Expected CSV at {data_dir / f} but file was not found.")
    books = pd.read_csv(data_dir / books_file, nrows=books_limit)
    inter = pd.read_csv(data_dir / interactions_file, nrows=interactions_limit,
                        dtype={"parent_asin": "string", "userId": "string", "timestamp": "Int64"})
    if not books.empty and "parent_asin" in books and "parent_asin" in inter:
        keep = inter["parent_asin"].astype(str).isin(set(books["parent_asin"].astype(str)))
        inter = inter[keep].reset_index(drop=True)
    return books, inter


# ---------------------------------------------------------------------------------------
# features.py:58-126 — category strings -> hierarchical tokens
# ---------------------------------------------------------------------------------------
def _category_paths(raw: Any) -> list[list[str]]:
    if raw is None or (isinstance(raw, float) and pd.isna(raw)):
        return []
    box = raw
    if isinstance(raw, str):
        text = raw.strip()
        if not text:
            return []
        try:
            box = ast.literal_eval(text)
        except (ValueError, SyntaxError):
            return [[t.strip() for t in text.split(",") if t.strip()]]
    if not isinstance(box, list):
        s = str(box).strip()
        return [[s]] if s else []
    if box and all(isinstance(x, (list, tuple)) for x in box):
        return [p for p in ([str(e).strip() for e in x if str(e).strip()] for x in box) if p]
    flat = [str(x).strip() for x in box if str(x).strip()]
    if flat:
        return [flat]
    out: list[list[str]] = []
    for x in box:
        if isinstance(x, (list, tuple)):
            p = [str(e).strip() for e in x if str(e).strip()]
            if p:
                out.append(p)
        elif str(x).strip():
            out.append([str(x).strip()])
    return out


def parse_category_tokens(raw: Any) -> list[str]:
    tokens: list[str] = []
    for path in _category_paths(raw):
        kept = [c for c in path if c and c.lower() != "books"]
        if not kept:
            continue
        tokens.append(kept[0])
        for depth in range(1, len(kept)):
            tokens.append(" > ".join([kept[0]] + kept[1:depth + 1]))
    return list(dict.fromkeys(tokens))  # dedupe, first occurrence wins


# ---------------------------------------------------------------------------------------
# features.py:129-266 — item feature matrix [categories | authors | numeric | title stats]
# ---------------------------------------------------------------------------------------
def _zscore(m: np.ndarray) -> np.ndarray:
    mean = np.nanmean(m, axis=0)
    std = np.nanstd(m, axis=0)
    std = np.where(std == 0, 1.0, std)
    m = np.where(np.isnan(m), mean, m)
    return ((m - mean) / std).astype(np.float32)


def _category_matrix(cats: list[list[str]], top_k: int) -> np.ndarray:
    counts: Counter[str] = Counter()
    depth: dict[str, int] = {}
    for row in cats:
        for c in row:
            counts[c] += 1
            depth.setdefault(c, c.count(" > "))
    vocab = [c for c, _ in counts.most_common(top_k) if c]
    out = np.zeros((len(cats), len(vocab)), dtype=np.float32)
    col = {c: i for i, c in enumerate(vocab)}
    for r, row in enumerate(cats):
        for c in row:
            j = col.get(c)
            if j is not None:
                out[r, j] = max(out[r, j], 1.0 / float(depth.get(c, c.count(" > ")) + 1))
    return out


def _author_matrix(authors: list, top_k: int) -> np.ndarray:
    s = pd.Series(authors).fillna("Unknown").astype(str)
    vocab = list(s.value_counts().head(top_k).index)
    out = np.zeros((len(s), len(vocab)), dtype=np.float32)
    col = {a: i for i, a in enumerate(vocab)}
    for r, a in enumerate(s.tolist()):
        j = col.get(a)
        if j is not None:
            out[r, j] = 1.0
    return out


def build_item_feature_matrix(books: pd.DataFrame, cfg: Mapping[str, Any] | None) -> np.ndarray:
    cfg = dict(cfg or {})
    numeric_cols = [c for c in cfg.get("numeric_columns", ["average_rating", "price", "rating_number"]) if c in books]
    numeric = np.zeros((len(books), len(numeric_cols)), dtype=np.float32)
    if numeric_cols:
        numeric = _zscore(books[numeric_cols].apply(pd.to_numeric, errors="coerce").to_numpy(dtype=np.float32, copy=True))
    titles = books["title"] if "title" in books else pd.Series([""] * len(books))
    words, chars = [], []
    for t in titles:
        text = "" if pd.isna(t) else str(t)
        words.append(len(text.split()))
        chars.append(len(text))
    title_stats = _zscore(np.stack([words, chars], axis=1).astype(np.float32))
    raw_cats = books["categories"] if "categories" in books else pd.Series([[] for _ in range(len(books))])
    cat = _category_matrix(raw_cats.apply(parse_category_tokens).tolist(), int(cfg.get("category_top_k", 500)))
    auth = _author_matrix((books["author"] if "author" in books else pd.Series(["Unknown"] * len(books))).tolist(),
                          int(cfg.get("author_top_k", 500)))
    parts = [p for p in (cat, auth, numeric, title_stats) if p.size > 0]
    return np.concatenate(parts, axis=1).astype(np.float32, copy=False)


def build_user_feature_matrix(inter: pd.DataFrame, item_features: np.ndarray, num_users: int) -> np.ndarray:
    """features.py:269-315, mean aggregation."""
    out = np.zeros((num_users, item_features.shape[1]), dtype=np.float32)
    for u, g in inter.groupby("user_idx"):
        rows = g["item_idx"].to_numpy(dtype=int, copy=False)
        if rows.size:
            out[int(u)] = item_features[rows].mean(axis=0).astype(np.float32, copy=False)
    return out


# ---------------------------------------------------------------------------------------
# indexers.py:38-55, preprocessing.py:42-166
# ---------------------------------------------------------------------------------------
def index_mapping(values) -> tuple[dict[str, int], list[str]]:
    fwd: dict[str, int] = {}
    order: list[str] = []
    for v in values:
        if v not in fwd:
            fwd[v] = len(order)
            order.append(v)
    return fwd, order


@dataclass
class PreparedData:
    items: pd.DataFrame
    interactions: pd.DataFrame
    num_users: int
    num_items: int
    user_positive_items: dict[int, set[int]]
    item_features: np.ndarray
    user_features: np.ndarray


def build_training_dataset(books: pd.DataFrame, inter: pd.DataFrame, *, feature_config=None,
                           min_user_interactions: int = 0, min_item_interactions: int = 0) -> PreparedData:
    books = books.dropna(subset=["parent_asin"]).drop_duplicates(subset=["parent_asin"]).copy()
    books["parent_asin"] = books["parent_asin"].astype(str)
    inter = inter.dropna(subset=["parent_asin", "userId"]).copy()
    inter["parent_asin"] = inter["parent_asin"].astype(str)
    inter["userId"] = inter["userId"].astype(str)
    inter = inter[inter["parent_asin"].isin(set(books["parent_asin"]))].reset_index(drop=True)
    mu, mi = max(int(min_user_interactions), 0), max(int(min_item_interactions), 0)
    if not inter.empty and (mu > 0 or mi > 0):
        prev = -1
        while prev != len(inter):  # alternate item / user frequency filters to a fixed point
            prev = len(inter)
            if mi > 0 and not inter.empty:
                vc = inter["parent_asin"].value_counts()
                inter = inter[inter["parent_asin"].isin(vc[vc >= mi].index)]
            if mu > 0 and not inter.empty:
                vc = inter["userId"].value_counts()
                inter = inter[inter["userId"].isin(vc[vc >= mu].index)]
            inter = inter.reset_index(drop=True)
    if not inter.empty:
        books = books[books["parent_asin"].isin(set(inter["parent_asin"]))].reset_index(drop=True)
    item_map, items_order = index_mapping(books["parent_asin"])
    user_map, users_order = index_mapping(inter["userId"])
    inter["item_idx"] = inter["parent_asin"].map(item_map).astype("int64")
    inter["user_idx"] = inter["userId"].map(user_map).astype("int64")
    books["item_idx"] = books["parent_asin"].map(item_map).astype("int64")
    item_features = build_item_feature_matrix(books, feature_config)
    user_features = build_user_feature_matrix(inter, item_features, len(users_order))
    positives = {int(u): set(map(int, g["item_idx"].tolist())) for u, g in inter.groupby("user_idx")}
    return PreparedData(books, inter, len(users_order), len(items_order), positives, item_features, user_features)


# ---------------------------------------------------------------------------------------
# training.py:193-257 — latest interaction per user -> validation, random fraction -> test
# ---------------------------------------------------------------------------------------
def split_train_validation_test(inter: pd.DataFrame, *, train_fraction, test_fraction, seed):
    df = inter.copy()
    if "timestamp" not in df.columns:
        train, val = df, df.iloc[0:0]
    else:
        df = df.sort_values("timestamp").reset_index(drop=True)
        held: list[int] = []
        for _, g in df.groupby("user_idx"):
            ts = g["timestamp"].dropna()
            if ts.empty or len(g) <= 1:
                continue
            held.append(int(ts.idxmax()))
        if held:
            train, val = df.drop(index=held).reset_index(drop=True), df.loc[held].reset_index(drop=True)
        else:
            train, val = df, df.iloc[0:0]
    if train_fraction is not None and test_fraction is None:
        test_fraction = max(0.0, 1.0 - float(train_fraction))
    test_fraction = float(test_fraction or 0.0)
    if test_fraction <= 0.0 or train.empty:
        return train, val, train.iloc[0:0]
    rng = np.random.default_rng(seed)
    n_test = max(1, int(round(len(train) * min(test_fraction, 1.0))))
    if n_test >= len(train):
        return train.iloc[0:0].reset_index(drop=True), val, train.copy().reset_index(drop=True)
    pick = rng.choice(train.index.to_numpy(), size=n_test, replace=False)
    test = train.loc[pick].copy().reset_index(drop=True)
    return train.drop(index=pick).reset_index(drop=True), val, test


def item_category_tensor(items: pd.DataFrame, num_items: int) -> tuple[torch.Tensor | None, int | None]:
    """training.py:582-610: each item's first category token (ids in first-seen order) and the
    most frequent one."""
    if num_items == 0 or "item_idx" not in items:
        return None, None
    primary = ["<unknown>"] * num_items
    counts: Counter[str] = Counter()
    for _, row in items.iterrows():
        toks = parse_category_tokens(row.get("categories"))
        first = toks[0] if toks else "<unknown>"
        primary[int(row["item_idx"])] = first
        counts[first] += 1
    if not counts:
        return None, None
    ids = {c: i for i, c in enumerate(counts.keys())}
    major = max(counts.items(), key=lambda kv: kv[1])[0]
    return torch.tensor([ids[c] for c in primary], dtype=torch.long), ids[major]
