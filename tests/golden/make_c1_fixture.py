"""Generate the joinable trimmed-scale fixture of BASELINE config C1.

The reference ships books_trimmed.csv / users_trimmed.csv, but the two share no parent_asin, so
its own pipeline cannot train on them (the book filter leaves 0 interactions).  This script
writes a deterministic replacement in the SAME CSV schema —

  books_c1.csv.gz  title, author, average_rating, rating_number, price, categories, parent_asin
  users_c1.csv.gz  parent_asin, userId, timestamp

— with planted structure so retrieval is learnable: 24 main categories ("clusters") with 14
subcategories each, authors tied to clusters, users preferring one or two clusters.  Sizes are
chosen so the reference's feature pipeline (category_top_k = author_top_k = 300,
configs/default.yaml:19-21) yields exactly F = 300 + 300 + 3 + 2 = 605 feature columns, and the
frequency filters (min_user_interactions 3, min_item_interactions 6) keep ~1.5k users x ~2k items.

Then it runs the oracle's restatement of the reference's data preparation
(oracle/data_prep.py) and records a summary (counts, feature checksums) in c1_expected.json;
tests/test_c1_cpu.py checks the preparation still reproduces it.

    python tests/golden/make_c1_fixture.py            # tests/golden/c1
    python tests/golden/make_c1_fixture.py --large    # tests/golden/c1_large (20,000 users)
"""

from __future__ import annotations

import hashlib
import json
import sys
from pathlib import Path

import numpy as np
import pandas as pd

HERE = Path(__file__).resolve().parent
OUT = HERE / "c1"
ROOT = HERE.parents[1]

N_CLUSTERS = 24
SUBCATS = 14
AUTHORS_PER_CLUSTER = 18
N_ITEMS = 3200
N_USERS = 1600
WORDS = ("the of and history art science love war night city secret garden river time world house "
         "light dark story guide life little great last first new lost dream stone song").split()

# configs/default.yaml data section, with the C1 overrides (BASELINE.json configs[0])
DATA_CONFIG = {
    "books_file": "books_c1.csv.gz",
    "users_file": "users_c1.csv.gz",
    "train_fraction": 0.85,
    "test_fraction": 0.15,
    "min_user_interactions": 3,
    "min_item_interactions": 6,
    "feature_params": {"numeric_columns": ["average_rating", "price", "rating_number"],
                       "category_top_k": 300, "author_top_k": 300, "user_aggregation": "mean"},
    "seed": 1234,
}


# The large variant (tests/golden/c1_large): the same schema and planted structure at 20,000 users
# (one validation pair each, so Recall@20's +-0.002 is 40 users, not 3), 6-14 interactions per
# user and 12-character user ids so the three training epochs and the committed CSVs stay small
LARGE = {"n_users": 20_000, "n_items": 4_000, "inter": (5, 11), "seed": 20261018, "id_len": 12}


def generate(rng: np.random.Generator, n_users: int = N_USERS, n_items: int = N_ITEMS,
             inter: tuple[int, int] = (8, 31), id_len: int = 28) -> tuple[pd.DataFrame, pd.DataFrame]:
    N_ITEMS, N_USERS = n_items, n_users  # noqa: N806 (module defaults = the C1 fixture)
    cluster_names = [f"Cluster {c:02d} Studies" for c in range(N_CLUSTERS)]
    item_cluster = rng.integers(0, N_CLUSTERS, N_ITEMS)
    books = []
    for i in range(N_ITEMS):
        c = int(item_cluster[i])
        sub = int(rng.integers(0, SUBCATS))
        author = f"Author {c:02d}-{int(rng.integers(0, AUTHORS_PER_CLUSTER)):02d}"
        title = " ".join(rng.choice(WORDS, size=int(rng.integers(1, 9))))
        rating = "" if rng.random() < 0.05 else f"{rng.uniform(1.0, 5.0):.1f}"
        price = "" if rng.random() < 0.1 else f"{rng.lognormal(2.3, 0.6):.2f}"
        books.append({
            "title": json.dumps([title.title()]),
            "author": author,
            "average_rating": rating,
            "rating_number": int(rng.zipf(1.6)) if rng.random() > 0.02 else "",
            "price": price,
            "categories": json.dumps(["Books", cluster_names[c], f"Topic {c:02d}.{sub:02d}"]),
            "parent_asin": f"B{i * 7919 % 10**9:09d}",
        })
    # item popularity inside each cluster: Zipf-like weights over a random order
    members = [np.flatnonzero(item_cluster == c) for c in range(N_CLUSTERS)]
    weights = []
    for m in members:
        w = 1.0 / np.arange(1, m.size + 1) ** 0.8
        weights.append(w[rng.permutation(m.size)] / w.sum())
    rows = []
    t0 = 1_600_000_000_000
    for u in range(N_USERS):
        uid = "".join(rng.choice(list("ABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789"), size=id_len))
        fav = rng.choice(N_CLUSTERS, size=int(rng.integers(1, 3)), replace=False)
        n = int(rng.integers(*inter))
        picked: set[int] = set()
        while len(picked) < n:
            if rng.random() < 0.85:
                c = int(rng.choice(fav))
                picked.add(int(rng.choice(members[c], p=weights[c])))
            else:
                picked.add(int(rng.integers(0, N_ITEMS)))
        ts = t0 + np.sort(rng.integers(0, 10**10, size=n))
        for it, t in zip(rng.permutation(sorted(picked)), ts):
            rows.append({"parent_asin": books[int(it)]["parent_asin"], "userId": uid, "timestamp": int(t)})
    users = pd.DataFrame(rows)
    return pd.DataFrame(books), users.iloc[rng.permutation(len(users))].reset_index(drop=True)


def prepare(data_dir: Path = OUT):
    """The reference's data path on the fixture (oracle restatement): returns
    (PreparedData, train, val, test, item_category_tensor, major_category_id)."""
    sys.path.insert(0, str(ROOT))
    from oracle import data_prep as dp

    cfg = DATA_CONFIG
    books, inter = dp.load_dataset(data_dir, books_file=cfg["books_file"], interactions_file=cfg["users_file"])
    data = dp.build_training_dataset(books, inter, feature_config=cfg["feature_params"],
                                     min_user_interactions=cfg["min_user_interactions"],
                                     min_item_interactions=cfg["min_item_interactions"])
    train, val, test = dp.split_train_validation_test(data.interactions, train_fraction=cfg["train_fraction"],
                                                      test_fraction=cfg["test_fraction"], seed=cfg["seed"])
    cats, major = dp.item_category_tensor(data.items, data.num_items)
    return data, train, val, test, cats, major


def summary(prepared) -> dict:
    data, train, val, test, cats, major = prepared

    def digest(a: np.ndarray) -> str:
        return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]

    return {
        "num_users": data.num_users,
        "num_items": data.num_items,
        "interactions": len(data.interactions),
        "train": len(train), "val": len(val), "test": len(test),
        "feature_dim": int(data.item_features.shape[1]),
        "item_features_sha": digest(data.item_features),
        "user_features_sha": digest(data.user_features),
        "train_pairs_sha": digest(train[["user_idx", "item_idx"]].to_numpy(np.int64)),
        "val_pairs_sha": digest(val[["user_idx", "item_idx"]].to_numpy(np.int64)),
        "num_categories": int(cats.max().item()) + 1,
        "major_category": int(major),
    }


OUT_LARGE = HERE / "c1_large"


def main(argv: list[str]) -> None:
    large = "--large" in argv
    out = OUT_LARGE if large else OUT
    out.mkdir(parents=True, exist_ok=True)
    if large:
        books, users = generate(np.random.default_rng(LARGE["seed"]), LARGE["n_users"], LARGE["n_items"],
                                LARGE["inter"], LARGE["id_len"])
    else:
        books, users = generate(np.random.default_rng(20251114))
    books.to_csv(out / "books_c1.csv.gz", index=False, compression={"method": "gzip", "mtime": 0})
    users.to_csv(out / "users_c1.csv.gz", index=False, compression={"method": "gzip", "mtime": 0})
    s = summary(prepare(out))
    (out / "c1_expected.json").write_text(json.dumps(s, indent=1) + "\n")
    print(json.dumps(s))


if __name__ == "__main__":
    main(sys.argv[1:])
