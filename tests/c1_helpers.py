"""BASELINE config C1 on the joinable fixture (tests/golden/c1, made by make_c1_fixture.py):
96-dim towers, MLP [192] -> 96 with dropout 0.15, gated fusion, adaptive mimic, batch 256,
AdamW + SparseAdam at lr 1e-3 (configs/default.yaml with the C1 overrides), cosine similarity for
evaluation.  Both the oracle and ttamm train through the reference's epoch loop shape — a
torch DataLoader (shuffle=True, drop_last=False, so the last batch is short) — with the RNG
streams the two devices cannot share (negatives, dropout masks) injected by one hook."""

from __future__ import annotations

import sys
from dataclasses import dataclass
from functools import lru_cache
from pathlib import Path

import torch
from torch.utils.data import DataLoader, TensorDataset

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE / "golden"))

from oracle import cpu_reference as ref  # noqa: E402

D, H, N, B, P_DROP = 96, 192, 5, 256, 0.15
LOSS_WEIGHTS = {"mimic_user": 0.15, "mimic_item": 0.15, "category_alignment": 0.01}
K_VALUES = (5, 10, 20)
SEED = 1234

TOWER_CFG = {
    "type": "tower",
    "id_embedding": {"params": {"embedding_dim": D, "sparse": True}, "init": {"type": "normal", "std": 0.02}},
    "feature_encoder": {"type": "mlp", "hidden_dims": [H], "activation": "relu", "output_dim": D, "dropout": P_DROP},
    "fusion": "gated",
}


@dataclass
class C1:
    num_users: int
    num_items: int
    train: torch.Tensor  # [n, 2] int64 (user_idx, item_idx)
    val_pairs: list
    positives: dict      # whole-dataset positives (training.py:1482)
    train_positive_map: dict
    user_features: torch.Tensor
    item_features: torch.Tensor
    categories: torch.Tensor
    major: int


@lru_cache(maxsize=2)
def load_c1(variant: str = "c1") -> C1:
    """The fixture: "c1" (tests/golden/c1, 1,600 users) or "c1_large" (20,000 users)."""
    import make_c1_fixture as fx

    data, train, val, test, cats, major = fx.prepare(fx.OUT_LARGE if variant == "c1_large" else fx.OUT)
    tp = {int(u): set(map(int, g["item_idx"].tolist())) for u, g in train.groupby("user_idx")}
    return C1(data.num_users, data.num_items, torch.tensor(train[["user_idx", "item_idx"]].to_numpy(), dtype=torch.long),
              [(int(u), int(i)) for u, i in val[["user_idx", "item_idx"]].to_numpy()], data.user_positive_items, tp,
              torch.from_numpy(data.user_features), torch.from_numpy(data.item_features), cats, int(major))


def build_oracle_model(c1: C1):
    torch.manual_seed(SEED)  # _seed_everything (training.py:185-190) before the towers are built
    return ref.build_model(TOWER_CFG, num_users=c1.num_users, num_items=c1.num_items,
                           user_feature_dim=c1.user_features.shape[1], item_feature_dim=c1.item_features.shape[1])


def loader(c1: C1, epoch: int) -> DataLoader:
    """_build_dataloader (training.py:260-264) with a per-epoch seeded shuffle, so every run sees
    the same batches."""
    ds = TensorDataset(c1.train[:, 0].contiguous(), c1.train[:, 1].contiguous())
    return DataLoader(ds, batch_size=B, shuffle=True, drop_last=False,
                      generator=torch.Generator().manual_seed(SEED * 31 + epoch))


class Streams:
    """The batch hook: negatives from the reference sampler (samplers.py:11-85, restated) and
    dropout keep-masks, from a generator keyed by (epoch, step) — a pure function of its inputs."""

    def __init__(self, c1: C1, epoch: int) -> None:
        self.c1, self.epoch = c1, epoch

    def __call__(self, step: int, users: torch.Tensor, pos: torch.Tensor):
        g = torch.Generator().manual_seed(SEED * 100_003 + self.epoch * 1_009 + step)
        neg = ref.sample_negative_items(users, num_items=self.c1.num_items, positives=self.c1.positives,
                                        num_negatives=N, generator=g)
        b = users.shape[0]
        um = [(torch.rand((b, H), generator=g) >= P_DROP).to(torch.uint8)]
        im = [(torch.rand((b * (1 + N), H), generator=g) >= P_DROP).to(torch.uint8)]
        return neg, {"user": um, "item": im}


def train_oracle(c1: C1, epochs: int):
    model = build_oracle_model(c1)
    opts = ref.build_optimizers(model, lr=1e-3, weight_decay=0.01)
    per_epoch, steps = [], []
    for ep in range(epochs):
        mean, _, _ = ref.train_one_epoch(model, loader(c1, ep), opts, negatives_per_positive=N, num_items=c1.num_items,
                                         positives=c1.positives, user_features=c1.user_features,
                                         item_features=c1.item_features, loss_weights=LOSS_WEIGHTS,
                                         item_category_tensor=c1.categories, major_category_id=c1.major,
                                         batch_hook=Streams(c1, ep), step_losses=steps)
        per_epoch.append(mean)
    return model, per_epoch, [s.total for s in steps]


def recall_at(model, c1: C1, k: int = 20) -> float:
    """_evaluate_model with the FAISS exact-IP branch on a cosine model (training.py:646-679,
    917-1043) + compute_ranking_metrics (metrics.py:74-116), all on the CPU restatement."""
    preds, truth = ref.evaluate_model(model, train_positive_map=c1.train_positive_map, val_pairs=c1.val_pairs,
                                      item_features=c1.item_features, user_features=c1.user_features,
                                      num_items=c1.num_items, k_values=K_VALUES, faiss_search_k=max(K_VALUES) * 4,
                                      normalize=True)
    return ref.ranking_metrics(preds, truth, K_VALUES).recall[k]
