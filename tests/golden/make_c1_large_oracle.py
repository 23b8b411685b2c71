"""The oracle's Recall@20 on the large C1-schema fixture (tests/golden/c1_large, 20,000 users), and
the oracle's own spread under summation-order-only changes.

Trains the CPU restatement (oracle/cpu_reference.py) for EPOCHS epochs exactly as
tests/test_c1_gpu.py trains ttamm (same init, DataLoader order, injected negatives and dropout
masks: tests/c1_helpers.py) and evaluates Recall@20 with the restated _evaluate_model (exact-IP
branch, cosine).  Variants that change only fp32 summation order:

  threads8   8 intra-op threads (the default run; its Recall@20 is the test's reference value)
  threads1   1 thread (other GEMM blocking in the CPU BLAS)
  splitk2    8 threads, the first feature layer's K = 605 reduction split in two halves summed
             (the reordering of ttamm's reverted split-K layer 1, round 4)
  float64    the same run in float64 (model, optimizer state, features): the trajectory of exact
             arithmetic that every fp32 run approximates (round 6: the fp32 variants' epoch means
             sit 1.2-2.1e-5 from it; tests/test_c1_gpu.py measures ttamm against it)

  python tests/golden/make_c1_large_oracle.py --only float64   adds / refreshes one variant in the
             existing oracle_recall.json without re-running the others

Writes tests/golden/c1_large/oracle_recall.json (Recall@5/10/20 per variant, epoch means, and
the largest pairwise Recall@20 difference among the variants = the oracle's own spread).

    python tests/golden/make_c1_large_oracle.py     (~5 minutes on 8 cores)
"""

from __future__ import annotations

import json
import sys
import time
from pathlib import Path

import torch

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path[:0] = [str(ROOT / "tests"), str(ROOT)]

from c1_helpers import K_VALUES, load_c1, train_oracle  # noqa: E402
from oracle import cpu_reference as ref  # noqa: E402

EPOCHS = 3


def _splitk_linear(orig):
    def lin(layer, x, bf16):
        k = layer.in_features
        if bf16 or k < 512:
            return orig(layer, x, bf16)
        h = k // 2
        w = layer.weight
        return x[:, :h] @ w[:, :h].t() + x[:, h:] @ w[:, h:].t() + layer.bias
    return lin


def _train_float64(c1):
    from c1_helpers import LOSS_WEIGHTS, N, Streams, build_oracle_model, loader

    model = build_oracle_model(c1).double()
    opts = ref.build_optimizers(model, lr=1e-3, weight_decay=0.01)
    uf, itf = c1.user_features.double(), c1.item_features.double()
    epochs = []
    for ep in range(EPOCHS):
        mean, _, _ = ref.train_one_epoch(model, loader(c1, ep), opts, negatives_per_positive=N, num_items=c1.num_items,
                                         positives=c1.positives, user_features=uf, item_features=itf,
                                         loss_weights=LOSS_WEIGHTS, item_category_tensor=c1.categories,
                                         major_category_id=c1.major, batch_hook=Streams(c1, ep))
        epochs.append(float(mean))
    m32 = build_oracle_model(c1)
    m32.load_state_dict({k: v.float() for k, v in model.state_dict().items()})
    return m32, epochs, None


def run(variant: str, c1) -> dict:
    orig = ref._linear
    torch.set_num_threads(1 if variant == "threads1" else 8)
    if variant == "splitk2":
        ref._linear = _splitk_linear(orig)
    try:
        t0 = time.time()
        model, epochs, _ = _train_float64(c1) if variant == "float64" else train_oracle(c1, EPOCHS)
        secs = time.time() - t0
    finally:
        ref._linear = orig
    torch.set_num_threads(8)
    preds, truth = ref.evaluate_model(model, train_positive_map=c1.train_positive_map, val_pairs=c1.val_pairs,
                                      item_features=c1.item_features, user_features=c1.user_features,
                                      num_items=c1.num_items, k_values=K_VALUES, faiss_search_k=max(K_VALUES) * 4,
                                      normalize=True)
    m = ref.ranking_metrics(preds, truth, K_VALUES)
    out = {"recall": {str(k): float(m.recall[k]) for k in K_VALUES}, "epoch_means": epochs,
           "train_seconds": round(secs, 1)}
    print(variant, json.dumps(out), flush=True)
    return out


FP32_VARIANTS = ("threads8", "threads1", "splitk2")


def main() -> None:
    c1 = load_c1("c1_large")
    path = HERE / "c1_large" / "oracle_recall.json"
    if len(sys.argv) > 2 and sys.argv[1] == "--only":
        doc = json.loads(path.read_text())
        doc["variants"][sys.argv[2]] = run(sys.argv[2], c1)
        path.write_text(json.dumps(doc, indent=1) + "\n")
        return
    res = {v: run(v, c1) for v in FP32_VARIANTS + ("float64",)}
    r20 = [res[v]["recall"]["20"] for v in FP32_VARIANTS]
    doc = {
        "fixture": "tests/golden/c1_large (make_c1_fixture.py --large)",
        "epochs": EPOCHS,
        "val_users": len(c1.val_pairs),
        "variants": res,
        "reference_recall20": res["threads8"]["recall"]["20"],
        "oracle_spread_recall20": max(r20) - min(r20),
        "torch": torch.__version__,
    }
    path.write_text(json.dumps(doc, indent=1) + "\n")
    print(json.dumps(doc))


if __name__ == "__main__":
    main()
