"""Developer diagnostic: the C1-large oracle trained in float64 (model,
optimizer state and features; every other input identical to tests/test_c1_gpu.py), to locate
where ttamm's epoch means sit between the fp32 oracle and the float64 trajectory.

    python tools/diag/c1_large_fp64.py   (~5 minutes on 8 cores)
"""
import json
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "tests"), str(ROOT)]
from c1_helpers import K_VALUES, LOSS_WEIGHTS, N, Streams, build_oracle_model, load_c1, loader  # noqa: E402
from oracle import cpu_reference as ref  # noqa: E402

torch.set_num_threads(8)
c1 = load_c1("c1_large")
model = build_oracle_model(c1).double()
opts = ref.build_optimizers(model, lr=1e-3, weight_decay=0.01)
uf, itf = c1.user_features.double(), c1.item_features.double()
means = []
t0 = time.time()
for ep in range(3):
    mean, _, _ = ref.train_one_epoch(model, loader(c1, ep), opts, negatives_per_positive=N, num_items=c1.num_items,
                                     positives=c1.positives, user_features=uf, item_features=itf,
                                     loss_weights=LOSS_WEIGHTS, item_category_tensor=c1.categories,
                                     major_category_id=c1.major, batch_hook=Streams(c1, ep))
    means.append(float(mean))
    print(f"epoch {ep} mean {mean:.9f}  ({time.time() - t0:.0f} s)", flush=True)
m32 = build_oracle_model(c1)
m32.load_state_dict({k: v.float() for k, v in model.state_dict().items()})
preds, truth = ref.evaluate_model(m32, train_positive_map=c1.train_positive_map, val_pairs=c1.val_pairs,
                                  item_features=c1.item_features, user_features=c1.user_features,
                                  num_items=c1.num_items, k_values=K_VALUES, faiss_search_k=max(K_VALUES) * 4,
                                  normalize=True)
r = ref.ranking_metrics(preds, truth, K_VALUES).recall
print(json.dumps({"float64_epoch_means": means, "recall": {str(k): float(r[k]) for k in K_VALUES}}))
