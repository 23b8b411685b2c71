"""BASELINE config C1 end to end through the drop-in entry point (north_star: "Recall@20 within
±0.002 of the CPU reference on the trimmed dataset").

Both sides start from the same weights (the reference's seeded init order) and train EPOCHS
epochs on the joinable C1 fixture through the reference's loop shape: a torch DataLoader with
shuffle=True, drop_last=False (21,244 training pairs at batch 256: 82 full batches and a short
one of 252), one `train_one_epoch` call per epoch, the category-alignment loss on (λ = 0.01).
Negatives and dropout masks come from one injected hook (tests/c1_helpers.Streams).

Checked:
  * every step's total loss: ttamm vs oracle, relative 1e-5 through the whole first epoch (measured
    max 2.0e-7).  Later steps drift apart by fp32 summation-order rounding that Adam amplifies
    (an update is ~lr whatever the gradient's size, so a near-zero gradient's rounding decides a
    whole lr step): the oracle run with 1 vs 8 CPU threads — the reference path against itself —
    drifts the same way (per-step max 1.6e-6 in epoch 2, 2.3e-4 in epoch 3; epoch-3 mean 3.1e-6).
    ttamm vs oracle: 1.4e-5, 3.2e-4; 7e-6 with the fp32-MFMA GEMMs (TTAMM_FP32_MFMA=exact), and
    1.7e-4, 8.2e-4; 8.5e-5 with the default split-bf16 GEMMs — which are as accurate as the fp32
    MFMA against fp64 (csrc/tools/gemm_bench: max |err| / max |C| 9.4e-7 vs 9.5e-7 on the
    608-deep layer-1 GEMM), so the larger later-epoch gap is the chaos growing from a different
    rounding pattern, not a less accurate step.  Bounds: epoch 1 as above, 1e-3 per step after,
    2e-4 on the later epochs' means;
  * Recall@20 of the ttamm-trained model vs the oracle-trained model, both evaluated by the CPU
    restatement of _evaluate_model (exact-IP / FAISS branch, cosine): |Δ| <= 0.002;
  * ttamm's own GPU retrieval (ttamm.evaluate_model) on the ttamm-trained weights gives the same
    Recall@20 as the CPU evaluation of those weights (|Δ| <= 0.002), with and without
    prepare_faiss_resources;
  * the no-FAISS sampled-candidate branch (training.py:974-1009): ttamm's batched
    candidate_topk vs the oracle's per-user loop on the same weights and the same rng stream.
"""

from __future__ import annotations

import pytest
import torch
from torch import nn

import ttamm
from c1_helpers import (K_VALUES, LOSS_WEIGHTS, N, TOWER_CFG, Streams, build_oracle_model, load_c1, loader, recall_at,
                        train_oracle)
from oracle import cpu_reference as ref

pytestmark = pytest.mark.gpu

EPOCHS = 3


def _ttamm_model(c1):
    om = build_oracle_model(c1)
    dev = torch.device("cuda")
    cfg = dict(TOWER_CFG)
    ue = ttamm.build_tower_encoder(cfg, num_embeddings=c1.num_users, feature_dim=c1.user_features.shape[1], device=dev)
    ie = ttamm.build_tower_encoder(cfg, num_embeddings=c1.num_items, feature_dim=c1.item_features.shape[1], device=dev)
    mm = ttamm.AdaptiveMimicMechanism(num_users=c1.num_users, num_items=c1.num_items, embedding_dim=ue.output_dim).to(dev)
    model = ttamm.TwoTowerModel(ue, ie, similarity=nn.CosineSimilarity(dim=-1), adaptive_mimic=mm)
    res = model.load_state_dict({k: v.to(dev) for k, v in om.state_dict().items()}, strict=True)
    assert not res.missing_keys and not res.unexpected_keys
    return model


@pytest.fixture(scope="module")
def trained():
    c1 = load_c1()
    om, o_epochs, o_steps = train_oracle(c1, EPOCHS)
    model = _ttamm_model(c1)
    dense, sparse = ttamm._collect_parameter_groups(model)
    opts = [torch.optim.AdamW(dense, lr=1e-3, weight_decay=0.01), torch.optim.SparseAdam(sparse, lr=1e-3)]
    dev = torch.device("cuda")
    uf, itf = c1.user_features.to(dev), c1.item_features.to(dev)
    t_epochs, t_steps = [], []
    for ep in range(EPOCHS):
        t_epochs.append(ttamm.train_one_epoch(
            model, loader(c1, ep), optimizers=opts, criterion=nn.BCEWithLogitsLoss(), negatives_per_positive=N,
            num_items=c1.num_items, user_positive_items=c1.positives, user_features=uf, item_features=itf,
            device=dev, gradient_clip_norm=None, loss_weights=LOSS_WEIGHTS,
            item_category_tensor=c1.categories.to(dev), major_category_id=c1.major,
            batch_hook=Streams(c1, ep), step_losses=t_steps))
    t_steps = [float(v[0]) for v in torch.stack(t_steps).cpu()]
    tm_cpu = build_oracle_model(c1)
    tm_cpu.load_state_dict({k: v.detach().cpu() for k, v in model.state_dict().items()})
    return dict(c1=c1, om=om, o_epochs=o_epochs, o_steps=o_steps, model=model, opts=opts, dense=dense, sparse=sparse,
                t_epochs=t_epochs, t_steps=t_steps, tm_cpu=tm_cpu, uf=uf, itf=itf, dev=dev)


def test_c1_drop_in_losses_match_oracle(trained):
    o_steps, t_steps = trained["o_steps"], trained["t_steps"]
    o_epochs, t_epochs = trained["o_epochs"], trained["t_epochs"]
    steps_per_epoch = len(o_steps) // EPOCHS
    assert len(t_steps) == len(o_steps) == EPOCHS * 83  # 82 full batches + the short last one (252)
    rel = [abs(t - o) / abs(o) for t, o in zip(t_steps, o_steps)]
    first = max(rel[:steps_per_epoch])
    print(f"\nC1 per-step total loss rel diff: epoch 1 max {first:.2e}, all epochs max {max(rel):.2e}")
    print(f"epoch means oracle {o_epochs} ttamm {t_epochs}")
    for e in range(EPOCHS):
        seg = rel[e * steps_per_epoch:(e + 1) * steps_per_epoch]
        print(f"epoch {e}: max {max(seg):.2e} median {sorted(seg)[len(seg) // 2]:.2e}")
    assert first <= 1e-5, first
    assert max(rel) <= 1e-3, max(rel)
    for t, o in zip(t_epochs, o_epochs):
        assert abs(t - o) <= 2e-4 * abs(o)
    assert abs(t_epochs[0] - o_epochs[0]) <= 1e-5 * abs(o_epochs[0])
    # optimizer step counters written back like torch's
    opts, dense, sparse = trained["opts"], trained["dense"], trained["sparse"]
    assert float(opts[0].state[dense[0]]["step"]) == float(EPOCHS * steps_per_epoch)
    assert opts[1].state[sparse[0]]["step"] == EPOCHS * steps_per_epoch


def test_c1_recall_at_20_matches_oracle(trained):
    c1, model, dev = trained["c1"], trained["model"], trained["dev"]
    r_oracle = recall_at(trained["om"], c1)
    r_ttamm = recall_at(trained["tm_cpu"], c1)
    print(f"\nRecall@20 oracle-trained {r_oracle:.6f}  ttamm-trained {r_ttamm:.6f}")
    assert r_oracle > 0.2  # the planted structure is learned (untrained: ~0.007)
    assert abs(r_ttamm - r_oracle) <= 0.002
    # ttamm's own GPU retrieval on the same weights: full-corpus search, and through the
    # prepare_faiss_resources drop-in (training.py:646-679 -> :1522-1535)
    kw = dict(train_positive_map=c1.train_positive_map, val_interactions=c1.val_pairs,
              item_feature_tensor=trained["itf"], user_feature_tensor=trained["uf"], device=dev,
              num_items=c1.num_items, k_values=K_VALUES, faiss_search_k=80)
    r_gpu = ref.ranking_metrics(*ttamm.evaluate_model(model, **kw), K_VALUES).recall[20]
    res = ttamm.prepare_faiss_resources(model, num_items=c1.num_items, item_features=trained["itf"], device=dev)
    assert res["normalize"]
    r_res = ref.ranking_metrics(*ttamm.evaluate_model(model, faiss_resources=res, **kw), K_VALUES).recall[20]
    print(f"Recall@20 ttamm-trained, GPU retrieval {r_gpu:.6f} (via faiss_resources {r_res:.6f})")
    assert abs(r_gpu - r_ttamm) <= 0.002
    assert r_res == r_gpu


def test_c1_sampled_candidate_branch_matches_oracle(trained):
    """No faiss (the branch a reference run takes in this image): ground truth + 50 sampled
    candidates per user (configs/default.yaml:92), rng = default_rng(seed * 997 + epoch)
    (training.py:1521), cosine scores, top-k."""
    import numpy as np

    c1, model, dev = trained["c1"], trained["model"], trained["dev"]
    seed = 1234 * 997 + 3
    preds_t, truth_t = ttamm.evaluate_model(
        model, train_positive_map=c1.train_positive_map, val_interactions=c1.val_pairs,
        item_feature_tensor=trained["itf"], user_feature_tensor=trained["uf"], device=dev, num_items=c1.num_items,
        candidate_samples=50, k_values=K_VALUES, rng=np.random.default_rng(seed))
    preds_o, truth_o = ref.evaluate_model_sampled(
        trained["tm_cpu"], train_positive_map=c1.train_positive_map, val_pairs=c1.val_pairs,
        item_features=c1.item_features, user_features=c1.user_features, num_items=c1.num_items, k_values=K_VALUES,
        candidate_samples=50, rng=np.random.default_rng(seed), cosine=True)
    assert truth_t == truth_o and preds_t.keys() == preds_o.keys()
    same = sum(preds_t[u] == preds_o[u] for u in preds_o)
    print(f"\nsampled branch: identical top-{max(K_VALUES)} lists for {same}/{len(preds_o)} users")
    assert same >= 0.99 * len(preds_o)
    mt, mo = ref.ranking_metrics(preds_t, truth_t, K_VALUES), ref.ranking_metrics(preds_o, truth_o, K_VALUES)
    for k in K_VALUES:
        assert abs(mt.recall[k] - mo.recall[k]) <= 0.002, (k, mt.recall[k], mo.recall[k])
    assert mo.recall[20] > 0.5  # 50 sampled candidates: an easier ranking than the full corpus


def test_c1_large_recall_at_20_within_oracle_band():
    """The Recall@20 gate at a resolution that separates training agreement from summation order
    (VERDICT r04): the C1-schema fixture at 20,000 users (tests/golden/c1_large, one validation
    pair each, so +-0.002 is 40 users; make_c1_fixture.py --large), trained EPOCHS epochs through
    ttamm.train_one_epoch exactly like the oracle runs committed in
    tests/golden/c1_large/oracle_recall.json (make_c1_large_oracle.py: the CPU restatement with 8
    threads = the reference value, with 1 thread, and with the first layer's K reduction split in
    two — summation-order-only variants whose Recall@20 spread is recorded there — and in float64).
    ttamm's Recall@20 (CPU evaluation of its weights, the same restated _evaluate_model) must lie
    within 0.002 of the reference value, and its epoch-1 mean as close to the float64 trajectory
    as the fp32 reference runs are (below)."""
    import json
    from pathlib import Path

    doc = json.loads((Path(__file__).resolve().parent / "golden" / "c1_large" / "oracle_recall.json").read_text())
    assert doc["epochs"] == EPOCHS and doc["oracle_spread_recall20"] < 0.002
    c1 = load_c1("c1_large")
    model = _ttamm_model(c1)
    dense, sparse = ttamm._collect_parameter_groups(model)
    opts = [torch.optim.AdamW(dense, lr=1e-3, weight_decay=0.01), torch.optim.SparseAdam(sparse, lr=1e-3)]
    dev = torch.device("cuda")
    uf, itf = c1.user_features.to(dev), c1.item_features.to(dev)
    means = []
    for ep in range(EPOCHS):
        means.append(ttamm.train_one_epoch(
            model, loader(c1, ep), optimizers=opts, criterion=nn.BCEWithLogitsLoss(), negatives_per_positive=N,
            num_items=c1.num_items, user_positive_items=c1.positives, user_features=uf, item_features=itf,
            device=dev, gradient_clip_norm=None, loss_weights=LOSS_WEIGHTS,
            item_category_tensor=c1.categories.to(dev), major_category_id=c1.major, batch_hook=Streams(c1, ep)))
    tm_cpu = build_oracle_model(c1)
    tm_cpu.load_state_dict({k: v.detach().cpu() for k, v in model.state_dict().items()})
    r_ttamm = recall_at(tm_cpu, c1)
    ref20 = doc["reference_recall20"]
    variants = {k: v["recall"]["20"] for k, v in doc["variants"].items()}
    print(f"\nC1-large Recall@20: ttamm {r_ttamm:.5f}  oracle {variants}  oracle spread "
          f"{doc['oracle_spread_recall20']:.5f}  |ttamm - oracle| {abs(r_ttamm - ref20):.5f}")
    print(f"epoch means ttamm {means} oracle {doc['variants']['threads8']['epoch_means']}")
    # Epoch means against the float64 trajectory (the "float64" variant: the same run, same streams,
    # in float64 — the arithmetic every fp32 run approximates).  Where an fp32 run's epoch-1 mean
    # lands depends on the KIND of rounding, not only its size: the fp32 CPU runs (threads8 = the
    # reference value, threads1, splitk2) all sit ABOVE the float64 mean by 4.0-6.8e-5, ttamm's
    # split-bf16 GEMMs (exact bf16 products, MFMA sums rounded once per 16 k) BELOW it by 4.0-4.5e-5
    # (with 8 instead of 6 bf16 products per fp32 product: the same), ttamm on the fp32-MFMA kernels
    # (fp32 fma chains like the CPU's, TTAMM_FP32_MFMA=exact) above it by 5.1e-5.  So
    # ttamm vs threads8 (~1.1e-4) is the two sides of the exact trajectory, not a larger error:
    # against float64, ttamm's epoch 1 is as close as the fp32 reference's own runs — the bound is
    # 5e-5.  Later epochs: Adam turns rounding-level differences into lr-sized steps and the
    # trajectories separate chaotically (ttamm builds that differ only in summation order land
    # 1.8e-5 to 2.5e-4 from float64 in epoch 3, the fp32 CPU runs up to 6.3e-5), so they keep the
    # chaos bound 5e-4 and the Recall gate below is the parity claim.
    f64 = doc["variants"]["float64"]["epoch_means"]
    fp32_runs = [doc["variants"][v]["epoch_means"] for v in ("threads8", "threads1", "splitk2")]
    dist = [abs(means[e] - f64[e]) / f64[e] for e in range(EPOCHS)]
    own = [max(abs(v[e] - f64[e]) for v in fp32_runs) / f64[e] for e in range(EPOCHS)]
    print(f"epoch means vs float64: ttamm {['%.2e' % d for d in dist]}  fp32 oracle runs up to "
          f"{['%.2e' % o for o in own]}")
    assert dist[0] <= 5e-5, dist
    assert max(dist) <= 5e-4, dist
    assert abs(r_ttamm - ref20) <= 0.002
