"""The reference's tower options in the row-sharded step (ttamm/sharded.py), in loopback on one
GPU against the one-process fused step over the global batch (as tests/test_sharded_gpu.py):
padding_idx (the padding row local to its owner), max_norm ID tables (the owner renorms every
requester's positives, then their negatives), gradient_clip_norm (the table updates wait for the
all-reduced global norm), the category-alignment loss over the global batch (per-category sums
and centered scatters all-reduced between TTAMM_PHASE_CAL_STATS / CAL_SCATTER, the reference's
default loss weight raised so its gradient is visible).  One step at lr = 0 / betas (0, 0.999) — every gradient at 1e-5 — and
three real steps — parameters within 5e-5 absolute."""

from __future__ import annotations

import dataclasses

import pytest
import torch

import ttamm
from helpers import LOSS_WEIGHTS, Shape, make_problem, named_optimizer_state, rel_err
from ttamm.sharded import RowOwnership, ShardedTrainStep, run_loopback

pytestmark = pytest.mark.gpu

TABLES = ("user_encoder.embedding.weight", "item_encoder.embedding.weight",
          "adaptive_mimic.user_augmented.weight", "adaptive_mimic.item_augmented.weight")
SEED = 4242


def _model(cfg, shape: Shape, U: int, I: int, state: dict):
    ue = ttamm.build_tower_encoder(cfg, num_embeddings=U, feature_dim=shape.F, device="cuda")
    ie = ttamm.build_tower_encoder(cfg, num_embeddings=I, feature_dim=shape.F, device="cuda")
    mm = ttamm.AdaptiveMimicMechanism(num_users=U, num_items=I, embedding_dim=shape.P).cuda()
    m = ttamm.TwoTowerModel(ue, ie, similarity=ttamm.DotProductSimilarity(), adaptive_mimic=mm)
    m.load_state_dict({k: v.cuda() for k, v in state.items()}, strict=True)
    return m


def _opts(model, lr, betas, sgd: bool = False):
    dense, sparse = ttamm._collect_parameter_groups(model)
    if sgd:  # torch.optim.SGD with momentum, dampening, coupled L2 (training.py:1311-1333's other choice)
        opts = [torch.optim.SGD(dense, lr=1e-3, momentum=0.9, dampening=0.1, weight_decay=0.01)]
    else:
        opts = [torch.optim.AdamW(dense, lr=1e-3, weight_decay=0.01, betas=betas)]
    if sparse:
        opts.append(torch.optim.SparseAdam(sparse, lr=1e-3, betas=betas))
    for o in opts:
        for g in o.param_groups:
            g["lr"] = lr
    return opts


def _shard_cfg(shape: Shape, own: RowOwnership) -> dict:
    cfg = shape.tower_cfg()
    params = dict(cfg["id_embedding"]["params"])
    if shape.padding_idx is not None:
        local = own.local_padding_idx(shape.padding_idx)
        if local is None:
            params.pop("padding_idx", None)
        else:
            params["padding_idx"] = local
    cfg["id_embedding"] = {**cfg["id_embedding"], "params": params}
    return cfg


CAL_WEIGHTS = {**LOSS_WEIGHTS, "category_alignment": 2.0}
C32 = dict(D=32, H=32, hidden_dims=(32,))  # D = Hg = 32: the fused gate, compact exchange rows


def _categories(I: int, C: int = 4, major_share: float = 0.4, seed: int = 9) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    cats = torch.randint(1, C, (I,), generator=g)
    cats[torch.rand(I, generator=g) < major_share] = 0
    return cats


def _run(shape: Shape, W: int, *, lr: float, betas, steps: int, clip: float | None, cal: bool = False,
         sgd: bool = False):
    prob = make_problem(shape, seed=77)
    lw = CAL_WEIGHTS if cal else LOSS_WEIGHTS
    cat_kw = dict(item_category_tensor=_categories(shape.I).cuda(), major_category_id=0) if cal else {}
    state = prob.model.state_dict()
    gen = torch.Generator().manual_seed(5)
    batches = []
    for _ in range(steps):
        per_rank = []
        for r in range(W):
            owned = torch.arange(r, shape.U, W)
            users = owned[torch.randint(0, owned.numel(), (shape.B,), generator=gen)]
            if shape.padding_idx is not None and shape.padding_idx % W == r:
                users[:2] = shape.padding_idx  # the padding id among this rank's users
            pos = torch.tensor([sorted(prob.positives[int(u)])[0] for u in users], dtype=torch.long)
            if shape.padding_idx is not None and r == 0:
                pos[2] = shape.padding_idx  # ... and among the positives
            per_rank.append((users, pos))
        batches.append(per_rank)
    gm = _model(shape.tower_cfg(), shape, shape.U, shape.I, state)
    gopts = _opts(gm, lr, betas, sgd)
    geng = ttamm.FusedTrainStep(gm, gopts, negatives_per_positive=shape.N, positives=prob.positives,
                                user_features=prob.user_features.cuda(), item_features=prob.item_features.cuda(),
                                loss_weights=lw, max_batch=W * shape.B, seed=SEED, gradient_clip_norm=clip,
                                **cat_kw)
    ranks = []
    for r in range(W):
        own = RowOwnership(W, r)
        st = {k: (own.shard(v) if k in TABLES else v.clone()) for k, v in state.items()}
        m = _model(_shard_cfg(shape, own), shape, own.local_count(shape.U), own.local_count(shape.I), st)
        opts = _opts(m, lr, betas, sgd)
        local_pos = {u // W: prob.positives[u] for u in range(r, shape.U, W)}
        eng = ShardedTrainStep(m, opts, world_size=W, rank=r, num_items=shape.I, negatives_per_positive=shape.N,
                               positives=local_pos, user_features=own.shard(prob.user_features).cuda(),
                               item_features=own.shard(prob.item_features).cuda(), loss_weights=lw,
                               max_batch=shape.B, seed=SEED, gradient_clip_norm=clip, **cat_kw)
        ranks.append((own, m, opts, eng))
    glosses, rlosses = [], []
    for per_rank in batches:
        geng.step(torch.cat([u for u, _ in per_rank]).cuda(), torch.cat([p for _, p in per_rank]).cuda())
        glosses.append(geng.last_losses())
        run_loopback([eng.program((u // W).cuda(), p.cuda()) for (_, _, _, eng), (u, p) in zip(ranks, per_rank)])
        rlosses.append([eng.last_losses() for (_, _, _, eng) in ranks])
    geng.finish()
    run_loopback([eng.finish_program() for (_, _, _, eng) in ranks])
    return (gm, gopts), ranks, glosses, rlosses


CASES = [
    (2, Shape(padding_idx=5), None, False),
    (3, Shape(sparse=False, padding_idx=4), None, False),
    (2, Shape(sparse=False, max_norm=0.05), None, False),
    (3, Shape(sparse=False, max_norm=0.05, N=3), None, False),
    (2, Shape(sparse=False), 0.05, False),
    (3, Shape(sparse=False), 100.0, False),
    (2, Shape(sparse=False, max_norm=0.05, padding_idx=6), 0.05, False),
    (2, Shape(), None, True),
    (3, Shape(N=3), None, True),
    (3, Shape(sparse=False, max_norm=0.05, padding_idx=6), 0.05, True),
    (2, Shape(fusion="concat", feature_out=12, concat_out=20), None, True),
    # the fused gate widths: compact exchange rows (ttamm.h exchange_counts) under every option
    (2, Shape(padding_idx=5, **C32), None, False),
    (3, Shape(sparse=False, max_norm=0.05, N=3, **C32), None, False),
    (2, Shape(sparse=False, **C32), 0.05, False),
    (3, Shape(N=3, **C32), None, True),
    (3, Shape(sparse=False, max_norm=0.05, padding_idx=6, **C32), 0.05, True),
]
IDS = ["padding-w2", "dense-padding-w3", "max-norm-w2", "max-norm-w3", "clip-w2", "noclip-w3", "all-w2",
       "cal-w2", "cal-w3", "cal-all-w3", "concat-out20-cal-w2", "padding-w2-compact", "max-norm-w3-compact",
       "clip-w2-compact", "cal-w3-compact", "cal-all-w3-compact"]


@pytest.mark.parametrize("W,shape,clip,cal", CASES, ids=IDS)
def test_sharded_options_gradients_match_global_step(W, shape, clip, cal):
    (gm, gopts), ranks, gl, rl = _run(shape, W, lr=0.0, betas=(0.0, 0.999), steps=1, clip=clip, cal=cal)
    assert all(eng.compact == (shape.D == 32) for (_, _, _, eng) in ranks)
    if cal:
        assert gl[0]["category_alignment"] > 0
    for key in ("total", "bce", "mimic_user", "mimic_item", "category_alignment"):
        for r in range(W):
            assert abs(rl[0][r][key] - gl[0][key]) <= 1e-5 * max(abs(gl[0][key]), 1e-12), (key, rl[0][r][key], gl[0][key])
    gstate = named_optimizer_state(gm, gopts)
    for own, m, opts, _ in ranks:
        for name, st in named_optimizer_state(m, opts).items():
            want = gstate[name]["exp_avg"]
            if name in TABLES:
                want = want[own.rank:: W]
            assert rel_err(st["exp_avg"], want) <= 1e-5, (own.rank, name)
    if shape.max_norm is not None:  # the renorm acted on the looked-up rows of every shard alike
        gsd = gm.state_dict()
        for own, m, _, _ in ranks:
            for k in ("user_encoder.embedding.weight", "item_encoder.embedding.weight"):
                assert rel_err(m.state_dict()[k], gsd[k][own.rank:: W]) <= 1e-6, (own.rank, k)


@pytest.mark.parametrize("W,shape,clip,cal", [CASES[0], CASES[3], CASES[4], CASES[6], CASES[8], CASES[9], CASES[14],
                                              CASES[15]],
                         ids=["padding-w2", "max-norm-w3", "clip-w2", "all-w2", "cal-w3", "cal-all-w3", "cal-w3-compact",
                              "cal-all-w3-compact"])
def test_sharded_options_three_steps_match_global_step(W, shape, clip, cal):
    (gm, _), ranks, gl, rl = _run(shape, W, lr=1e-3, betas=(0.9, 0.999), steps=3, clip=clip, cal=cal)
    for s in range(3):
        assert abs(rl[s][0]["total"] - gl[s]["total"]) <= 1e-5 * abs(gl[s]["total"])
    gsd = gm.state_dict()
    for own, m, _, _ in ranks:
        for k, v in m.state_dict().items():
            want = gsd[k][own.rank:: W] if k in TABLES else gsd[k]
            d = (v - want).abs().max().item()
            assert d <= 5e-5, f"rank {own.rank} {k}: {d:.2e}"
    if shape.padding_idx is not None and shape.sparse:  # SparseAdam never touched the padding row
        own = RowOwnership(W, shape.padding_idx % W)
        m = ranks[own.rank][1]
        init = make_problem(shape, seed=77).model.state_dict()
        for n in ("user_encoder.embedding.weight", "item_encoder.embedding.weight"):
            assert torch.equal(m.state_dict()[n][shape.padding_idx // W].cpu(), init[n][shape.padding_idx]), n


@pytest.mark.parametrize("W,shape,clip", [(2, Shape(), None), (3, Shape(sparse=False, max_norm=0.05), 0.05)],
                         ids=["sparse-w2", "dense-clip-w3"])
def test_sharded_sgd_three_steps_match_global_step(W, shape, clip):
    """The dense group under SGD (momentum buffers written by the first step, then damped): every
    rank's replicated dense parameters and its table shard follow the global step's."""
    (gm, gopts), ranks, gl, rl = _run(shape, W, lr=0.05, betas=(0.9, 0.999), steps=3, clip=clip, sgd=True)
    for s in range(3):
        assert abs(rl[s][0]["total"] - gl[s]["total"]) <= 1e-5 * abs(gl[s]["total"])
    gsd = gm.state_dict()
    gstate = named_optimizer_state(gm, gopts)
    for own, m, opts, _ in ranks:
        for k, v in m.state_dict().items():
            want = gsd[k][own.rank:: W] if k in TABLES else gsd[k]
            d = (v - want).abs().max().item()
            assert d <= 5e-5, f"rank {own.rank} {k}: {d:.2e}"
        for name, st in named_optimizer_state(m, opts).items():
            if "momentum_buffer" in st:
                want = gstate[name]["momentum_buffer"]
                want = want[own.rank:: W] if name in TABLES else want
                assert rel_err(st["momentum_buffer"], want) <= 1e-4, (own.rank, name)


def test_sharded_clipping_needs_grouped_schedule():
    prob = make_problem(Shape(sparse=False), seed=1)
    m = _model(Shape(sparse=False).tower_cfg(), Shape(sparse=False), 32, 128, {
        k: (v[0::2].contiguous() if k in TABLES else v) for k, v in prob.model.state_dict().items()})
    with pytest.raises(NotImplementedError, match="group_towers"):
        ShardedTrainStep(m, _opts(m, 1e-3, (0.9, 0.999)), world_size=2, rank=0, num_items=256, negatives_per_positive=5,
                         positives=None, user_features=prob.user_features[0::2].cuda(),
                         item_features=prob.item_features[0::2].cuda(), max_batch=32, gradient_clip_norm=1.0,
                         group_towers=False)
