"""The row-sharded multi-GPU step (ttamm/sharded.py) against the one-process step over the
global batch, on one GPU: W virtual ranks run in lock step in this process (run_loopback
serves their all-to-alls / all-reduces), each with its shard of the tables and a replica of
the MLP / gate weights.

A W-rank step is the reference step over the concatenated (rank-major) global batch, so:
  * sampled negatives are bit-identical (Philox streams keyed by global slot);
  * dropout masks are identical (keyed by global request position) — checked implicitly;
  * losses and every gradient agree to 1e-5 norm-wise relative (only fp32 summation order
    differs: per-rank partial sums, then the all-reduce);
  * after three real optimizer steps parameters agree within 5e-5 absolute (golden-test
    tolerance: Adam normalises each update to ~lr)."""

from __future__ import annotations

import pytest
import torch

import ttamm
from helpers import LOSS_WEIGHTS, Shape, make_problem, named_optimizer_state, rel_err
from ttamm.sharded import RowOwnership, ShardedTrainStep, run_loopback

pytestmark = pytest.mark.gpu

TABLES = ("user_encoder.embedding.weight", "item_encoder.embedding.weight",
          "adaptive_mimic.user_augmented.weight", "adaptive_mimic.item_augmented.weight")
SEED = 4242


def _model(shape: Shape, U: int, I: int, state: dict):
    cfg = shape.tower_cfg()
    ue = ttamm.build_tower_encoder(cfg, num_embeddings=U, feature_dim=shape.F, device="cuda")
    ie = ttamm.build_tower_encoder(cfg, num_embeddings=I, feature_dim=shape.F, device="cuda")
    mm = ttamm.AdaptiveMimicMechanism(num_users=U, num_items=I, embedding_dim=shape.D).cuda() if shape.mimic else None
    m = ttamm.TwoTowerModel(ue, ie, similarity=ttamm.DotProductSimilarity(), adaptive_mimic=mm)
    m.load_state_dict({k: v.cuda() for k, v in state.items()}, strict=True)
    return m


def _opts(model, lr, betas):
    dense, sparse = ttamm._collect_parameter_groups(model)
    opts = [torch.optim.AdamW(dense, lr=1e-3, weight_decay=0.01, betas=betas),
            torch.optim.SparseAdam(sparse, lr=1e-3, betas=betas)]
    for o in opts:
        for g in o.param_groups:
            g["lr"] = lr
    return opts


def _setup(shape: Shape, W: int, *, lr: float, betas, steps: int, in_batch: bool = False, group: bool = True):
    prob = make_problem(shape, seed=77)
    state = prob.model.state_dict()
    gen = torch.Generator().manual_seed(5)
    # rank r's interactions use only users it owns (u % W == r); global batch is rank-major
    batches = []
    for _ in range(steps):
        per_rank = []
        for r in range(W):
            owned = torch.arange(r, shape.U, W)
            users = owned[torch.randint(0, owned.numel(), (shape.B,), generator=gen)]
            pos = torch.tensor([sorted(prob.positives[int(u)])[0] for u in users], dtype=torch.long)
            per_rank.append((users, pos))
        batches.append(per_rank)
    # one process over the global batch
    gm = _model(shape, shape.U, shape.I, state)
    gopts = _opts(gm, lr, betas)
    geng = ttamm.FusedTrainStep(gm, gopts, negatives_per_positive=shape.N, positives=prob.positives,
                                user_features=prob.user_features.cuda(), item_features=prob.item_features.cuda(),
                                loss_weights=LOSS_WEIGHTS, max_batch=W * shape.B, seed=SEED,
                                in_batch_negatives=in_batch)
    # W ranks
    ranks = []
    for r in range(W):
        own = RowOwnership(W, r)
        st = {k: (own.shard(v) if k in TABLES else v.clone()) for k, v in state.items()}
        m = _model(shape, own.local_count(shape.U), own.local_count(shape.I), st)
        opts = _opts(m, lr, betas)
        local_pos = {u // W: prob.positives[u] for u in range(r, shape.U, W)}
        eng = ShardedTrainStep(m, opts, world_size=W, rank=r, num_items=shape.I, negatives_per_positive=shape.N,
                               positives=local_pos, user_features=own.shard(prob.user_features).cuda(),
                               item_features=own.shard(prob.item_features).cuda(), loss_weights=LOSS_WEIGHTS,
                               max_batch=shape.B, seed=SEED, in_batch_negatives=in_batch, group_towers=group)
        ranks.append((own, m, opts, eng))
    return prob, batches, (gm, gopts, geng), ranks


def _run(batches, g, ranks, W):
    gm, gopts, geng = g
    glosses, rlosses, negs = [], [], []
    for per_rank in batches:
        users = torch.cat([u for u, _ in per_rank]).cuda()
        pos = torch.cat([p for _, p in per_rank]).cuda()
        geng.step(users, pos)
        glosses.append(geng.last_losses())
        progs = [eng.program((u // W).cuda(), p.cuda()) for (own, m, o, eng), (u, p) in zip(ranks, per_rank)]
        run_loopback(progs)
        rlosses.append([eng.last_losses() for (_, _, _, eng) in ranks])
        negs.append((geng.neg_buffer.clone(), [eng.neg_buffer.clone() for (_, _, _, eng) in ranks]))
    gavg = geng.finish()
    ravg = run_loopback([eng.finish_program() for (_, _, _, eng) in ranks])
    return glosses, rlosses, negs, gavg, ravg


@pytest.mark.parametrize("W,shape,in_batch,group", [
    (2, Shape(), False, True),
    # the overlapped schedule (ITEM_FWD, exchange under USER_FWD, USER, ITEM_BWD)
    (2, Shape(), False, False),
    (3, Shape(N=2), True, False),
    # one rank: no exchange at all (the requester's buffers are the owner's)
    (1, Shape(), False, True),
    (1, Shape(N=2), True, True),
    (3, Shape(hidden_dims=(16, 12)), False, True),
    (2, Shape(dropout=0.0, gate_hidden=20), False, True),
    # in-batch negatives: all-gather of the positives + reduce-scatter of dP (ttamm.h INBATCH phases)
    (2, Shape(N=2), True, True),
    (3, Shape(U=300, I=900, N=0, B=70), True, True),
    # C4 widths (D = 128, MLP 40 -> 64 -> 128: the generic gate path), in-batch, 2 ranks
    (2, Shape(U=200, I=900, F=40, H=64, D=128, B=48, N=0, hidden_dims=(64,)), True, True),
    # C5 arithmetic (bf16 tower GEMMs, D = 64, H = 128) through the sharded phases
    (2, Shape(U=200, I=900, F=37, H=128, D=64, B=40, N=3, hidden_dims=(128,), matmul_dtype="bf16"), False, True),
    # the C4 topology: 8 ranks, in-batch negatives over the all-gathered global batch (Bg = 8 x 256
    # = 2048 positives per user), D = 128 (generic gate path)
    (8, Shape(U=800, I=4000, F=40, H=64, D=128, B=256, N=0, hidden_dims=(64,)), True, True),
    # 8 ranks, sampled negatives (the C2 topology at W = 8), both schedules
    (8, Shape(U=800, I=4000, B=64, N=3), False, True),
    # 8 ranks at C2's widths (605 -> 192 -> 96, the fused D = 96 gate, N = 5), 512 interactions per
    # rank: the production kernels of the rank-of-8 step (3,072 owner rows per rank on average)
    (8, Shape(U=4000, I=40000, F=605, H=192, D=96, B=512, N=5, hidden_dims=(192,)), False, True),
    (8, Shape(U=800, I=4000, B=64, N=3), False, False),
])
def test_sharded_gradients_match_global_step(W, shape, in_batch, group):
    _one_step_check(W, shape, in_batch, group)


def _one_step_check(W, shape, in_batch, group, compact=None):
    prob, batches, g, ranks = _setup(shape, W, lr=0.0, betas=(0.0, 0.999), steps=1, in_batch=in_batch, group=group)
    if compact is not None:
        assert all(eng.compact == compact for (_, _, _, eng) in ranks)
    glosses, rlosses, negs, gavg, ravg = _run(batches, g, ranks, W)
    B, N = shape.B, shape.N
    gneg, rneg = negs[0]
    for r in range(W):
        assert torch.equal(rneg[r][: B * N], gneg[r * B * N:(r + 1) * B * N]), f"rank {r} negatives differ"
    for key in ("total", "bce", "mimic_user", "mimic_item"):
        for r in range(W):
            assert abs(rlosses[0][r][key] - glosses[0][key]) <= 1e-5 * max(abs(glosses[0][key]), 1e-12), key
    for r in range(W):
        assert abs(ravg[r] - gavg) <= 1e-5 * abs(gavg)
    gm, gopts, _ = g
    gstate = named_optimizer_state(gm, gopts)
    for own, m, opts, _ in ranks:
        rstate = named_optimizer_state(m, opts)
        for name, st in rstate.items():
            want = gstate[name]["exp_avg"]
            if name in TABLES:
                want = want[own.rank:: W]
            assert rel_err(st["exp_avg"], want) <= 1e-5, (own.rank, name)


# Compact exchange rows (ttamm.h ttamm_step_args.exchange_counts): with mimic on and the item gate
# on the fused kernels a negative request moves D floats each way (t + a, dT) instead of 2 D.  The
# shapes above mostly run the generic gate (D = 8) and so the 2 D-wide rows; these run the fused
# gate widths (D = Hg = 32 on gate.hip, D = Hg = 128 bf16 on gate16.hip, C2's D = 96).
C32 = dict(D=32, H=32, hidden_dims=(32,))
COMPACT_CASES = [
    (2, Shape(**C32), False, True),
    (2, Shape(**C32), False, False),
    (3, Shape(N=2, **C32), True, False),
    (1, Shape(**C32), False, True),
    (1, Shape(N=2, **C32), True, True),
    (3, Shape(U=300, I=900, N=1, B=70, **C32), True, True),
    (2, Shape(dropout=0.0, **C32), False, True),
    (2, Shape(U=200, I=900, F=37, H=128, D=128, B=40, N=3, hidden_dims=(128,), matmul_dtype="bf16"), False, True),
    (8, Shape(U=800, I=4000, B=64, N=3, **C32), False, False),
    (8, Shape(U=4000, I=40000, F=605, H=192, D=96, B=512, N=5, hidden_dims=(192,)), False, True),
]
COMPACT_IDS = ["w2", "w2-overlapped", "w3-in-batch-overlapped", "w1", "w1-in-batch", "w3-in-batch-n1", "w2-nodrop",
               "w2-bf16-d128", "w8-overlapped", "w8-c2-widths"]


@pytest.mark.parametrize("W,shape,in_batch,group", COMPACT_CASES, ids=COMPACT_IDS)
def test_compact_exchange_matches_global_step(W, shape, in_batch, group):
    _one_step_check(W, shape, in_batch, group, compact=True)


def test_no_negatives_keeps_wide_exchange():
    """In-batch only (num_neg = 0): every request is a positive, both layouts move the same bytes,
    and the step keeps the wide rows (no unit maps)."""
    _one_step_check(2, Shape(U=300, I=900, N=0, B=70, **C32), True, True, compact=False)


@pytest.mark.parametrize("W,shape,in_batch,group", [COMPACT_CASES[i] for i in (0, 2, 7, 8)],
                         ids=[COMPACT_IDS[i] for i in (0, 2, 7, 8)])
def test_wide_exchange_matches_global_step(W, shape, in_batch, group, monkeypatch):
    """TTAMM_WIDE_EXCHANGE=1 keeps the 2 D-wide rows on the same shapes."""
    monkeypatch.setenv("TTAMM_WIDE_EXCHANGE", "1")
    _one_step_check(W, shape, in_batch, group, compact=False)


def test_compact_exchange_payload():
    """The rank-of-8 exchange at C2's widths: each rank's (dT | dA) send is D (B (1 + N) + B) floats
    — its B positives two units, its B N negatives one — against the wide rows' 2 D B (1 + N), a
    (2 + N) / (2 + 2 N) share (C2, B = 8192, N = 5, D = 96: 37.7 -> 22.0 MB per rank per direction);
    the owners' (t | a) sends add up to the same total."""
    W, shape = 8, COMPACT_CASES[-1][1]
    prob, batches, g, ranks = _setup(shape, W, lr=0.0, betas=(0.0, 0.999), steps=1)
    _run(batches, g, ranks, W)
    B, N, D = shape.B, shape.N, shape.D
    sends = [eng.exchange_floats for (_, _, _, eng) in ranks]
    assert all(eng.compact for (_, _, _, eng) in ranks)
    assert all(bwd == D * (B * (1 + N) + B) for _, bwd in sends)
    assert sum(fwd for fwd, _ in sends) == sum(bwd for _, bwd in sends)
    assert sends[0][1] * (2 + 2 * N) == 2 * D * B * (1 + N) * (2 + N)


@pytest.mark.parametrize("group", [True, False], ids=["grouped", "overlapped"])
@pytest.mark.parametrize("in_batch", [False, True], ids=["sampled", "in-batch"])
def test_sharded_three_steps_match_global_step(in_batch, group):
    W, shape = 2, Shape()
    prob, batches, g, ranks = _setup(shape, W, lr=1e-3, betas=(0.9, 0.999), steps=3, in_batch=in_batch, group=group)
    glosses, rlosses, _, _, _ = _run(batches, g, ranks, W)
    for s in range(3):
        assert abs(rlosses[s][0]["total"] - glosses[s]["total"]) <= 1e-5 * abs(glosses[s]["total"])
    gm = g[0]
    gsd = gm.state_dict()
    for own, m, _, _ in ranks:
        for k, v in m.state_dict().items():
            want = gsd[k][own.rank:: W] if k in TABLES else gsd[k]
            d = (v - want).abs().max().item()
            assert d <= 5e-5, f"rank {own.rank} {k}: {d:.2e}"


@pytest.mark.parametrize("W,in_batch,group,d32", [(2, False, True, False), (3, True, True, False),
                                                 (2, False, False, False), (8, False, True, False),
                                                 (2, False, True, True), (3, True, False, True), (8, False, True, True)],
                         ids=["w2", "w3-in-batch", "w2-overlapped", "w8", "w2-compact", "w3-in-batch-overlapped-compact",
                              "w8-compact"])
def test_look_ahead_routing_matches_global_step(W, in_batch, group, d32):
    """program(next_batch=...): each step draws the next step's negatives, groups its requests
    and exchanges its counts after the forward exchange (look-ahead routing).  Three steps
    against the one-process step over the global batches: the same losses and final state as
    test_sharded_three_steps_match_global_step, and the look-ahead's draws are the ones the
    one-process sampler makes (Philox keyed by global slot and step)."""
    shape = Shape(N=2, **(C32 if d32 else {})) if in_batch else Shape(**(C32 if d32 else {}))
    prob, batches, g, ranks = _setup(shape, W, lr=1e-3, betas=(0.9, 0.999), steps=3, in_batch=in_batch, group=group)
    assert all(eng.compact == d32 for (_, _, _, eng) in ranks)  # (the look-ahead's count rows carry positives)
    gm, gopts, geng = g
    dev = [[((u // W).cuda(), p.cuda()) for (u, p) in per_rank] for per_rank in batches]
    for s, per_rank in enumerate(batches):
        users = torch.cat([u for u, _ in per_rank]).cuda()
        pos = torch.cat([p for _, p in per_rank]).cuda()
        geng.step(users, pos)
        gl = geng.last_losses()
        gneg = geng.neg_buffer.clone()
        progs = [eng.program(*dev[s][r], next_batch=dev[s + 1][r] if s + 1 < len(batches) else None)
                 for r, (own, m, o, eng) in enumerate(ranks)]
        run_loopback(progs)
        for r, (_, _, _, eng) in enumerate(ranks):
            assert abs(eng.last_losses()["total"] - gl["total"]) <= 1e-5 * abs(gl["total"]), (s, r)
            if s > 0:  # this step ran on the look-ahead's negatives
                B, N = shape.B, shape.N
                got = torch.from_numpy(eng._ahead_bufs[(s - 1) % 2][: B * N].cpu().numpy())
                assert torch.equal(got, gneg[r * B * N:(r + 1) * B * N].cpu()), (s, r)
    gavg = geng.finish()
    ravg = run_loopback([eng.finish_program() for (_, _, _, eng) in ranks])
    for r in range(W):
        assert abs(ravg[r] - gavg) <= 1e-5 * abs(gavg)
    gsd = gm.state_dict()
    for own, m, _, _ in ranks:
        for k, v in m.state_dict().items():
            want = gsd[k][own.rank:: W] if k in TABLES else gsd[k]
            d = (v - want).abs().max().item()
            assert d <= 5e-5, f"rank {own.rank} {k}: {d:.2e}"


def test_bench_two_ranks_one_gpu_gloo():
    """The real multi-process path (torch.distributed.run, TorchComm, ShardedTrainStep, bench
    timing) with 2 ranks on one GPU; gloo stages the exchanges through the host because RCCL
    needs one GPU per rank.  The 8-GPU RCCL run is the driver's."""
    import json
    import socket
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}", str(root / "bench.py"), "--gpus", "2",
           "--config", "tiny", "--dist-backend", "gloo", "--no-cpu-baseline", "--steps", "3", "--warmup", "1"]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=root)
    assert res.returncode == 0, res.stderr[-3000:]
    line = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1
    out = json.loads(line[0])
    assert out["n_gpus"] == 2 and out["value"] > 0 and out["scaling"] == "weak"
    assert "row-sharded" in out["config"]["parallelism"]
    assert out["final_loss"] == out["final_loss"]  # finite, not NaN


def test_bench_gpus_two_self_launches():
    """`bench.py --gpus 2` with no external launcher starts the two ranks itself (a child
    torch.distributed.run) and relays rank 0's line, which must say n_gpus = 2."""
    import json
    import os
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, str(root / "bench.py"), "--gpus", "2", "--config", "tiny", "--dist-backend", "gloo",
           "--no-cpu-baseline", "--steps", "3", "--warmup", "1"]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=root, env=env)
    assert res.returncode == 0, res.stderr[-3000:]
    line = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1
    out = json.loads(line[0])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 2 * 1024 and out["value"] > 0


def test_sharded_epoch_routes_pairs_to_user_owners():
    """ttamm.sharded.epoch_program: every rank reads its own slice of the interaction stream
    (any users); each batch's pairs go to their users' owners by all-to-all and the routed
    batches (different sizes per rank) make one global step.  Against the one-process step fed
    the same global batches (the routed pairs, rank-major): the same epoch loss and, after three
    real optimizer steps, the same parameters (5e-5 absolute, as the three-step test)."""
    from ttamm.sharded import epoch_program

    W, shape, steps, b = 2, Shape(), 3, 24
    prob = make_problem(shape, seed=91)
    state = prob.model.state_dict()
    gen = torch.Generator().manual_seed(8)
    users = torch.randint(0, shape.U, (W * steps * b,), generator=gen)
    items = torch.tensor([sorted(prob.positives[int(u)])[0] for u in users], dtype=torch.long)
    # rank r reads pairs r, r + W, ...; step s takes the next b of them
    per_rank = [[(users[r::W][s * b:(s + 1) * b], items[r::W][s * b:(s + 1) * b]) for s in range(steps)]
                for r in range(W)]
    # the one-process view: step s = the pairs rank 0 owns (from source 0, then 1), then rank 1's
    gbatches = []
    for s in range(steps):
        gu, gi = [], []
        for owner in range(W):
            for src in range(W):
                u, i = per_rank[src][s]
                sel = u % W == owner
                gu.append(u[sel])
                gi.append(i[sel])
        gbatches.append((torch.cat(gu), torch.cat(gi)))
    cap = max(x[0].numel() for x in gbatches)
    gm = _model(shape, shape.U, shape.I, state)
    gopts = _opts(gm, 1e-3, (0.9, 0.999))
    geng = ttamm.FusedTrainStep(gm, gopts, negatives_per_positive=shape.N, positives=prob.positives,
                                user_features=prob.user_features.cuda(), item_features=prob.item_features.cuda(),
                                loss_weights=LOSS_WEIGHTS, max_batch=cap, seed=SEED)
    for u, i in gbatches:
        geng.step(u.cuda(), i.cuda())
    gavg = geng.finish()
    progs, ranks = [], []
    for r in range(W):
        own = RowOwnership(W, r)
        st = {k: (own.shard(v) if k in TABLES else v.clone()) for k, v in state.items()}
        m = _model(shape, own.local_count(shape.U), own.local_count(shape.I), st)
        opts = _opts(m, 1e-3, (0.9, 0.999))
        local_pos = {u // W: prob.positives[u] for u in range(r, shape.U, W)}
        eng = ShardedTrainStep(m, opts, world_size=W, rank=r, num_items=shape.I, negatives_per_positive=shape.N,
                               positives=local_pos, user_features=own.shard(prob.user_features).cuda(),
                               item_features=own.shard(prob.item_features).cuda(), loss_weights=LOSS_WEIGHTS,
                               max_batch=2 * b, seed=SEED)
        ranks.append((own, m))
        progs.append(epoch_program(eng, [(u.cuda(), i.cuda()) for u, i in per_rank[r]]))
    ravg = run_loopback(progs)
    for r in range(W):
        assert abs(ravg[r] - gavg) <= 1e-5 * abs(gavg)
    gsd = gm.state_dict()
    for own, m in ranks:
        for k, v in m.state_dict().items():
            want = gsd[k][own.rank:: W] if k in TABLES else gsd[k]
            d = (v - want).abs().max().item()
            assert d <= 5e-5, f"rank {own.rank} {k}: {d:.2e}"


def _ranks_only(shape: Shape, W: int, *, max_batch: int, in_batch: bool = False, lr: float = 1e-3):
    prob = make_problem(shape, seed=31)
    state = prob.model.state_dict()
    ranks = []
    for r in range(W):
        own = RowOwnership(W, r)
        st = {k: (own.shard(v) if k in TABLES else v.clone()) for k, v in state.items()}
        m = _model(shape, own.local_count(shape.U), own.local_count(shape.I), st)
        opts = _opts(m, lr, (0.9, 0.999))
        local_pos = {u // W: prob.positives[u] for u in range(r, shape.U, W)}
        eng = ShardedTrainStep(m, opts, world_size=W, rank=r, num_items=shape.I, negatives_per_positive=shape.N,
                               positives=local_pos, user_features=own.shard(prob.user_features).cuda(),
                               item_features=own.shard(prob.item_features).cuda(), loss_weights=LOSS_WEIGHTS,
                               max_batch=max_batch, seed=SEED, in_batch_negatives=in_batch)
        ranks.append((own, m, opts, eng))
    return prob, ranks


@pytest.mark.parametrize("in_batch", [False, True], ids=["capacity", "in-batch-unequal"])
def test_sharded_epoch_rejects_bad_routing_on_every_rank(in_batch):
    """epoch_program: a routed batch over max_batch, or unequal routed batches with in-batch
    negatives, raise ValueError on EVERY rank before the step's first collective (one rank
    raising alone would leave the others waiting in an all-to-all under RCCL)."""
    from ttamm.sharded import epoch_program

    W, b = 2, 24
    shape = Shape(N=2 if in_batch else 5)
    prob, ranks = _ranks_only(shape, W, max_batch=b if not in_batch else 2 * b, in_batch=in_batch)
    # 3/4 of every source's pairs belong to rank 0's users: routed sizes (36, 12) per step
    gen = torch.Generator().manual_seed(3)
    per_rank = []
    for r in range(W):
        owned0 = torch.arange(0, shape.U, W)
        owned1 = torch.arange(1, shape.U, W)
        u = torch.cat([owned0[torch.randint(0, owned0.numel(), (3 * b // 4,), generator=gen)],
                       owned1[torch.randint(0, owned1.numel(), (b // 4,), generator=gen)]])
        i = torch.tensor([sorted(prob.positives[int(x)])[0] for x in u], dtype=torch.long)
        per_rank.append([(u.cuda(), i.cuda())])

    def catching(prog):
        try:
            return (yield from prog)
        except ValueError as e:
            return e

    res = run_loopback([catching(epoch_program(eng, per_rank[r])) for r, (_, _, _, eng) in enumerate(ranks)])
    for r in range(W):
        assert isinstance(res[r], ValueError), (r, res[r])
        assert ("max_batch" in str(res[r])) if not in_batch else ("same routed batch size" in str(res[r]))


def test_sharded_poisoned_step_is_skipped_by_every_rank():
    """An id outside rank 1's user shard in step 2: both ranks skip step 2 and 3 (the status
    words ride with the request counts), finish raises IndexError on both, and both ranks hold
    exactly the state after step 1 — bit for bit that of a run that stopped after step 1."""
    W, shape = 2, Shape()

    def batches(prob, steps):
        gen = torch.Generator().manual_seed(9)
        out = []
        for _ in range(steps):
            per = []
            for r in range(W):
                owned = torch.arange(r, shape.U, W)
                users = owned[torch.randint(0, owned.numel(), (shape.B,), generator=gen)]
                pos = torch.tensor([sorted(prob.positives[int(u)])[0] for u in users], dtype=torch.long)
                per.append(((users // W).cuda(), pos.cuda()))
            out.append(per)
        return out

    def catching(prog):
        try:
            return (yield from prog)
        except (IndexError, RuntimeError) as e:
            return e

    prob, ranks = _ranks_only(shape, W, max_batch=shape.B)
    steps = batches(prob, 3)
    bad = steps[1][1][0].clone()
    bad[5] = 10 ** 6  # not a row of rank 1's user shard
    steps[1][1] = (bad, steps[1][1][1])
    for per in steps:
        run_loopback([eng.program(u, p) for (_, _, _, eng), (u, p) in zip(ranks, per)])
    res = run_loopback([catching(eng.finish_program()) for (_, _, _, eng) in ranks])
    assert all(isinstance(x, IndexError) for x in res), res

    prob2, ref = _ranks_only(shape, W, max_batch=shape.B)
    run_loopback([eng.program(u, p) for (_, _, _, eng), (u, p) in zip(ref, steps[0])])
    run_loopback([eng.finish_program() for (_, _, _, eng) in ref])
    for (own, m, opts, _), (_, m2, opts2, _) in zip(ranks, ref):
        for (k, v), (_, v2) in zip(m.state_dict().items(), m2.state_dict().items()):
            assert torch.equal(v, v2), (own.rank, k)
        st, st2 = named_optimizer_state(m, opts), named_optimizer_state(m2, opts2)
        for n in st:
            assert float(st[n]["step"]) == float(st2[n]["step"]) == 1.0, (own.rank, n)
            assert torch.equal(st[n]["exp_avg"], st2[n]["exp_avg"]), (own.rank, n)


def _owned_batches(prob, shape: Shape, W: int, steps: int, seed: int = 9):
    gen = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(steps):
        per = []
        for r in range(W):
            owned = torch.arange(r, shape.U, W)
            users = owned[torch.randint(0, owned.numel(), (shape.B,), generator=gen)]
            pos = torch.tensor([sorted(prob.positives[int(u)])[0] for u in users], dtype=torch.long)
            per.append(((users // W).cuda(), pos.cuda()))
        out.append(per)
    return out


def _catching(prog, kinds=(IndexError, RuntimeError, ValueError)):
    try:
        return (yield from prog)
    except kinds as e:
        return e


@pytest.mark.parametrize("W", [2, 3])
def test_look_ahead_poison_in_next_batch_skipped_by_every_rank(W):
    """A bad user id in ONE rank's next_batch (step 2's batch, checked and routed by step 1's
    look-ahead): every rank skips step 2 and 3 (the look-ahead's status rides with the counts it
    exchanges), finish raises IndexError on every rank, and every rank holds exactly the state
    after step 1."""
    shape = Shape()
    prob, ranks = _ranks_only(shape, W, max_batch=shape.B)
    steps = _owned_batches(prob, shape, W, 3)
    bad = steps[1][W - 1][0].clone()
    bad[3] = 10 ** 6  # not a row of the last rank's user shard
    steps[1][W - 1] = (bad, steps[1][W - 1][1])
    for s, per in enumerate(steps):
        nxt = steps[s + 1] if s + 1 < len(steps) else None
        run_loopback([eng.program(u, p, next_batch=nxt[r] if nxt else None)
                      for r, ((_, _, _, eng), (u, p)) in enumerate(zip(ranks, per))])
    res = run_loopback([_catching(eng.finish_program()) for (_, _, _, eng) in ranks])
    assert all(isinstance(x, IndexError) for x in res), res

    prob2, ref = _ranks_only(shape, W, max_batch=shape.B)
    run_loopback([eng.program(u, p) for (_, _, _, eng), (u, p) in zip(ref, steps[0])])
    run_loopback([eng.finish_program() for (_, _, _, eng) in ref])
    for (own, m, opts, _), (_, m2, opts2, _) in zip(ranks, ref):
        for (k, v), (_, v2) in zip(m.state_dict().items(), m2.state_dict().items()):
            assert torch.equal(v, v2), (own.rank, k)


def test_look_ahead_batch_copy_is_used_and_other_batch_raises_on_every_rank():
    """A prepared look-ahead is consumed by every rank (its count exchange already ran on all of
    them), so the collective sequence never diverges.  (a) A rank handed a COPY of the prepared
    batch (equal values, another tensor) steps normally: the same state as identity-passing
    ranks.  (b) A rank handed ANOTHER batch skips that step (nothing written) and finish raises
    ValueError on every rank instead of one rank hanging the others."""
    W, shape = 2, Shape()
    prob, ranks = _ranks_only(shape, W, max_batch=shape.B)
    prob_b, twin = _ranks_only(shape, W, max_batch=shape.B)
    steps = _owned_batches(prob, shape, W, 2)
    # (a) rank 1 gets a copy at step 2
    for s, per in enumerate(steps):
        nxt = steps[s + 1] if s + 1 < len(steps) else None
        progs = []
        for r, ((_, _, _, eng), (u, p)) in enumerate(zip(ranks, per)):
            if s == 1 and r == 1:
                u, p = u.clone(), p.clone()
            progs.append(eng.program(u, p, next_batch=nxt[r] if nxt else None))
        run_loopback(progs)
        run_loopback([eng.program(u, p, next_batch=nxt[r] if nxt else None)
                      for r, ((_, _, _, eng), (u, p)) in enumerate(zip(twin, per))])
    la = run_loopback([eng.finish_program() for (_, _, _, eng) in ranks])
    lb = run_loopback([eng.finish_program() for (_, _, _, eng) in twin])
    assert la == lb
    for (_, m, _, _), (_, m2, _, _) in zip(ranks, twin):
        for (k, v), (_, v2) in zip(m.state_dict().items(), m2.state_dict().items()):
            assert torch.equal(v, v2), k
    # (b) rank 0 gets a different batch at step 2
    prob_c, bad = _ranks_only(shape, W, max_batch=shape.B)
    other = _owned_batches(prob, shape, W, 1, seed=123)[0]
    for s, per in enumerate(steps):
        nxt = steps[s + 1] if s + 1 < len(steps) else None
        progs = []
        for r, ((_, _, _, eng), (u, p)) in enumerate(zip(bad, per)):
            if s == 1 and r == 0:
                u, p = other[0]
            progs.append(eng.program(u, p, next_batch=nxt[r] if nxt else None))
        run_loopback(progs)
    res = run_loopback([_catching(eng.finish_program()) for (_, _, _, eng) in bad])
    assert all(isinstance(x, ValueError) and "look-ahead" in str(x) for x in res), res


def test_look_ahead_rejects_bad_next_batch_before_any_collective():
    """A malformed next_batch raises ValueError at the top of program(), before the step's first
    collective, on the rank that got it (not halfway through the step, after the forward
    exchange, with the peers blocked in the next collective)."""
    W, shape = 2, Shape()
    prob, ranks = _ranks_only(shape, W, max_batch=shape.B)
    steps = _owned_batches(prob, shape, W, 1)
    eng = ranks[0][3]
    u, p = steps[0][0]
    prog = eng.program(u, p, next_batch=(u.to(torch.int32), p))
    with pytest.raises(ValueError, match="next_batch"):
        next(prog)


def test_look_ahead_checks_next_batch_after_a_prepared_look_ahead_replaces_row_base():
    """a step that consumes a prepared look-ahead runs at default positions whatever
    row_base / global_batch the call passes, so its own look-ahead runs too — and its next_batch
    must be validated on that effective condition.  An oversized next_batch passed together with
    row_base raises ValueError before the step's first collective (never a B x N draw into the
    max_batch x N look-ahead buffers)."""
    W, shape = 2, Shape()
    prob, ranks = _ranks_only(shape, W, max_batch=shape.B)
    steps = _owned_batches(prob, shape, W, 2)
    run_loopback([eng.program(u, p, next_batch=steps[1][r])
                  for r, ((_, _, _, eng), (u, p)) in enumerate(zip(ranks, steps[0]))])
    eng = ranks[0][3]
    u, p = steps[1][0]
    big_u = torch.cat([u, u])[: shape.B + 1]
    big_p = torch.cat([p, p])[: shape.B + 1]
    prog = eng.program(u, p, row_base=0, next_batch=(big_u, big_p))
    with pytest.raises(ValueError, match="next_batch"):
        next(prog)
