#!/usr/bin/env python3
"""Throughput benchmark of the fused two-tower training step on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c4|c5|tiny]
                    [--negatives sampled|in-batch] [--neg N]

--gpus N > 1 without WORLD_SIZE in the environment starts the N ranks itself (a child
`torch.distributed.run --nproc-per-node N`, rendezvous on 127.0.0.1) and prints rank 0's line;
under an external launcher (WORLD_SIZE set) it runs as one of the ranks.

Workload (BASELINE.json configs[1], "C2"): 2M items x 200K users, 96-dim towers, feature
MLP 605 -> 192 -> 96 (ReLU, dropout 0.15), gated fusion, adaptive mimic on, batch 8192,
5 sampled negatives per positive (the reference's semantics), AdamW
(lr 1e-3, wd 0.01) over the dense group incl. the full mimic tables + SparseAdam over the
ID tables.  Synthetic data of that shape, random-init weights; inputs resident in HBM.
--negatives in-batch switches to ttamm's in-batch mode (BASELINE C2/C4 "in-batch negatives":
every user scored against every positive of the global batch, plus --neg sampled negatives,
default 0).  --config c4 is BASELINE configs[3] per GPU: a 1/8 shard of 50M items x 200K
users (6.25M x 25K), D = 128, MLP 605 -> 256 -> 128, in-batch negatives (all-gathered across
ranks); at --gpus 8 the global model is the full C4.

One step = the loader's next batch (ttamm.DeviceInteractionLoader: the epoch order evaluated on
the device, pairs resident in HBM) + one call of ttamm_train_step on it (sampling, forward,
loss, backward, both optimizers).  `value` = interactions (positives) per second over all ranks.  The timed
region is K steps plus the closing flush of the deferred table AdamW (every row brought
current, as `finish()` does at the end of an epoch); K defaults to one epoch of the config
(C2: ceil(200K users x 20 positives / 8192) = 489 steps), so the flush is priced as the
reference's per-epoch work, not per 20 steps.
Multi-GPU (weak scaling): one process per GPU (torch.distributed.run, RCCL).  Rank r owns
users and items with id % N == r — C2-sized shards, so the global model is N x C2 — and runs
the row-sharded step of ttamm/sharded.py on a C2 batch of its own users: item requests and
(t | a) / (dT | dA) rows go through all-to-alls, the MLP / gate gradients through one
all-reduce.

The JSON line also carries
  kernels:      the step's largest kernels, each timed live with HIP events on the stream it
                runs on, over the timed steps: the deferred table AdamW replay (rolling slice +
                both towers' catch-up, + the closing flush's share; VALU-bound), the first
                feature-layer forward GEMM, the wide weight-gradient GEMM launch, the in-batch
                scoring kernel (MFMA-bound; algorithmic FLOPs 2 R F H, 2 R M N, 6 B Bg D);
  roofline:     the one of them with the most time per step;
  cpu_baseline: the CPU oracle (oracle/cpu_reference.py, the reference's step restated on
                PyTorch-CPU incl. its per-row sampler loop) timed on this host, rank 0, N=1.
--emulate-world W (one GPU, developer): rank 0 of a W-rank row-sharded job whose other ranks
mirror it (ttamm.sharded.MirrorComm: the per-rank work of the W-rank step — W x the item
requests as owner, the W B all-gathered in-batch positives — without interconnect traffic);
`value` is then this rank's own throughput.
"""

from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "two-tower-augmented-with-adaptive-mimic-mechanism_amd"))
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

METRIC = "training interactions/sec at 1/2/4/8 MI355X; Recall@20 parity vs CPU ref"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
MFMA_FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: fp32 matrix (v_mfma_f32_32x32x2_f32), dense
MFMA_BF16_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: bf16 MFMA ~2.5 PF dense (no sparsity)
# VALU issue: 256 CUs x 4 SIMD-32, one wave64 instruction per 2 cycles at 2.4 GHz
# (MI355X_MICROARCH.md "Wave scheduling" and the v_fma_f32 row of the cycle constants)
VALU_WAVE_INSTR_PEAK = 1024 * 2.4e9 / 2

CONFIGS = {
    "c2": dict(U=200_000, I=2_000_000, D=96, H=192, F=605, B=8192, N=5, dropout=0.15, pos_per_user=20),
    # BASELINE configs[4] per GPU: bf16 towers, 256-dim embeddings, 512-wide MLP, gate on
    # (weak scaling: each of N ranks holds a shard of this size; at --gpus 8 the 8-GPU C5)
    "c5": dict(U=200_000, I=2_000_000, D=256, H=512, F=605, B=8192, N=5, dropout=0.15, pos_per_user=20,
               matmul="bf16"),
    # BASELINE configs[3] per GPU (weak scaling): 1/8 of 50M items x 200K users, D = 128, H = 256;
    # in-batch negatives, all-gathered across ranks ("all-gather negatives")
    # (replay_slices: the deferred AdamW's rolling slice; the C4 shard's mostly cold 6.25 M-row
    # tables replay cheaper in longer, rarer passes — 8.04 M vs 7.77 M interactions/s at 64)
    "c4": dict(U=25_000, I=6_250_000, D=128, H=256, F=605, B=8192, N=0, dropout=0.15, pos_per_user=20,
               negatives="in-batch", replay_slices=128),
    # small sanity config (not a bench line)
    "tiny": dict(U=2_000, I=20_000, D=96, H=192, F=605, B=1024, N=5, dropout=0.15, pos_per_user=20),
}


class HipTimingEvent:
    """A timing hipEvent_t created with hipEventDisableSystemFence (device-scope release), the
    interface bench.py uses of torch.cuda.Event (record / elapsed_time / cuda_event).  torch's
    timing events take the default system-scope fence (an L2 writeback + invalidate): each record
    between two kernels of a stream added ≈2 µs to the ≈5 µs of stream idle an event operation costs
    there, so the per-kernel pairs inside the timed steps cost the step more than their own gaps
    (C2 0.668 -> 0.659 ms/step, profiles/r06_s23_*).  The HIP entry
    points come through libttamm.so's dependency on the process's one HIP runtime (torch's)."""

    _hip = None

    def __init__(self) -> None:
        import ctypes

        if HipTimingEvent._hip is None:
            from ttamm import _lib

            HipTimingEvent._hip = _lib.load()
        self._c = ctypes
        h = ctypes.c_void_p()
        rc = self._hip.hipEventCreateWithFlags(ctypes.byref(h), ctypes.c_uint(0x20000000))
        if rc != 0:  # a runtime without the flag: a default timing event
            rc = self._hip.hipEventCreateWithFlags(ctypes.byref(h), ctypes.c_uint(0))
        if rc != 0:
            raise RuntimeError(f"hipEventCreateWithFlags failed ({rc})")
        self.cuda_event = h.value
        self._recorded = False

    def record(self, stream=None) -> None:
        s = (stream or torch.cuda.current_stream()).cuda_stream
        rc = self._hip.hipEventRecord(self._c.c_void_p(self.cuda_event), self._c.c_void_p(s))
        if rc != 0:
            raise RuntimeError(f"hipEventRecord failed ({rc})")

    def elapsed_time(self, end: "HipTimingEvent") -> float:
        ms = self._c.c_float()
        rc = self._hip.hipEventElapsedTime(self._c.byref(ms), self._c.c_void_p(self.cuda_event),
                                           self._c.c_void_p(end.cuda_event))
        if rc != 0:  # not recorded (e.g. a pair the step did not use)
            self._hip.hipGetLastError()  # not left as the thread's error for torch's next check
            raise RuntimeError(f"hipEventElapsedTime failed ({rc})")
        return float(ms.value)

    def __del__(self) -> None:
        # not at interpreter shutdown: the HIP runtime may already be torn down (the process's exit
        # releases the events anyway)
        if sys.is_finalizing() or self._hip is None or not getattr(self, "cuda_event", None):
            return
        try:
            self._hip.hipEventDestroy(self._c.c_void_p(self.cuda_event))
        except Exception:
            pass


def tower_cfg(c: dict) -> dict:
    return {
        "type": "tower",
        "id_embedding": {"params": {"embedding_dim": c["D"], "sparse": True}, "init": {"type": "normal", "std": 0.02}},
        "feature_encoder": {"type": "mlp", "hidden_dims": [c["H"]], "activation": "relu", "output_dim": c["D"],
                            "dropout": c["dropout"]},
        "fusion": "gated",
        "output_dim": c["D"],
        "matmul_dtype": c.get("matmul", "fp32"),
    }


# ---------------------------------------------------------------------------------------
# synthetic data (SURVEY.md §8 d), generated on the device
# ---------------------------------------------------------------------------------------
def make_item_features(I: int, F: int, device, gen: torch.Generator) -> torch.Tensor:
    """[I, F] inside a [I, round_up(F, 4)] zero-padded buffer: 3 category weights {1, .5, .333}
    in cols 0-299, one author one-hot in cols 300-599, 5 N(0,1) numeric/text z-scores."""
    Fp = (F + 3) // 4 * 4
    x = torch.zeros((I, Fp), dtype=torch.float32, device=device)
    ncat = min(300, F - 5)
    nauth = min(300, F - 5 - ncat)
    rows = torch.arange(I, device=device)
    for w in (1.0, 0.5, 1.0 / 3.0):
        cols = torch.randint(0, ncat, (I,), device=device, generator=gen)
        x[rows, cols] = torch.maximum(x[rows, cols], torch.tensor(w, device=device))
    if nauth > 0:
        x[rows, ncat + torch.randint(0, nauth, (I,), device=device, generator=gen)] = 1.0
    x[:, ncat + nauth:F] = torch.randn((I, F - ncat - nauth), device=device, generator=gen)
    return x[:, :F]


def zipf_items(n: int, I: int, s: float, device, gen: torch.Generator, perm: torch.Tensor) -> torch.Tensor:
    ranks = torch.arange(1, I + 1, device=device, dtype=torch.float64)
    cdf = torch.cumsum(ranks.pow(-s), 0)
    cdf /= cdf[-1].clone()
    u = torch.rand(n, device=device, dtype=torch.float64, generator=gen)
    r = torch.searchsorted(cdf, u).clamp_(max=I - 1)
    return perm[r]


class Workload:
    """C2 data + model on one GPU, or rank `rank`'s C2-sized shard of an N x C2 model."""

    def __init__(self, c: dict, device, seed: int, world: int = 1, rank: int = 0, step_seed: int | None = None,
                 deferred: bool = True, overlap: bool = True, in_batch: bool = False, table_math: str = "fast",
                 replay_slices: int = 64, aux_cus: int = 0, sharded_single: bool = False,
                 group_towers: bool = True, emulate: bool = False):
        import ttamm
        from ttamm.samplers import PositivesCSR

        self.c = c
        self.world = world
        gen = torch.Generator(device=device).manual_seed(seed)
        torch.manual_seed(seed)
        U, I, F = c["U"], c["I"], c["F"]  # this rank's rows
        Ig = I * world  # global item count
        self.item_features = make_item_features(I, F, device, gen)
        # popularity ranks over the global catalogue: same permutation on every rank
        perm = torch.randperm(Ig, device=device, generator=torch.Generator(device=device).manual_seed(7))
        per = c["pos_per_user"]
        items = zipf_items(U * per, Ig, 1.05, device, gen, perm).view(U, per)
        items, _ = torch.sort(items, dim=1)
        offsets = torch.arange(0, U * per + 1, per, device=device, dtype=torch.long)
        self.csr = PositivesCSR(offsets, items.reshape(-1).contiguous(), U, per)
        # user features: mean of the user's positives (features.py:269-315)
        Fp = self.item_features.stride(0)
        uf = torch.zeros((U, Fp), dtype=torch.float32, device=device)
        full = self.item_features.as_strided((I, Fp), (Fp, 1))
        for lo in range(0, U, 16384):
            hi = min(U, lo + 16384)
            # sharded: the positives' feature rows live on their owners; a local row of the
            # same shape stands in (the values do not change the work)
            rows = torch.div(items[lo:hi].reshape(-1), world, rounding_mode="floor")
            uf[lo:hi] = full[rows].view(hi - lo, per, Fp).mean(dim=1)
        self.user_features = uf[:, :F]
        # interactions: every (user, positive) pair, HBM-resident; batches come from the on-device
        # loader (ttamm.DeviceInteractionLoader = DataLoader(shuffle=True), a new order per epoch;
        # drop_last keeps every step at B)
        self.users_all = torch.arange(U, device=device).repeat_interleave(per)
        self.items_all = items.reshape(-1).contiguous()
        self.loader = ttamm.DeviceInteractionLoader(self.users_all, self.items_all, c["B"], shuffle=True,
                                                    drop_last=True, seed=seed)
        self._it = iter(self.loader)
        # model + optimizers (training.py:1266-1350)
        cfg = tower_cfg(c)
        ue = ttamm.build_tower_encoder(cfg, num_embeddings=U, feature_dim=F, device=device)
        ie = ttamm.build_tower_encoder(cfg, num_embeddings=I, feature_dim=F, device=device)
        mm = ttamm.AdaptiveMimicMechanism(num_users=U, num_items=I, embedding_dim=c["D"]).to(device)
        self.model = ttamm.TwoTowerModel(ue, ie, similarity=ttamm.DotProductSimilarity(), adaptive_mimic=mm)
        dense, sparse = ttamm._collect_parameter_groups(self.model)
        self.opts = [torch.optim.AdamW(dense, lr=1e-3, weight_decay=0.01), torch.optim.SparseAdam(sparse, lr=1e-3)]
        kw = dict(negatives_per_positive=c["N"], positives=self.csr, user_features=self.user_features,
                  item_features=self.item_features, loss_weights={"mimic_user": 0.15, "mimic_item": 0.15},
                  max_batch=c["B"], deferred_adamw=deferred, overlap=overlap, in_batch_negatives=in_batch,
                  table_adamw_math=table_math, replay_slices=replay_slices, aux_cus=aux_cus or None)
        if world == 1 and not sharded_single:
            self.engine = ttamm.FusedTrainStep(self.model, self.opts, seed=seed, **kw)
        elif world == 1:  # developer: the row-sharded phases at W = 1 (their overhead, no exchange cost)
            from ttamm.sharded import ShardedTrainStep, run_loopback

            class _One:
                @staticmethod
                def run(program):
                    return run_loopback([program])[0]

            self.engine = ShardedTrainStep(self.model, self.opts, world_size=1, rank=0, num_items=Ig, comm=_One(),
                                           seed=seed, group_towers=group_towers, **kw)
        else:
            from ttamm.sharded import MirrorComm, ShardedTrainStep, TorchComm

            # step_seed: the same on every rank (the Philox streams are keyed by global position)
            comm = MirrorComm(world, rank) if emulate else TorchComm()
            self.engine = ShardedTrainStep(self.model, self.opts, world_size=world, rank=rank, num_items=Ig,
                                           comm=comm, seed=step_seed, group_towers=group_towers, **kw)

    def batch(self):
        """The next batch of the on-device loader (epochs run back to back)."""
        try:
            return next(self._it)
        except StopIteration:
            self._it = iter(self.loader)
            return next(self._it)


# ---------------------------------------------------------------------------------------
# CPU baseline: the oracle's restatement of the reference step on this host
# ---------------------------------------------------------------------------------------
def cpu_baseline(c: dict, steps: int, warmup: int, seed: int, in_batch: bool = False) -> dict:
    from oracle import cpu_reference as ref

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, len(os.sched_getaffinity(0)))
    torch.set_num_threads(threads)
    gen = torch.Generator().manual_seed(seed)
    torch.manual_seed(seed)
    U, I, F, B, N = c["U"], c["I"], c["F"], c["B"], c["N"]
    item_features = make_item_features(I, F, "cpu", gen).contiguous()
    per = c["pos_per_user"]
    perm = torch.randperm(I, generator=gen)
    items = zipf_items(U * per, I, 1.05, "cpu", gen, perm).view(U, per)
    user_features = item_features[items[:, 0]]  # cheap stand-in of the same shape (values do not change the work)
    tcfg = tower_cfg(c)
    tcfg = {**tcfg, "adaptive_mimic": {}}
    model = ref.build_model(tcfg, num_users=U, num_items=I, user_feature_dim=F, item_feature_dim=F, mimic=True)
    opts = ref.build_optimizers(model, lr=1e-3, weight_decay=0.01)
    # positives as the reference holds them: dict[user] -> set(items) (preprocessing.py:151-154)
    need_users = torch.randint(0, U, ((steps + warmup) * B,), generator=gen)
    positives = {int(u): set(items[int(u)].tolist()) for u in need_users.unique().tolist()}
    batches = []
    for k in range(steps + warmup):
        us = need_users[k * B:(k + 1) * B]
        ps = items[us, torch.randint(0, per, (B,), generator=gen)]
        batches.append((us, ps))
    lw = {"mimic_user": 0.15, "mimic_item": 0.15}
    ref.train_one_epoch(model, batches[:warmup], opts, negatives_per_positive=N, num_items=I, positives=positives,
                        user_features=user_features, item_features=item_features, loss_weights=lw, in_batch=in_batch)
    _, seen, secs = ref.train_one_epoch(model, batches[warmup:], opts, negatives_per_positive=N, num_items=I,
                                        positives=positives, user_features=user_features,
                                        item_features=item_features, loss_weights=lw, in_batch=in_batch)
    return {
        "value": round(seen / secs, 1),
        "unit": "interactions/s",
        "cores": threads,
        "cpu_model": cpu_model(),
        "kind": "port",
        "sample": f"{steps} timed steps (+{warmup} warm-up) of the same-shaped step, batch {B}, on "
                  f"{threads} host threads: oracle/cpu_reference.py (reference per-row sampler, AdamW over the "
                  f"full {U}x{c['D']} + {I}x{c['D']} mimic tables, SparseAdam"
                  f"{', in-batch B x B logits' if in_batch else ''}); {secs:.1f} s timed",
    }


def gather_bulk(device, rows: int = 50_000_000, dim: int = 128, n: int = 2_000_000, reps: int = 10) -> dict:
    """north_star's "50M x 128 embedding gather" in bulk, after the timed
    region: a 50M x 128 fp32 table (25.6 GB, N(0, 0.02)), 2M uniform row ids (every row a cold HBM
    read).  `materialising`: the step's product gather (ttamm_gather_rows) copying the rows out —
    it writes every byte it reads, so its read rate is at most half of HBM and `total_frac` prices
    both directions; `read_only`: the product's consumer that reads the same rows by id and keeps
    4 B per row (ttamm_candidate_topk, the sampled-candidate evaluation, 100 candidates per
    query).  Every materialising launch is checked bit-exact against torch.index_select."""
    from ttamm import _lib as L

    lib = L.load()
    gen = torch.Generator(device=device).manual_seed(4321)
    table = torch.empty((rows, dim), dtype=torch.float32, device=device)
    for lo in range(0, rows, 1 << 22):
        table[lo:lo + (1 << 22)].normal_(0.0, 0.02, generator=gen)
    idx = torch.randint(0, rows, (n,), generator=gen, device=device)
    out = torch.empty((n, dim), dtype=torch.float32, device=device)
    sp = torch.cuda.current_stream().cuda_stream

    def launch():
        L.check(lib.ttamm_gather_rows(table.data_ptr(), rows, dim, idx.data_ptr(), n, out.data_ptr(), dim, sp))

    launch()
    torch.cuda.synchronize()
    exact = bool(torch.equal(out, torch.index_select(table, 0, idx)))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        launch()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    rd, tot = n * dim * 4, n * (2 * dim * 4 + 8)
    mat = {"kernel": "gather_rows_wide (ttamm_gather_rows)", "rows_per_launch": n, "avg_launch_ms": round(ms, 4),
           "read_GBps": round(rd / ms / 1e6, 1), "read_frac": round(rd / ms / 1e6 / HBM_PEAK_GBS, 4),
           "total_GBps": round(tot / ms / 1e6, 1), "total_frac": round(tot / ms / 1e6 / HBM_PEAK_GBS, 4),
           "bit_exact_vs_torch": exact}
    del out
    per_q, k = 100, 20
    nq = n // per_q
    q = torch.randn((nq, dim), generator=gen, device=device, dtype=torch.float32)
    off = torch.arange(0, nq * per_q + 1, per_q, device=device, dtype=torch.long)
    out_s = torch.empty((nq, k), dtype=torch.float32, device=device)
    out_p = torch.empty((nq, k), dtype=torch.long, device=device)

    def launch_c():
        L.check(lib.ttamm_candidate_topk(q.data_ptr(), nq, dim, table.data_ptr(), rows, dim, dim, off.data_ptr(),
                                         idx.data_ptr(), per_q, 0, k, out_s.data_ptr(), out_p.data_ptr(), sp))

    launch_c()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        launch_c()
    e1.record()
    torch.cuda.synchronize()
    ms_c = e0.elapsed_time(e1) / reps
    ro = {"kernel": "candidate_topk_v_kernel (ttamm_candidate_topk)", "rows_per_launch": n,
          "avg_launch_ms": round(ms_c, 4), "read_GBps": round(rd / ms_c / 1e6, 1),
          "read_frac": round(rd / ms_c / 1e6 / HBM_PEAK_GBS, 4)}
    del table
    torch.cuda.empty_cache()
    pmc = load_traffic("c4_gather_bulk") or {}
    mat["traffic"] = pmc.get("materialising_bytes_per_launch")
    ro["traffic"] = pmc.get("read_only_bytes_per_launch")
    return {"table": f"{rows} x {dim} fp32", "indices": "uniform", "materialising": mat, "read_only": ro,
            "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "note": "traffic: HBM bytes per launch from rocprofv3 FETCH_SIZE (x2, gfx950) / WRITE_SIZE passes "
                    "(profiles/pmc_traffic.json c4_gather_bulk, profiles/r06_gather_bulk_*)"}


def cpu_model() -> str:
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def load_traffic(config: str) -> dict | None:
    """HBM bytes per launch of the roofline kernels, from the committed rocprofv3 PMC passes
    (profiles/pmc_traffic.json)."""
    path = ROOT / "profiles" / "pmc_traffic.json"
    try:
        return json.loads(path.read_text()).get(config)
    except (OSError, ValueError):
        return None


def wgrad_problems(c: dict, rows: dict) -> list[tuple[int, int, int]]:
    """(R, M, N) of the step's weight gradients (tower_backward): per tower the feature MLP's
    layers, then the gate's two Linear (Hg = D)."""
    F, H, D = c["F"], c["H"], c["D"]
    out = []
    for R in rows.values():
        out += [(R, H, F), (R, D, H), (R, D, 2 * D), (R, D, D)]
    return out


def launch_command(argv: list[str], gpus: int, port: int) -> list[str]:
    """The torch.distributed.run command that starts `gpus` ranks of this script (one process
    per GPU, rendezvous on 127.0.0.1), forwarding the caller's arguments unchanged."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", str(Path(__file__).resolve()), *argv]


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(argv: list[str], gpus: int) -> int:
    """`bench.py --gpus N` without a launcher: start the N ranks as a child torch.distributed.run
    (this process never touches the GPU), relay rank 0's JSON line and check it covers N GPUs."""
    import subprocess

    proc = subprocess.run(launch_command(argv, gpus, free_port()), stdout=subprocess.PIPE, text=True)
    line = None
    for ln in proc.stdout.splitlines():
        if ln.startswith("{") and '"metric"' in ln:
            line = ln
        else:
            print(ln, flush=True)
    if proc.returncode != 0 or line is None:
        print(f"bench.py: the {gpus}-rank run failed (exit {proc.returncode})", file=sys.stderr)
        return proc.returncode or 1
    out = json.loads(line)
    if out.get("n_gpus") != gpus:
        print(f"bench.py: the {gpus}-rank run reported n_gpus={out.get('n_gpus')}", file=sys.stderr)
        return 1
    print(line, flush=True)
    return 0


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default: one epoch of the config, ceil(U x positives per user / B))")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--cpu-steps", type=int, default=20)
    ap.add_argument("--cpu-warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo stages the exchanges through host memory (several ranks on one GPU, tests only)")
    ap.add_argument("--eager-adamw", action="store_true",
                    help="sweep AdamW(g=0) over the whole mimic tables every step instead of the deferred exact replay")
    ap.add_argument("--overlap-exchange", action="store_true",
                    help="row-sharded step: overlap the (t | a) all-to-all with a separate user-tower forward "
                         "instead of grouping the two towers' launches (ShardedTrainStep(group_towers=False))")
    ap.add_argument("--no-look-ahead", action="store_true",
                    help="row-sharded step: route each batch in its own step (a host synchronisation on the "
                         "request counts every step) instead of one step ahead")
    ap.add_argument("--sharded-single", action="store_true",
                    help="developer: run the row-sharded step's phases at one GPU (W = 1, in-process exchange)")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="developer: rank 0 of a W-rank sharded job on one GPU, the other ranks mirrored "
                         "(ttamm.sharded.MirrorComm: per-rank work without interconnect traffic)")
    ap.add_argument("--aux-cus", type=int, default=0,
                    help="run the step's aux-stream prologue on this many CUs only (0 = all)")
    ap.add_argument("--replay-slices", type=int, default=None,
                    help="deferred table AdamW: every row is replayed at least once per this many steps "
                         "(default: the config's, 64 unless it says otherwise)")
    ap.add_argument("--exact-table-math", action="store_true",
                    help="IEEE sqrt / division for the g = 0 table AdamW updates (bit-identical to torch) "
                         "instead of v_sqrt / v_rcp")
    ap.add_argument("--no-exact-line", dest="exact_line", action="store_false",
                    help="skip the exact_table_math sub-line (K more steps with the drop-in default's "
                         "bit-exact g = 0 table arithmetic)")
    ap.add_argument("--no-gather-bulk", dest="gather_bulk", action="store_false",
                    help="--config c4: skip the 50M x 128 bulk gather sub-line (after the timed region)")
    ap.add_argument("--kernel-events", choices=["every-step", "roofline", "none"], default="every-step",
                    help="every-step: every pair in the timed steps.  roofline: the timed steps carry the "
                         "aux-stream replay pairs, the in-batch and c4 gather pairs only; the main-stream GEMM "
                         "pairs (first layer, wide weight gradient) are timed in a detail pass of K more steps "
                         "after it (C2 +0.6 %%, within noise: profiles/r06_s29_*).  none: no pairs (the "
                         "roofline entries then have no live launch durations; the events' own cost)")
    ap.add_argument("--event-kind", choices=["device", "torch"], default="device",
                    help="device: timing events with a device-scope release (HipTimingEvent); torch: "
                         "torch.cuda.Event (system-scope fence, ≈2 µs more stream idle per record)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="run the step's index-only prologue on the main stream (no aux stream)")
    ap.add_argument("--negatives", choices=["sampled", "in-batch"], default=None,
                    help="sampled (the reference's, default for c2/c5) or ttamm's in-batch mode (default for c4)")
    ap.add_argument("--neg", type=int, default=None,
                    help="sampled negatives per positive (default: 5 sampled, 0 on top of in-batch)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no external launcher: this process only spawns the ranks (no GPU call before this point)
        sys.exit(self_launch(sys.argv[1:], args.gpus))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist_mod

        dist = dist_mod
        if args.dist_backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    emulate = args.emulate_world > 1 and world == 1
    shard_world = args.emulate_world if emulate else world  # the W of the sharded step's shapes
    # more ranks than GPUs only with --dist-backend gloo (RCCL needs one GPU per rank)
    device = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(device)
    c = dict(CONFIGS[args.config])
    in_batch = (args.negatives or c.get("negatives", "sampled")) == "in-batch"
    if args.neg is not None:
        c["N"] = args.neg
    elif in_batch and args.negatives == "in-batch" and "negatives" not in c:
        c["N"] = 0

    if args.replay_slices is None:
        args.replay_slices = int(c.get("replay_slices", 64))
    if args.steps is None:  # one epoch: the deferred-AdamW flush closes it, as at the reference's epoch end
        args.steps = max(1, math.ceil(c["U"] * c["pos_per_user"] / c["B"]))
    w = Workload(c, device, args.seed + rank, world=shard_world, rank=rank, step_seed=args.seed,
                 deferred=not args.eager_adamw, overlap=not args.no_overlap, in_batch=in_batch,
                 table_math="exact" if args.exact_table_math else "fast", replay_slices=args.replay_slices,
                 aux_cus=args.aux_cus, sharded_single=args.sharded_single,
                 group_towers=not args.overlap_exchange, emulate=emulate)
    eng = w.engine
    # row-sharded step: each step routes the next batch ahead (look-ahead routing, its request
    # counts reach the host during this step's backward); one process: the batch only
    from ttamm.sharded import ShardedTrainStep

    look_ahead = isinstance(eng, ShardedTrainStep) and not args.no_look_ahead
    nxt = w.batch()

    def step(**kw) -> None:
        nonlocal nxt
        u, p = nxt
        nxt = w.batch()
        if look_ahead:
            eng.step(u, p, next_batch=nxt, **kw)
        else:
            eng.step(u, p, **kw)

    for _ in range(args.warmup):
        step()
    eng.flush()  # the timed region starts with every table row current
    torch.cuda.synchronize()

    # per-step HIP event pairs (ttamm.h ttamm_step_args.timing_events), each recorded on the
    # stream its kernel runs on: [0,1] the deferred slice's replay kernel, [2,3] the grouped first
    # feature-layer forward GEMM, [4,5] the in-batch kernel, [6,7] the wide weight-gradient GEMM
    # launch, [8,9] / [10,11] the user / item catch-up replay kernels, [12,13] the ID-row gather
    NEV = 14
    if args.event_kind == "device":
        new_event = HipTimingEvent
    else:  # torch's (system-scope) timing events, for the A/B of their cost
        def new_event():
            e = torch.cuda.Event(enable_timing=True)
            e.record()  # materialise the hipEvent_t handle
            return e
    evs = [[new_event() for _ in range(NEV)] for _ in range(args.steps)]
    torch.cuda.synchronize()
    rows0 = getattr(eng, "item_rows_seen", 0)

    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    marks = [new_event() for _ in range(3)]
    t0 = time.perf_counter()
    marks[0].record()
    for k in range(args.steps):
        # the loader's gather of the next batch (ttamm_epoch_batch) runs inside the timed region
        if args.kernel_events == "none":
            step()
        else:
            # the ID-row gather's pair [12, 13] only for --config c4 (SURVEY §8 g2's 50M x 128 gather):
            # an event pair on the aux stream between its gather and catch-up launches is measured
            # overhead in the C2 step under rocprofv3
            n_ev = NEV if args.config == "c4" else 12
            handles = [e.cuda_event for e in evs[k][:n_ev]]
            if args.kernel_events == "roofline":
                # the main-stream GEMM pairs [2, 3] / [6, 7] are timed in the detail pass below: each
                # event record on the main stream holds it idle a few µs (profiles/r06_s22_*)
                for i in (2, 3, 6, 7):
                    handles[i] = None
            step(timing_events=handles)
    marks[1].record()
    # deferred AdamW: the g = 0 updates still owed to untouched rows are part of the K steps' work
    eng.flush()
    marks[2].record()
    torch.cuda.synchronize()
    rows1 = getattr(eng, "item_rows_seen", 0)  # the timed steps' owner rows (before the exact sub-line)
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], device=device if args.dist_backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    exact_line = None
    if args.exact_line and not args.eager_adamw and not args.exact_table_math and hasattr(eng, "args"):
        # the drop-in default's table arithmetic (ttamm.FusedTrainStep(table_adamw_math="exact"),
        # IEEE sqrt / division, bit-identical to torch's AdamW): the same step, K more steps + the
        # flush, timed the same way.  Every row is current here (the flush above), so the switch
        # applies from the next step on.
        from ttamm import _lib as ttamm_lib

        eng.args.table_g0_math = ttamm_lib.G0_EXACT
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            step()
        eng.flush()
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        ex_elapsed = time.perf_counter() - t1
        if dist is not None:
            t = torch.tensor([ex_elapsed], device=device if args.dist_backend == "nccl" else "cpu", dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            ex_elapsed = float(t.item())
        eng.args.table_g0_math = ttamm_lib.G0_FAST
        exact_line = {"value": round(args.steps * c["B"] * world / ex_elapsed, 1), "unit": "interactions/s",
                      "ms_per_step": round(ex_elapsed / args.steps * 1e3, 4), "steps": args.steps,
                      "note": "table_adamw_math='exact' (the ttamm.FusedTrainStep / train_one_epoch default: IEEE "
                              "sqrt and division in the g = 0 table AdamW, bit-identical to torch): the same "
                              "workload, K steps + the closing flush, right after the main timed region"}
    evs_detail = evs
    if args.kernel_events == "roofline":
        # detail pass: K more steps (+ the flush) carrying the main-stream GEMM pairs [2, 3] (first
        # feature layer) and [6, 7] (wide weight gradient), for the kernels entries beside the roofline
        evs_detail = [[new_event() for _ in range(NEV)] for _ in range(args.steps)]
        torch.cuda.synchronize()
        for k in range(args.steps):
            handles = [None] * 12
            for i in (2, 3, 6, 7):
                handles[i] = evs_detail[k][i].cuda_event
            step(timing_events=handles)
        eng.flush()
        torch.cuda.synchronize()
    loss = eng.finish()
    steps_only_ms = marks[0].elapsed_time(marks[1]) / args.steps
    flush_ms = marks[1].elapsed_time(marks[2])

    def pair_ms(i: int) -> float:  # mean over the timed steps of event pair (i, i + 1); 0 if unused
        tot = 0.0
        for q in (evs_detail if i in (2, 6) else evs):
            try:
                tot += q[i].elapsed_time(q[i + 1])
            except RuntimeError:  # not recorded this step
                return 0.0
        return tot / args.steps

    B, U, I, D, F, H, N = c["B"], c["U"], c["I"], c["D"], c["F"], c["H"], c["N"]
    sharded = shard_world > 1 or args.sharded_single
    interactions = args.steps * B * world
    value = interactions / elapsed
    bf16 = c.get("matmul", "fp32") == "bf16"
    exact_mfma = os.environ.get("TTAMM_FP32_MFMA") == "exact"
    mfma_peak = MFMA_BF16_PEAK_TFLOPS if bf16 else MFMA_FP32_PEAK_TFLOPS
    split_ceiling = None if (bf16 or exact_mfma) else MFMA_BF16_PEAK_TFLOPS / 6.0  # six bf16 MFMAs per product
    # PMC entry: the config's own, or "<config>_inbatch" when in-batch negatives replace its sampled ones;
    # the sharded shapes of a W-rank step carry their own passes ("<key>_w<W>"): a 1-GPU pass never
    # stands in for a launch of another shape (no entry -> traffic null)
    tkey = args.config + ("_inbatch" if in_batch and CONFIGS[args.config].get("negatives", "sampled") != "in-batch" else "")
    if shard_world > 1 or args.sharded_single:
        tkey += f"_w{shard_world}"
    traffic = load_traffic(tkey) or {}
    # tower rows of one step: users B; items B (1 + N) (one process) or the owner's requested rows
    if not sharded:
        item_rows = B * (1 + N)
    else:
        item_rows = (rows1 - rows0) / args.steps
    rows = {"user": B, "item": item_rows}
    if bf16:
        impl = "bf16 operands, v_mfma_f32_32x32x16_bf16"
    elif exact_mfma:
        impl = "fp32 v_mfma_f32_32x32x2_f32"
    else:
        impl = "fp32 as split-bf16 (hi/mid/lo planes, 6 x v_mfma_f32_32x32x16_bf16 per product)"

    def mfma_entry(name: str, flops: float, ms: float, ceiling: float | None, traffic_key: str,
                   alg_bytes: float | None = None) -> dict:
        """peak = the roof of the MFMA the kernel runs on: the split-bf16 kernels' own ceiling (the
        bf16 dense peak / 6 bf16 MFMAs per fp32 product; work a kernel repeats, such as the in-batch
        kernel's second formation of S, counts against it, not as a lower roof), the bf16 peak for
        bf16 towers, the fp32 MFMA peak for TTAMM_FP32_MFMA=exact; the
        fp32 MFMA peak (what an fp32 GEMM could reach on the fp32 instruction) is kept beside it."""
        tf = flops / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
        peak = ceiling or mfma_peak
        e = {"bound": "mfma", "kernel": name, "achieved": round(tf, 2), "peak": round(peak, 1), "unit": "TFLOP/s",
             "frac": round(tf / peak, 4), "traffic": traffic.get(traffic_key),
             "algorithmic_flops_per_launch": flops, "avg_launch_ms": round(ms, 4), "ms_per_step": round(ms, 4)}
        if alg_bytes is not None:
            e["algorithmic_bytes_per_launch"] = alg_bytes
        if ceiling:
            e["peak_note"] = ("split-bf16 ceiling: v_mfma_f32_32x32x16_bf16 dense peak "
                              f"{MFMA_BF16_PEAK_TFLOPS:.0f} TF/s / bf16 MFMAs per fp32 product")
            e["fp32_mfma_peak_tflops"] = MFMA_FP32_PEAK_TFLOPS
            e["frac_of_fp32_mfma_peak"] = round(tf / MFMA_FP32_PEAK_TFLOPS, 4)
        return e

    kernels = []
    # first feature layer, grouped launch: rows x F x H multiply-adds (algorithmic F, not the
    # MFMA's zero-padded K); sharded + grouped towers: the owner's item rows + its B user rows
    l1_rows = rows["item"] + (B if (not sharded or eng.group_towers) else 0)
    kernels.append(mfma_entry(
        f"first feature layer forward GEMM (Linear {F}->{H} + ReLU + dropout, user and item rows grouped), {impl}",
        2.0 * l1_rows * F * H, pair_ms(2), split_ceiling, "l1_forward_gemm_bytes_per_launch",
        alg_bytes=l1_rows * (F * 4 + H * 4)))
    wide = [(R, M, Nn) for R, M, Nn in wgrad_problems(c, rows) if M > 96]
    if wide:
        kernels.append(mfma_entry(
            "wide weight-gradient GEMM launch (dW = dY^T X, split-K slabs; "
            + ", ".join(f"{M}x{Nn}" for _, M, Nn in wide[: len(wide) // 2]) + f" per tower), {impl}",
            sum(2.0 * R * M * Nn for R, M, Nn in wide), pair_ms(6), split_ceiling, "wgrad_wide_bytes_per_launch"))
    if args.kernel_events == "roofline":
        for e in kernels:
            e["events"] = "detail pass: K steps after the timed region, the same step with these pairs recorded"
    if in_batch:
        Bg = B * shard_world if sharded else B
        ib_flops = 6.0 * B * Bg * D  # S = U P^T, dU = dS P, dP = dS^T U (S recomputed: not counted)
        # priced against the full split-bf16 ceiling: the kernel forms S twice (user and item roles,
        # 8 B Bg D executed flops), and that second formation is overhead of this kernel, not a lower roof
        ent = mfma_entry(
            f"inbatch_x_kernel (S = U P^T [{B} x {Bg}] + BCE + dU + dP), {impl.replace('6 x', '5 x')}" if not exact_mfma else
            f"inbatch_kernel (S = U P^T [{B} x {Bg}] + BCE + dU + dP, fp32 MFMA 32x32x2)",
            ib_flops, pair_ms(4), MFMA_BF16_PEAK_TFLOPS / 5.0 if split_ceiling else None, "inbatch_bytes_per_launch")
        if split_ceiling:  # five bf16 products per fp32 product in the in-batch kernel (round 6)
            ent["peak_note"] = ("split-bf16 ceiling: v_mfma_f32_32x32x16_bf16 dense peak "
                                f"{MFMA_BF16_PEAK_TFLOPS:.0f} TF/s / 5 bf16 MFMAs per fp32 product (hh, hm, mh, hl, lh)")
        ent["executed_flops_per_launch"] = 8.0 * B * Bg * D
        kernels.append(ent)
    gather = None
    g_ms = pair_ms(12) if args.config == "c4" else 0.0
    if g_ms > 0 and not sharded:
        # the step's ID-row gather (encoders.py:222-223: the user and item tables'
        # rows of the batch, one grouped launch on the aux stream into the [e | f] rows): table-row
        # bytes read against the HBM-read roofline (north_star's gather target), and every byte the
        # copy moves (rows read + rows written + int64 ids)
        g_rows = B + item_rows
        rd = g_rows * D * 4
        tot = g_rows * (2 * D * 4 + 8)
        gather = {"kernel": "gather_rows_wide_seg (the step's user + item ID-row gather)", "bound": "hbm",
                  "rows_per_launch": g_rows, "avg_launch_ms": round(g_ms, 4),
                  "read_bytes_per_launch": rd, "read_GBps": round(rd / g_ms / 1e6, 1),
                  "read_frac": round(rd / g_ms / 1e6 / HBM_PEAK_GBS, 4),
                  "total_bytes_per_launch": tot, "total_GBps": round(tot / g_ms / 1e6, 1),
                  "total_frac": round(tot / g_ms / 1e6 / HBM_PEAK_GBS, 4), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                  "traffic": traffic.get("gather_bytes_per_launch")}
    deferred = not args.eager_adamw
    slice_ms, cu_user_ms, cu_item_ms = pair_ms(0), pair_ms(8), pair_ms(10)
    if deferred:
        # every element of the dense-group tables moves one AdamW(g = 0) step per training step
        # (the rows a step touches take their real update in row_update_kernel instead)
        table_rows = (U + I) if not sharded else (U + I)  # this rank's shards
        es_per_step = table_rows * D
        flush_share = flush_ms / args.steps
        rep_ms = slice_ms + cu_user_ms + cu_item_ms + flush_share
        rv = traffic.get("replay_valu_roofline") or {}
        per_es = rv.get("valu_lane_instr_per_element_step")
        ent = {"bound": "valu",
               "kernel": "replay_kernel (deferred AdamW g=0): rolling slice + user / item catch-up lists + the "
                         "closing flush's share, per step",
               "ms_per_step": round(rep_ms, 4),
               # the catch-up of both towers' touched rows is one replay launch (user + item
               # events when the towers are prepared separately)
               "parts_ms_per_step": {"slice": round(slice_ms, 4), "catchup": round(cu_user_ms + cu_item_ms, 4),
                                     "closing_flush_share": round(flush_share, 4)},
               "element_steps_per_step": es_per_step, "unit": "wave-instr/s", "peak": VALU_WAVE_INSTR_PEAK,
               "valu_lane_instr_per_element_step": per_es,
               "note": "achieved = element-steps per step x VALU lane-instructions per element-step (SQ_INSTS_VALU "
                       "from the committed rocprofv3 pass, profiles/pmc_traffic.json) / 64 / ms_per_step; peak = "
                       "one wave64 VALU instruction per 2 cycles per SIMD (1024 SIMDs, 2.4 GHz)",
               "traffic": rv.get("hbm_bytes_per_step")}
        if per_es and rep_ms > 0:
            ach = es_per_step * per_es / 64 / (rep_ms * 1e-3)
            ent["achieved"] = round(ach, 0)
            ent["frac"] = round(ach / VALU_WAVE_INSTR_PEAK, 4)
        cyc = rv.get("issue_cycles_per_step")
        if cyc and rep_ms > 0:
            # the same work priced per instruction at its measured sustained issue cost
            # (v_sqrt / v_rcp 8.4 SIMD cycles, other VALU 4.08: profiles/r03_valu_issue_rates.txt)
            ent["issue_roofline"] = {
                "issue_cycles_per_step": cyc, "unit": "SIMD cycles at 2.4 GHz",
                "available_per_step": round(rep_ms * 1e-3 * 1024 * 2.4e9),
                "frac": round(cyc / (rep_ms * 1e-3 * 1024 * 2.4e9), 4),
                "cost_model": rv.get("issue_cost_model")}
        kernels.insert(0, ent)
        maint = ent
    else:
        maint_ms = pair_ms(0)
        sweep_bytes = 24 * (U + I) * D
        gbs = sweep_bytes / (maint_ms * 1e-3) / 1e9 if maint_ms > 0 else 0.0
        maint = {"kernel": "dense_sweep_kernel (eager AdamW g=0 over the mimic tables)", "bound": "hbm",
                 "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                 "traffic": traffic.get("dense_sweep_kernel_bytes_per_launch"),
                 "algorithmic_bytes_per_launch": sweep_bytes, "avg_launch_ms": round(maint_ms, 4),
                 "ms_per_step": round(maint_ms, 4)}
        kernels.insert(0, maint)
    roof = max(kernels, key=lambda k: k.get("ms_per_step", 0.0))
    Bg_desc = B * shard_world if sharded else B
    neg_desc = (f"in-batch negatives (all {Bg_desc} positives of the global batch)"
                + (f" + {N} sampled" if N else "")) if in_batch else f"N={N} sampled negatives"
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "interactions/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16 GEMM operands, fp32 accumulate/state" if bf16 else "fp32",
        "data": f"synthetic: {args.config.upper()} shapes, Zipf(1.05) positives (20/user), features shaped like "
                "features.py, random-init weights",
        "config": {
            "workload": f"{args.config.upper()}: {I * shard_world} items x {U * shard_world} users, D={D}, "
                        f"MLP {F}->{H}->{D} (ReLU, dropout {c['dropout']}), gated fusion, adaptive mimic, "
                        f"{'bf16' if bf16 else 'fp32'} tower GEMMs, "
                        f"B={B} per GPU, {neg_desc}, AdamW + SparseAdam",
            "global_batch": B * world,
            "negatives": "in-batch" if in_batch else "sampled",
            "negatives_per_positive": N,
            "parallelism": f"row-sharded tables x{world} (all-to-all) + replicated MLP (all-reduce)"
                           if world > 1 else "single",
            "adamw_tables": ("deferred replay" if deferred else "eager sweep")
                            + (", IEEE g=0 arithmetic" if args.exact_table_math else ", v_sqrt/v_rcp g=0 arithmetic"),
        },
        "final_loss": round(loss, 6),
        "roofline": roof,
        "kernels": kernels,
        "table_maintenance": maint,
        "timeline": {"ms_per_step_excl_closing_flush": round(steps_only_ms, 4),
                     "closing_flush_ms": round(flush_ms, 4),
                     "note": "GPU-event split of the timed region: K steps, then the one flush that brings "
                             "every deferred table row current (part of the K steps' work)"},
        "cpu_baseline": None,
    }
    if exact_line is not None:
        out["exact_table_math"] = exact_line
    if gather is not None:
        out["gather"] = gather
    if args.config == "c4" and not emulate and world == 1 and args.gather_bulk:
        out["gather"] = dict(gather or {}, bulk=gather_bulk(device))
    if emulate:
        out["emulated_world"] = shard_world
        out["config"]["parallelism"] = (f"EMULATED rank 0 of {shard_world}: row-sharded step with mirrored ranks "
                                        "(ttamm.sharded.MirrorComm, no interconnect traffic)")
        out["note"] = ("value = this rank's own interactions/s; a W-rank job's aggregate is at most W x value "
                       "(collectives over xGMI not included)")
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not emulate:
        try:
            out["cpu_baseline"] = cpu_baseline(c, args.cpu_steps, args.cpu_warmup, args.seed, in_batch=in_batch)
        except Exception as exc:  # reported, not fatal to the GPU measurement
            out["cpu_baseline"] = {"error": repr(exc)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
