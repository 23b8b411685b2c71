#!/usr/bin/env python3
"""C3 retrieval benchmark (SURVEY §8 f1 / BASELINE configs C3): exact inner-product top-K over
a 2M x 96 item matrix for a 65,536-query batch, K = 80 (faiss_search_k = 20 x 4,
training.py:1413-1415), 20 blocked train positives per query.

    python tools/bench_retrieval.py [--queries 65536] [--items 2000000] [--dim 96] [--k 80]

Prints one JSON line: queries/s, the kernel's fp32 MFMA rate (algorithmic 2*Q*I*D FLOPs over
HIP-event time on the launch stream) and a CPU baseline: numpy float32 matmul + argpartition
(the work faiss.IndexFlatIP does) on a bounded query sample, on this host's cores."""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "two-tower-augmented-with-adaptive-mimic-mechanism_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

MFMA_FP32_PEAK_TFLOPS = 157.3
# the split kernel computes each fp32 product as 6 bf16 MFMA products: its ceiling is the dense
# bf16 MFMA peak / 6 (MI355X_MICROARCH.md: 2.5 PF/s dense bf16)
SPLIT_BF16_CEILING_TFLOPS = 2500.0 / 6


def cpu_baseline(items: np.ndarray, queries: np.ndarray, k: int) -> dict:
    threads = len(os.sched_getaffinity(0))
    t0 = time.perf_counter()
    n = 0
    for lo in range(0, queries.shape[0], 256):
        s = queries[lo:lo + 256] @ items.T
        part = np.argpartition(-s, k, axis=1)[:, :k]
        np.take_along_axis(s, part, axis=1)
        n += s.shape[0]
    secs = time.perf_counter() - t0
    return {"value": round(n / secs, 1), "unit": "queries/s", "cores": threads, "kind": "port",
            "sample": f"{n} queries x {items.shape[0]} items x {items.shape[1]}: numpy fp32 matmul + argpartition "
                      f"(faiss IndexFlatIP's work), BLAS threads = host cores"}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--queries", type=int, default=65536)
    ap.add_argument("--items", type=int, default=2_000_000)
    ap.add_argument("--dim", type=int, default=96)
    ap.add_argument("--k", type=int, default=80)
    ap.add_argument("--blocked", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cpu-queries", type=int, default=1024)
    args = ap.parse_args()
    from ttamm.retrieval import retrieve_topk

    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    nq, ni, D, k = args.queries, args.items, args.dim, args.k
    items = torch.randn((ni, D), device=dev, generator=g)
    queries = torch.randn((nq, D), device=dev, generator=g)
    nb = args.blocked
    boff = bval = None
    if nb > 0:
        boff = torch.arange(0, nb * nq + 1, nb, device=dev)
        bval = torch.randint(0, ni, (nq, nb), device=dev, generator=g).sort(dim=1).values.reshape(-1)
    retrieve_topk(queries, items, k, blocked_offsets=boff, blocked_values=bval)  # warm-up
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.reps)]
    t0 = time.perf_counter()
    for a, b in ev:
        a.record()
        retrieve_topk(queries, items, k, blocked_offsets=boff, blocked_values=bval)
        b.record()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.reps
    ms = sum(a.elapsed_time(b) for a, b in ev) / args.reps
    flops = 2.0 * nq * ni * D
    split = D <= 128 and "TTAMM_RETRIEVAL_FP32" not in os.environ  # retrieval.hip retrieval_split()
    tf = flops / (ms * 1e-3) / 1e12
    cpu = (cpu_baseline(items[: ni].cpu().numpy(), queries[: args.cpu_queries].cpu().numpy(), k)
           if args.cpu_queries > 0 else None)
    # HBM bytes per launch of the scan kernel from the committed rocprofv3 PMC passes
    # (profiles/pmc_traffic.json "c3", tools/gpu/pmc_c3.sh), at the default C3 shape only
    traffic = None
    if (nq, ni, D, k, nb) == (65536, 2_000_000, 96, 80, 20):
        try:
            traffic = json.loads((ROOT / "profiles" / "pmc_traffic.json").read_text())["c3"]["retrieval_bytes_per_launch"]
        except (OSError, ValueError, KeyError):
            traffic = None
    print(json.dumps({
        "metric": "C3 exact-IP retrieval top-K (queries/s)",
        "value": round(nq / (ms * 1e-3), 1),
        "unit": "queries/s",
        "config": {"queries": nq, "items": ni, "dim": D, "k": k, "blocked_per_query": nb},
        "ms_per_batch": round(ms, 3),
        "wall_ms_per_batch": round(wall * 1e3, 3),
        "roofline": ({"bound": "mfma", "kernel": "retrieval_x_kernel (split-bf16 scan + in-kernel top-K merge)",
                      "achieved": round(tf, 2), "peak": round(SPLIT_BF16_CEILING_TFLOPS, 1), "unit": "TFLOP/s",
                      "frac": round(tf / SPLIT_BF16_CEILING_TFLOPS, 4),
                      "peak_basis": "dense bf16 MFMA peak / 6 (six bf16 products per fp32 product)",
                      "vs_fp32_mfma_peak": round(tf / MFMA_FP32_PEAK_TFLOPS, 4), "algorithmic_flops": flops,
                      "traffic": traffic}
                     if split else
                     {"bound": "mfma", "kernel": "retrieval_partial_kernel + retrieval_merge_kernel (fp32 MFMA)",
                      "achieved": round(tf, 2), "peak": MFMA_FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                      "frac": round(tf / MFMA_FP32_PEAK_TFLOPS, 4), "algorithmic_flops": flops}),
        "cpu_baseline": cpu,
    }), flush=True)


if __name__ == "__main__":
    main()
