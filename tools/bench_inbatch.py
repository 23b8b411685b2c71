#!/usr/bin/env python3
"""In-batch scoring kernel benchmark (ttamm.inbatch_bce -> inbatch_x_kernel + ib_reduce_kernel).

    python tools/bench_inbatch.py [--batch 8192] [--positives 65536] [--dim 128] [--reps 20]

Default shape: one rank of the 8-rank C4 step (BASELINE configs[3]): 8192 users x the 65,536
all-gathered positives, D = 128.  Algorithmic work 6 B Bg D flops (S = U P^T, dU = dS P,
dP = dS^T U); the kernel forms S twice (user and item roles), so its split-bf16 ceiling for the
algorithmic flops is (2.5 PF / 6) x 6 / 8 = 312.5 TF/s.  Timed with HIP events on the launch
stream; the first launch is checked against the chunked fp64 oracle definition."""

from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "two-tower-augmented-with-adaptive-mimic-mechanism_amd"))
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

CEILING = 2500.0 / 6.0 * 6.0 / 8.0


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--positives", type=int, default=65536)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--no-check", action="store_true")
    args = ap.parse_args()
    import ttamm

    B, Bc, D = args.batch, args.positives, args.dim
    g = torch.Generator(device="cuda").manual_seed(11)
    u = torch.randn((B, D), device="cuda", generator=g) * 0.3
    p = torch.randn((Bc, D), device="cuda", generator=g) * 0.3
    row_base = (Bc - B) // 2
    p[row_base:row_base + B] += 0.5 * u
    inv = 1.0 / (Bc * Bc)
    loss, du, dp = ttamm.inbatch_bce(u, p, row_base=row_base, inv_count=inv)
    torch.cuda.synchronize()
    err = None
    if not args.no_check:
        from oracle import cpu_reference as ref

        wl, wdu, wdp = ref.inbatch_bce_chunked(u, p, row_base=row_base, inv_count=inv)
        err = {"loss": abs(float(loss) - wl) / abs(wl),
               "dU": float((du.double() - wdu).abs().max() / wdu.abs().max()),
               "dP": float((dp.double() - wdp).abs().max() / wdp.abs().max())}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(args.reps):
        ttamm.inbatch_bce(u, p, row_base=row_base, inv_count=inv)
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / args.reps
    flops = 6.0 * B * Bc * D
    tf = flops / (ms * 1e-3) / 1e12
    print(json.dumps({"kernel": "inbatch_x_kernel + ib_reduce_kernel (ttamm_inbatch_bce)", "B": B, "Bc": Bc, "D": D,
                      "ms_per_launch": round(ms, 4), "achieved_tflops": round(tf, 2),
                      "peak": round(CEILING, 1), "frac": round(tf / CEILING, 4), "rel_err_vs_fp64": err}),
          flush=True)


if __name__ == "__main__":
    main()
