#!/usr/bin/env python3
"""Developer probe: does HIP stream priority keep the aux stream's row work off the main
stream's GEMMs?  C2 one-process step, alternating arms on one box, ms/step of K steps + flush.

    python3 tools/diag/prio_probe.py [--steps 20] [--rounds 3]

Arms: default (caller's stream, aux at default priority); aux_low (aux stream created at the
least priority); main_high (the steps enqueued on a greatest-priority stream, aux default);
both."""
from __future__ import annotations

import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "two-tower-augmented-with-adaptive-mimic-mechanism_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--config", default="c2")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    least, greatest = torch.cuda.Stream.priority_range()
    print(f"priority range: least {least} greatest {greatest}", flush=True)
    c = dict(bench.CONFIGS[a.config])
    w = bench.Workload(c, dev, 1234)
    eng = w.engine
    aux_default = eng.aux_stream
    aux_low = torch.cuda.Stream(device=dev, priority=least)
    main_high = torch.cuda.Stream(device=dev, priority=greatest)
    print(f"aux_low priority {aux_low.priority}, main_high priority {main_high.priority}", flush=True)

    def run(aux, main) -> float:
        eng.aux_stream = aux
        eng.args.aux_stream = aux.cuda_stream
        with torch.cuda.stream(main):
            for _ in range(a.warmup):
                u, p = w.batch()
                eng.step(u, p)
            eng.flush()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                u, p = w.batch()
                eng.step(u, p)
            eng.flush()
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) / a.steps * 1e3

    cur = torch.cuda.current_stream(dev)
    arms = [("default", aux_default, cur), ("aux_low", aux_low, cur), ("main_high", aux_default, main_high),
            ("both", aux_low, main_high)]
    for r in range(a.rounds):
        for name, aux, main in arms:
            ms = run(aux, main)
            print(f"round {r} {name:10s} {ms:.4f} ms/step  {c['B'] / ms * 1e3:,.0f} interactions/s", flush=True)


if __name__ == "__main__":
    main()
