"""Host-side cost of the row-sharded step (emulated W ranks, bench.py's C2 workload): the
Python / ctypes / torch time the host spends enqueuing each step, from cProfile over the timed
steps only, next to the GPU time per step.  Prints per-function totals per step (microseconds).

python tools/prof_host.py [--emulate-world 8] [--steps 200]
"""

from __future__ import annotations

import argparse
import cProfile
import pstats
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--emulate-world", type=int, default=8)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--no-look-ahead", action="store_true")
    ap.add_argument("--top", type=int, default=45)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    c = dict(bench.CONFIGS["c2"])
    w = bench.Workload(c, dev, 0, world=args.emulate_world, rank=0, step_seed=0, emulate=True)
    eng = w.engine
    nxt = [w.batch()]

    def step():
        u, p = nxt[0]
        nxt[0] = w.batch()
        if args.no_look_ahead:
            eng.step(u, p)
        else:
            eng.step(u, p, next_batch=nxt[0])

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"plain: host enqueue {1e6 * (t1 - t0) / args.steps:.1f} us/step, wall {1e6 * (t2 - t0) / args.steps:.1f} "
          f"us/step")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(args.steps):
        step()
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    rows = []
    for (fn, line, name), (cc, nc, tt, ct, _) in st.stats.items():
        rows.append((tt, ct, nc, f"{Path(fn).name}:{line}({name})"))
    print(f"\nby own time (us per step), {args.steps} steps under cProfile")
    for tt, ct, nc, name in sorted(rows, reverse=True)[: args.top]:
        print(f"  own {1e6 * tt / args.steps:8.1f}  cum {1e6 * ct / args.steps:8.1f}  calls/step {nc / args.steps:6.1f}  {name}")
    print("\nby cumulative time (ttamm / bench functions)")
    for tt, ct, nc, name in sorted(((r[1], r[0], r[2], r[3]) for r in rows), reverse=True):
        if any(k in name for k in ("sharded.py", "training.py", "_lib.py", "bench.py", "data.py")):
            print(f"  cum {1e6 * tt / args.steps:8.1f}  own {1e6 * ct / args.steps:8.1f}  calls/step {nc / args.steps:6.1f}  {name}")


if __name__ == "__main__":
    main()
