"""Diagnostic: the C2 deferred-vs-eager bitwise comparison broken down (repeatability of each
mode, exact vs fast g = 0 arithmetic, which rows / which tensors differ)."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


def run(deferred, math, steps=4, seed=8, overlap=True):
    c2 = bench.CONFIGS["c2"]
    w = bench.Workload(c2, torch.device("cuda"), seed=seed, deferred=deferred, table_math=math, overlap=overlap)
    batches = []
    for _ in range(steps):
        u, p = w.batch()
        batches.append((u.clone(), p.clone()))
        w.engine.step(u, p)
    w.engine.finish()
    mm = w.model.adaptive_mimic
    st = w.opts[0].state[mm.item_augmented.weight]
    out = dict(w=mm.item_augmented.weight.detach().clone(), m=st["exp_avg"].clone(), v=st["exp_avg_sq"].clone())
    stu = w.opts[0].state[mm.user_augmented.weight]
    out.update(uw=mm.user_augmented.weight.detach().clone(), um=stu["exp_avg"].clone(), uv=stu["exp_avg_sq"].clone())
    out["batches"] = batches
    del w
    torch.cuda.empty_cache()
    return out


def cmp(tag, a, b):
    for k in ("w", "m", "v", "uw", "um", "uv"):
        d = (a[k] != b[k])
        n = int(d.sum())
        rows = d.any(dim=1).nonzero().flatten()
        mx = (a[k] - b[k]).abs().max().item()
        print(f"{tag} {k}: {n} elements differ in {rows.numel()} rows, max |diff| {mx:.3e}, first rows {rows[:8].tolist()}")
    same_b = all(torch.equal(x[0], y[0]) and torch.equal(x[1], y[1]) for x, y in zip(a["batches"], b["batches"]))
    print(f"{tag} batches identical: {same_b}")


import os

if os.environ.get("DIAG_MODE") == "overlap":
    for ov in (False, True):
        a = run(True, "fast", overlap=ov)
        b = run(True, "fast", overlap=ov)
        cmp(f"[fast overlap={ov}] deferred vs deferred", a, b)
        e = run(False, "fast", overlap=ov)
        cmp(f"[fast overlap={ov}] eager vs deferred", e, a)
        sys.stdout.flush()
    sys.exit(0)
if os.environ.get("DIAG_MODE") == "repeat":
    base = run(True, "fast")
    for r in range(4):
        cmp(f"[fast repeat {r}] deferred vs deferred", base, run(True, "fast"))
        sys.stdout.flush()
    sys.exit(0)
if os.environ.get("DIAG_MODE") == "scalar":
    a = run(True, "fast")
    b = run(True, "fast")
    cmp("[fast replay_s] deferred vs deferred", a, b)
    e = run(False, "fast")
    cmp("[fast replay_s] eager vs deferred", e, a)
    sys.exit(0)
for math in ("fast", "exact"):
    e1 = run(False, math)
    e2 = run(False, math)
    cmp(f"[{math}] eager vs eager", e1, e2)
    d1 = run(True, math)
    cmp(f"[{math}] eager vs deferred", e1, d1)
    d2 = run(True, math)
    cmp(f"[{math}] deferred vs deferred", d1, d2)
    if math == "fast":
        # which item rows were touched (positives / negatives of the 4 batches)?
        touched = torch.zeros(e1["w"].shape[0], dtype=torch.bool, device="cuda")
        for u, p in e1["batches"]:
            touched[p] = True
        diff_rows = (e1["w"] != d1["w"]).any(dim=1)
        print("differing rows that were positives:", int((diff_rows & touched).sum()), "untouched:",
              int((diff_rows & ~touched).sum()))
        m0 = (e1["m"] == 0).all(dim=1)
        print("differing rows with m == 0 (cold):", int((diff_rows & m0).sum()))
    sys.stdout.flush()
