#!/usr/bin/env python3
"""Regenerate the committed golden fixtures from the CPU oracle (oracle/cpu_reference.py).

    python tests/golden/make_golden.py

Each fixture holds one tiny problem (SURVEY.md §7 step 1 shapes: U=64, I=256, F=12, H=16,
D=8, B=32, N=5), its inputs (initial parameters, feature rows, batches with injected
negatives and dropout keep-masks) and the oracle's outputs:
  * grads:  one step with lr = 0, beta1 = 0 — every optimizer's exp_avg then equals the
            parameter's gradient exactly (torch lerp with weight 1; SparseAdam (g - 0) * 1);
  * steps3: three steps of AdamW(lr 1e-3, wd 0.01) + SparseAdam(lr 1e-3): per-step losses,
            final parameters and optimizer state.
The fixtures are data (inputs and expected outputs); nothing of the reference is stored.
"""

from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]

from helpers import Shape, make_problem, named_optimizer_state, run_oracle  # noqa: E402

OUT = Path(__file__).resolve().parent

CASES = {
    "tiny_gated_mimic": Shape(),
    "odd_dims_2hidden": Shape(U=48, I=200, F=37, D=12, B=24, N=3, gate_hidden=20, hidden_dims=(24, 16)),
    "dense_id_nomimic": Shape(sparse=False, mimic=False),
}


def pack(prefix: str, d: dict, out: dict) -> None:
    for k, v in d.items():
        out[f"{prefix}/{k}"] = v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v)


def build(name: str, shape: Shape) -> dict:
    prob = make_problem(shape, steps=3)
    arrays: dict[str, np.ndarray] = {}
    pack("init", prob.model.state_dict(), arrays)
    arrays["inputs/user_features"] = prob.user_features.numpy()
    arrays["inputs/item_features"] = prob.item_features.numpy()
    for s, (users, pos, neg, um, im) in enumerate(prob.batches):
        arrays[f"batch{s}/users"] = users.numpy()
        arrays[f"batch{s}/pos"] = pos.numpy()
        arrays[f"batch{s}/neg"] = neg.numpy()
        for l, m in enumerate(um):
            arrays[f"batch{s}/user_keep{l}"] = m.numpy()
        for l, m in enumerate(im):
            arrays[f"batch{s}/item_keep{l}"] = m.numpy()
    gm, go, gres = run_oracle(prob, lr=0.0, betas=(0.0, 0.999), steps=1)
    arrays["grads/loss"] = np.array([gres[0].total, gres[0].bce, gres[0].mimic_user, gres[0].mimic_item])
    for pname, st in named_optimizer_state(gm, go).items():
        arrays[f"grads/{pname}"] = st["exp_avg"].numpy()
    sm, so, sres = run_oracle(prob, steps=3)
    arrays["steps3/loss"] = np.array([[r.total, r.bce, r.mimic_user, r.mimic_item] for r in sres])
    pack("steps3/param", sm.state_dict(), arrays)
    for pname, st in named_optimizer_state(sm, so).items():
        arrays[f"steps3/exp_avg/{pname}"] = st["exp_avg"].numpy()
        arrays[f"steps3/exp_avg_sq/{pname}"] = st["exp_avg_sq"].numpy()
        arrays[f"steps3/step/{pname}"] = np.asarray(float(st["step"]))
    return arrays


def shape_of(name: str) -> Shape:
    return CASES[name]


def main() -> None:
    for name, shape in CASES.items():
        arrays = build(name, shape)
        np.savez_compressed(OUT / f"{name}.npz", **arrays)
        print(f"wrote {name}.npz ({len(arrays)} arrays)")


if __name__ == "__main__":
    main()
