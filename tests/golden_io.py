"""Load committed golden fixtures (tests/golden/*.npz) back into problems."""

from __future__ import annotations

from pathlib import Path

import numpy as np
import torch

from helpers import Problem
from oracle import cpu_reference as ref

GOLDEN = Path(__file__).resolve().parent / "golden"
NAMES = ("tiny_gated_mimic", "odd_dims_2hidden", "dense_id_nomimic")


def load(name: str):
    import importlib.util

    spec = importlib.util.spec_from_file_location("make_golden", GOLDEN / "make_golden.py")
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    shape = mg.shape_of(name)
    data = np.load(GOLDEN / f"{name}.npz")  # allow_pickle=False (default)
    arr = {k: data[k] for k in data.files}
    model = ref.build_model(shape.tower_cfg(), num_users=shape.U, num_items=shape.I, user_feature_dim=shape.F,
                            item_feature_dim=shape.F, mimic=shape.mimic)
    init = {k[len("init/"):]: torch.from_numpy(v) for k, v in arr.items() if k.startswith("init/")}
    model.load_state_dict(init, strict=True)
    prob = Problem(shape, model, torch.from_numpy(arr["inputs/user_features"]),
                   torch.from_numpy(arr["inputs/item_features"]), positives={})
    s = 0
    while f"batch{s}/users" in arr:
        nh = len(shape.hidden_dims)
        um = [torch.from_numpy(arr[f"batch{s}/user_keep{l}"]) for l in range(nh) if f"batch{s}/user_keep{l}" in arr]
        im = [torch.from_numpy(arr[f"batch{s}/item_keep{l}"]) for l in range(nh) if f"batch{s}/item_keep{l}" in arr]
        prob.batches.append((torch.from_numpy(arr[f"batch{s}/users"]), torch.from_numpy(arr[f"batch{s}/pos"]),
                             torch.from_numpy(arr[f"batch{s}/neg"]), um, im))
        s += 1
    return prob, arr
