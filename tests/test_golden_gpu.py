"""The fused MI355X step against the committed golden fixtures (tests/golden/*.npz).
Loss and gradients: 1e-5 norm-wise relative (helpers.rel_err).  After three real optimizer
steps, optimizer moments within 1e-4 and parameters within 5e-5 absolute (Adam normalises
each update to ~lr = 1e-3, so rounding-level gradient differences move a parameter by at most
a small fraction of lr)."""

import pytest
import torch

from golden_io import NAMES, load
from helpers import named_optimizer_state, rel_err

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", NAMES)
def test_step_matches_golden(name):
    from gpu_helpers import run_ttamm

    prob, arr = load(name)
    tm, to, tres = run_ttamm(prob, lr=0.0, betas=(0.0, 0.999), steps=1)
    want = arr["grads/loss"]
    got = [tres[0]["total"], tres[0]["bce"], tres[0]["mimic_user"], tres[0]["mimic_item"]]
    for g, w in zip(got, want):
        assert abs(g - w) <= 1e-5 * max(abs(w), 1e-12)
    grads = named_optimizer_state(tm, to)
    for pname, st in grads.items():
        assert rel_err(st["exp_avg"], torch.from_numpy(arr[f"grads/{pname}"])) <= 1e-5, pname

    tm, to, tres = run_ttamm(prob, steps=3)
    for s, row in enumerate(arr["steps3/loss"]):
        assert abs(tres[s]["total"] - row[0]) <= 1e-5 * abs(row[0])
    for k, v in tm.state_dict().items():
        d = (v.cpu() - torch.from_numpy(arr[f"steps3/param/{k}"])).abs().max().item()
        assert d <= 5e-5, f"{k}: {d:.2e}"
    for pname, st in named_optimizer_state(tm, to).items():
        assert rel_err(st["exp_avg"], torch.from_numpy(arr[f"steps3/exp_avg/{pname}"])) <= 1e-4, pname
        assert rel_err(st["exp_avg_sq"], torch.from_numpy(arr[f"steps3/exp_avg_sq/{pname}"])) <= 1e-4, pname
        assert float(st["step"]) == float(arr[f"steps3/step/{pname}"]), pname
