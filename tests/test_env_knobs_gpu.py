"""The default library ignores the developer switches: one fused step with
every A/B, ablation and measured-slower variable set leaves bit-for-bit the same model and
optimizer state as the same step without them (csrc/common.h dev_env; the switch list is
tests/test_abi_cpu.py DEV_SWITCHES plus the kernel-placement ones)."""

from __future__ import annotations

import pytest
import torch

from helpers import Shape, make_problem, named_optimizer_state

pytestmark = pytest.mark.gpu

SWITCHES = ("TTAMM_GATE_ABLATE", "TTAMM_GATE_DIRECT_STORES", "TTAMM_GATE_SPLIT", "TTAMM_GATE_4W",
            "TTAMM_GATE16_SPLIT", "TTAMM_GATE_OUT_EPILOGUE", "TTAMM_BF16_WGRAD256", "TTAMM_WGRAD_X16",
            "TTAMM_WGRAD_ALL_NARROW", "TTAMM_WGRAD_WIDE_FIRST", "TTAMM_GEMM_WIDE_TILES", "TTAMM_PROLOGUE_PREP",
            "TTAMM_SLICE_LATE", "TTAMM_SLICE_MAIN", "TTAMM_ROWS_MAIN", "TTAMM_FINALIZE_MAIN", "TTAMM_EARLY_FORK",
            "TTAMM_GATHER_MAIN", "TTAMM_REPLAY_SCALAR", "TTAMM_PIECE_SDA", "TTAMM_FEATURE_PLANES")


def _run(prob):
    from gpu_helpers import run_ttamm

    m, o, losses = run_ttamm(prob, lr=1e-3)
    state = {k: v.detach().clone() for k, v in m.state_dict().items()}
    opt = {n: {k: v.clone() for k, v in st.items() if torch.is_tensor(v)} for n, st in named_optimizer_state(m, o).items()}
    return state, opt, [x["total"] for x in losses]


def test_developer_switches_do_not_change_the_default_library(monkeypatch):
    from ttamm import _lib

    if _lib.load().ttamm_developer_build():
        pytest.skip("a developer library honours the switches by design")
    prob = make_problem(Shape(), steps=2)
    base = _run(prob)
    for name in SWITCHES:
        monkeypatch.setenv(name, "1")
    monkeypatch.setenv("TTAMM_GEMM_TILES", "legacy")
    monkeypatch.setenv("TTAMM_WGRAD_ROWS_PER_SPLIT", "1024")
    monkeypatch.setenv("TTAMM_IB_KERNEL", "p")
    switched = _run(prob)
    assert base[2] == switched[2]
    for k in base[0]:
        assert torch.equal(base[0][k], switched[0][k]), k
    for n in base[1]:
        for k in base[1][n]:
            assert torch.equal(base[1][n][k], switched[1][n][k]), (n, k)
