"""The in-batch scoring kernel as one op (ttamm.inbatch_bce -> ttamm_inbatch_bce ->
inbatch_x_kernel) against a chunked float64 evaluation of the oracle's in-batch definition
(oracle/cpu_reference.inbatch_bce_chunked; train_step(in_batch=True)), at the shapes the
training step launches it with:

  * C2 in-batch (BASELINE configs[1]): B = 8192 users x 8192 positives, D = 96;
  * C4 at 8 ranks (BASELINE configs[3]): one rank's 8192 users x the all-gathered 65,536 positives,
    D = 128, the rank's label diagonal at row_base = 3 x 8192 and the global 1 / (B_global Bg);
  * small ragged shapes (rows not a multiple of the 128-row blocks / 64-column tiles).

Tolerance: 1e-5 relative on the BCE sum, 1e-5 norm-wise (max|ours - fp64| / max|fp64|) on dU and dP."""

from __future__ import annotations

import pytest
import torch

import ttamm
from oracle import cpu_reference as ref

pytestmark = pytest.mark.gpu

TOL = 1e-5


def _rel(a: torch.Tensor, b: torch.Tensor) -> float:
    return float((a.double() - b).abs().max() / b.abs().max())


@pytest.mark.parametrize("B,Bc,D,row_base,scale", [
    (300, 300, 96, 0, 0.3),
    (200, 900, 128, 450, 0.3),
    (77, 77, 12, 0, 0.5),
    (8192, 8192, 96, 0, 0.3),
    (8192, 65536, 128, 3 * 8192, 0.3),
], ids=["c2-dims-small", "sharded-small", "odd-d12", "c2-inbatch-full", "c4-rank3-of-8"])
def test_inbatch_op_matches_fp64_definition(B, Bc, D, row_base, scale):
    g = torch.Generator(device="cuda").manual_seed(B + Bc + D)
    users = torch.randn((B, D), device="cuda", generator=g) * scale
    pos = torch.randn((Bc, D), device="cuda", generator=g) * scale
    # the own positive scores higher, as after training (label-1 logits away from 0)
    pos[row_base:row_base + B] += 0.5 * users
    world_batch = Bc if Bc > B else B  # sharded: the global batch is all the gathered positives
    inv = 1.0 / (world_batch * Bc)
    loss, du, dp = ttamm.inbatch_bce(users, pos, row_base=row_base, inv_count=inv)
    torch.cuda.synchronize()
    want_loss, want_du, want_dp = ref.inbatch_bce_chunked(users, pos, row_base=row_base, inv_count=inv)
    assert abs(float(loss) - want_loss) <= TOL * abs(want_loss), (float(loss), want_loss)
    assert _rel(du, want_du) <= TOL, _rel(du, want_du)
    assert _rel(dp, want_dp) <= TOL, _rel(dp, want_dp)


def test_inbatch_op_rejects_bad_shapes():
    u = torch.zeros((16, 32), device="cuda")
    with pytest.raises(ValueError):
        ttamm.inbatch_bce(u, torch.zeros((16, 24), device="cuda"))
    with pytest.raises(ValueError):
        ttamm.inbatch_bce(u, torch.zeros((20, 32), device="cuda"), row_base=8)
