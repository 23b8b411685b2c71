"""In-batch negatives as one op (ttamm's in-batch mode, BASELINE configs C2 / C4).

The reference scores sampled negatives only (training.py:770-798); the in-batch definition is
ttamm's own (oracle/cpu_reference.py train_step(in_batch=True)): every user is scored against
every positive of the (global) batch, label 1 on its own positive.  ``inbatch_bce`` runs the
fused kernel the training step uses (libttamm ``ttamm_inbatch_bce``, inbatch_x_kernel on
split-bf16 MFMA; nothing batch x n_positives is stored)."""

from __future__ import annotations

import torch

from . import _lib


def inbatch_bce(users: torch.Tensor, positives: torch.Tensor, *, row_base: int = 0,
                inv_count: float | None = None) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """S = users @ positives.T with Y(b, row_base + b) = 1.  Returns (the BCE-with-logits sum over
    S as a float64 device scalar, dL/dusers, dL/dpositives) for L = inv_count * that sum
    (inv_count default 1 / S.numel(), the BCE mean)."""
    _lib.require_rocm(users, "inbatch_bce")
    if users.dim() != 2 or positives.dim() != 2 or users.shape[1] != positives.shape[1]:
        raise ValueError("inbatch_bce: users [B, D] and positives [Bc, D] with one D")
    if users.dtype != torch.float32 or positives.dtype != torch.float32:
        raise ValueError("inbatch_bce: float32 rows")
    B, D = users.shape
    Bc = positives.shape[0]
    if not 0 <= row_base or row_base + B > Bc:
        raise ValueError("inbatch_bce: every user's own positive must lie in positives (row_base + B <= Bc)")
    users = users.contiguous()
    positives = positives.contiguous()
    if inv_count is None:
        inv_count = 1.0 / float(B * Bc)
    lib = _lib.load()
    dev = users.device
    d_users = torch.empty_like(users)
    d_pos = torch.empty_like(positives)
    loss = torch.empty((), dtype=torch.float64, device=dev)
    ws = torch.empty(int(lib.ttamm_inbatch_workspace_size(B, Bc, D)), dtype=torch.uint8, device=dev)
    _lib.check(lib.ttamm_inbatch_bce(users.data_ptr(), B, users.stride(0), positives.data_ptr(), Bc,
                                     positives.stride(0), D, int(row_base), float(inv_count), d_users.data_ptr(),
                                     D, d_pos.data_ptr(), D, loss.data_ptr(), ws.data_ptr(), ws.numel(),
                                     _lib.stream_handle(dev)))
    return loss, d_users, d_pos
