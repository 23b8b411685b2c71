"""CPU restatement of ttamm_route_rows (csrc/route.hip, include/ttamm.h).

TEST INFRASTRUCTURE ONLY: tests/ use it as the checker of the HIP kernel and as the router of
the exchange-layer tests on CPU; the product never imports it.

The reference has no sharded path (SURVEY §8 e); ttamm's row-sharded step routes each item
request to its owner rank (id % world).  The routing is a stable sort of the positions by owner
— exactly torch.argsort(id % world, stable=True) — so this restatement is that sort, and parity
with the kernel is bit-exact (integer work)."""

from __future__ import annotations

import torch


def route_rows(world: int, id0: torch.Tensor, id1: torch.Tensor | None = None, payload: torch.Tensor | None = None,
               key0: int = 0, key1: int = 0, counts_out: torch.Tensor | None = None,
               status: torch.Tensor | None = None) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """(packed [n, 2], slot [n], counts [world]) as ttamm_route_rows defines them; a [world, 2]
    ``counts_out`` gets the counts in column 0 and, with ``status``, the status word in column 1; a
    [world, >= 3] one also the count of id0 ids per owner in column 2, and slot then holds each
    request's first unit of the compact exchange layout (ttamm.h exchange_counts): the groups in
    owner order, each [its id0 ids, two units each | its id1 ids, one unit each]."""
    ids = id0.reshape(-1).cpu() if id1 is None else torch.cat([id0.reshape(-1).cpu(), id1.reshape(-1).cpu()])
    n0 = id0.numel()
    n = ids.numel()
    owner = torch.remainder(ids, world)
    order = torch.argsort(owner, stable=True)  # grouped position -> request position
    slot = torch.empty(n, dtype=torch.long)
    slot[order] = torch.arange(n)
    pos = torch.arange(n)
    second = payload.reshape(-1).cpu() if payload is not None else torch.where(pos < n0, key0 + pos, key1 + (pos - n0))
    packed = torch.stack([torch.div(ids, world, rounding_mode="floor")[order], second[order]], dim=1)
    counts = torch.bincount(owner, minlength=world)
    dev = id0.device
    if counts_out is not None:
        if counts_out.dim() == 2:
            counts_out[:, 0].copy_(counts)
            if status is not None:
                counts_out[:, 1] = int(status.reshape(-1)[0])
            if counts_out.shape[1] >= 3:
                first = torch.bincount(owner[:n0], minlength=world)
                counts_out[:, 2].copy_(first)
                start, pcum = torch.cumsum(counts, 0) - counts, torch.cumsum(first, 0) - first
                slot = slot + pcum[owner] + torch.minimum(slot - start[owner], first[owner])
        else:
            counts_out.copy_(counts)
        counts = counts_out
    return packed.to(dev), slot.to(dev), counts.to(dev)
