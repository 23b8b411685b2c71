"""Negative sampling — drop-in for ``src/data/samplers.py`` (samplers.py:11-85).

The reference loops over the batch in Python, drawing ``num_negatives`` uniform items per
row with ``torch.randint`` and redrawing those that hit the user's known positives
(``torch.isin`` against a per-user tensor), raising after too many redraw rounds.  Here the
positives are a device-resident CSR (per-user sorted ids) and one gfx950 kernel samples the
whole batch: every slot walks its own counter-based Philox stream and binary-searches the
user's positives (``ttamm_sample_negatives``).  The draws are therefore not the CPU
``torch.randint`` stream; the contract kept is the reference's: uniform over
[0, num_items) minus the user's positives, same errors.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Mapping, Set

import numpy as np
import torch

from . import _lib


@dataclass
class PositivesCSR:
    """Each user's positive item ids, sorted: values[offsets[u]:offsets[u+1]]."""

    offsets: torch.Tensor  # int64 [num_users + 1]
    values: torch.Tensor  # int64 [nnz]
    num_users: int
    max_degree: int

    @classmethod
    def from_mapping(cls, positives: Mapping[int, Set[int]], *, device: torch.device, num_users: int | None = None) -> "PositivesCSR":
        n = max(num_users or 0, (max(positives) + 1) if positives else 0)
        counts = np.zeros(n + 1, dtype=np.int64)
        for u, items in positives.items():
            counts[int(u) + 1] = len(items)
        offsets = np.cumsum(counts)
        values = np.empty(int(offsets[-1]), dtype=np.int64)
        for u, items in positives.items():
            lo = offsets[int(u)]
            values[lo : lo + len(items)] = np.sort(np.fromiter(items, dtype=np.int64, count=len(items)))
        return cls.from_arrays(offsets, values, device=device)

    @classmethod
    def from_arrays(cls, offsets, values, *, device: torch.device) -> "PositivesCSR":
        off = torch.as_tensor(offsets, dtype=torch.long)
        val = torch.as_tensor(values, dtype=torch.long)
        deg = int((off[1:] - off[:-1]).max().item()) if off.numel() > 1 else 0
        return cls(off.to(device), val.to(device), off.numel() - 1, deg)


_csr_cache: dict[tuple, PositivesCSR] = {}


def positives_csr(positives, *, device: torch.device, num_users: int | None = None) -> PositivesCSR:
    """The device CSR of a dict[user] -> set(items), cached per mapping.  The key holds the user
    count and the total positive count, so a caller that grows (or shrinks) a user's set in place
    gets a rebuilt CSR; an in-place edit that keeps both counts (one item swapped for another)
    needs a fresh mapping or an explicit PositivesCSR."""
    if isinstance(positives, PositivesCSR):
        return positives
    total = sum(len(items) for items in positives.values())
    key = (id(positives), len(positives), total, str(device))
    hit = _csr_cache.get(key)
    if hit is None or (num_users is not None and hit.num_users < num_users):
        hit = PositivesCSR.from_mapping(positives, device=device, num_users=num_users)
        _csr_cache.clear()
        _csr_cache[key] = hit
    return hit


def draw_seed() -> int:
    """A 64-bit Philox key drawn from torch's global generator (reproducible under
    ``torch.manual_seed`` as in training.py:185-190)."""
    hi = int(torch.randint(0, 2**31, (1,)).item())
    lo = int(torch.randint(0, 2**31, (1,)).item())
    return (hi << 32) | lo


def sample_negative_items(
    user_indices: torch.Tensor,
    *,
    num_items: int,
    positives: Mapping[int, Set[int]] | PositivesCSR,
    num_negatives: int,
    device: torch.device,
) -> torch.Tensor:
    """[batch, num_negatives] int64 negatives for each user (samplers.py:11-85)."""
    if num_negatives <= 0:
        raise ValueError("num_negatives must be greater than zero.")
    if num_items <= 1:
        raise ValueError("num_items must be greater than one.")
    device = torch.device(device)
    users = user_indices.to(device=device, dtype=torch.long).reshape(-1).contiguous()
    _lib.require_rocm(users, "sample_negative_items")
    need = int(users.max().item()) + 1 if users.numel() else 0
    if users.numel() and int(users.min().item()) < 0:
        # positives.get(u, set()) in the reference: an id with no entry has no positives; point
        # negative ids at an empty CSR row past the largest user
        need = max(need, (max(positives) + 1) if isinstance(positives, Mapping) and positives else 0,
                   positives.num_users if isinstance(positives, PositivesCSR) else 0)
        users = torch.where(users < 0, torch.full_like(users, need), users)
        need += 1
    csr = positives_csr(positives, device=device, num_users=need)
    if csr.max_degree >= num_items:
        degrees = (csr.offsets[1:] - csr.offsets[:-1]).index_select(0, users.clamp(max=csr.num_users - 1))
        full = (degrees >= num_items) & (users < csr.num_users)
        if bool(full.any()):
            u = int(users[full.nonzero()[0, 0]].item())
            raise RuntimeError(f"User {u} interacted with all items; cannot sample negatives.")
    out = torch.empty((users.numel(), num_negatives), dtype=torch.long, device=device)
    status = torch.zeros(1, dtype=torch.int32, device=device)
    lib = _lib.load()
    _lib.check(
        lib.ttamm_sample_negatives(
            users.data_ptr(), users.numel(), num_negatives, num_items, csr.offsets.data_ptr(), csr.values.data_ptr(),
            csr.offsets.numel() - 1, draw_seed(), 0, 0, out.data_ptr(), status.data_ptr(), _lib.stream_handle(device),
        )
    )
    if int(status.item()) & _lib.STATUS_SAMPLER_EXHAUSTED:
        raise RuntimeError("Exceeded resampling attempts while drawing negatives.")
    return out
