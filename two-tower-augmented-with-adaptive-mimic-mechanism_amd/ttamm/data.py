"""HBM-resident training data: binary interaction / feature files and an on-device loader.

The reference builds its loader from pandas each run (training.py:260-264):

    DataLoader(InteractionDataset(train_df), batch_size=batch_size, shuffle=True, drop_last=False)

with InteractionDataset holding (user_idx, item_idx) as int64 tensors (datasets.py:12-45) and
the feature matrices built by src/data/features.py.  ttamm keeps the same contract on the
device:

* ``save_interactions`` / ``load_interactions`` — the pairs as a flat binary file (64-byte
  header, then int64 users[n], int64 items[n]), memory-mapped and copied to HBM in chunks;
* ``save_features`` / ``load_features`` — a float32 matrix with rows padded to a multiple of 4
  floats (the layout ttamm_tower.features reads: 16-byte aligned rows, zero padding);
* ``DeviceInteractionLoader`` — an iterable over one epoch's batches, each a pair of int64
  device tensors (users, items) like the DataLoader's, written by ttamm_epoch_batch: the epoch
  order is a seeded bijection evaluated on the device (no host shuffle, no collation), the
  last batch short unless ``drop_last``.  ``set_epoch`` advances the order, as a new
  DataLoader iterator does.

Any iterable of (users, items) batches works with ``ttamm.train_one_epoch``; this one keeps the
whole input path on the GPU.
"""

from __future__ import annotations

import ctypes
import os
import struct
from dataclasses import dataclass
from pathlib import Path

import numpy as np
import torch

from . import _lib

_I_MAGIC = b"TTAMMI01"
_F_MAGIC = b"TTAMMF01"
_HEADER = 64
_CHUNK_ROWS = 1 << 22  # host -> device copies in 4M-row pieces (bounded host memory)


@dataclass(frozen=True)
class InteractionMeta:
    n: int
    num_users: int
    num_items: int


def save_interactions(path: str | os.PathLike, users: torch.Tensor, items: torch.Tensor, *,
                      num_users: int | None = None, num_items: int | None = None) -> InteractionMeta:
    """Write (users[i], items[i]) pairs: header (magic, n, num_users, num_items), int64 users,
    int64 items.  ``num_users`` / ``num_items`` default to max id + 1."""
    u = torch.as_tensor(users).detach().to("cpu", torch.int64).reshape(-1)
    v = torch.as_tensor(items).detach().to("cpu", torch.int64).reshape(-1)
    if u.numel() != v.numel():
        raise ValueError("ttamm: users and items must have the same length")
    if u.numel() and (int(u.min()) < 0 or int(v.min()) < 0):
        raise ValueError("ttamm: interaction ids must be non-negative")
    nu = int(num_users) if num_users is not None else (int(u.max()) + 1 if u.numel() else 0)
    ni = int(num_items) if num_items is not None else (int(v.max()) + 1 if v.numel() else 0)
    if u.numel() and (int(u.max()) >= nu or int(v.max()) >= ni):
        raise ValueError("ttamm: an interaction id is outside [0, num_users) x [0, num_items)")
    meta = InteractionMeta(u.numel(), nu, ni)
    with open(path, "wb") as f:
        f.write(struct.pack("<8sqqq", _I_MAGIC, meta.n, meta.num_users, meta.num_items).ljust(_HEADER, b"\0"))
        f.write(u.numpy().tobytes())
        f.write(v.numpy().tobytes())
    return meta


def _read_header(path: str | os.PathLike, magic: bytes) -> tuple[int, int, int]:
    with open(path, "rb") as f:
        head = f.read(_HEADER)
    if len(head) != _HEADER or head[:8] != magic:
        raise ValueError(f"ttamm: {path} is not a ttamm {magic[5:6].decode()} file")
    return struct.unpack_from("<qqq", head, 8)


_DTYPES = {np.dtype("<i8"): torch.int64, np.dtype("<f4"): torch.float32}


def _to_device(mm: np.ndarray, device: torch.device) -> torch.Tensor:
    out = torch.empty(mm.shape, dtype=_DTYPES[mm.dtype], device=device)
    for lo in range(0, mm.shape[0], _CHUNK_ROWS):
        hi = min(mm.shape[0], lo + _CHUNK_ROWS)
        out[lo:hi].copy_(torch.from_numpy(np.array(mm[lo:hi])))  # one writable host chunk at a time
    return out


def load_interactions(path: str | os.PathLike, device: torch.device | str = "cuda"
                      ) -> tuple[torch.Tensor, torch.Tensor, InteractionMeta]:
    """(users, items, meta): int64 tensors on ``device`` (memory-mapped, copied in chunks)."""
    n, nu, ni = _read_header(path, _I_MAGIC)
    if n < 0 or Path(path).stat().st_size != _HEADER + 16 * n:
        raise ValueError(f"ttamm: {path} is truncated or has a bad header")
    mm = np.memmap(path, dtype="<i8", mode="r", offset=_HEADER, shape=(2, n))
    dev = torch.device(device)
    return _to_device(mm[0], dev), _to_device(mm[1], dev), InteractionMeta(n, nu, ni)


def save_features(path: str | os.PathLike, features: torch.Tensor) -> None:
    """Write a [rows, cols] float32 matrix with rows padded to a multiple of 4 floats."""
    x = torch.as_tensor(features).detach().to("cpu", torch.float32)
    if x.dim() != 2:
        raise ValueError("ttamm: features must be a 2-D matrix")
    rows, cols = x.shape
    ld = (cols + 3) // 4 * 4
    with open(path, "wb") as f:
        f.write(struct.pack("<8sqqq", _F_MAGIC, rows, cols, ld).ljust(_HEADER, b"\0"))
        for lo in range(0, rows, _CHUNK_ROWS):
            hi = min(rows, lo + _CHUNK_ROWS)
            blk = torch.zeros((hi - lo, ld), dtype=torch.float32)
            blk[:, :cols] = x[lo:hi]
            f.write(blk.numpy().tobytes())


def load_features(path: str | os.PathLike, device: torch.device | str = "cuda") -> torch.Tensor:
    """The [rows, cols] matrix on ``device`` as a view of its padded [rows, ld] storage (the
    row stride ttamm_tower.feat_ld; FusedTrainStep uses it without a copy)."""
    rows, cols, ld = _read_header(path, _F_MAGIC)
    if rows < 0 or not 0 <= cols <= ld or ld % 4 or Path(path).stat().st_size != _HEADER + 4 * rows * ld:
        raise ValueError(f"ttamm: {path} is truncated or has a bad header")
    mm = np.memmap(path, dtype="<f4", mode="r", offset=_HEADER, shape=(rows, ld))
    return _to_device(mm, torch.device(device))[:, :cols]


class DeviceInteractionLoader:
    """On-device DataLoader(InteractionDataset, batch_size, shuffle, drop_last) over HBM pairs.

    Iterating yields (users, items) int64 device tensors of ``batch_size`` rows (the last one
    short unless ``drop_last``), in the order ttamm_epoch_batch defines for (``seed``, epoch).
    The epoch advances by one after every full iteration (or set it with ``set_epoch``), so
    successive epochs see different orders, like successive DataLoader iterators."""

    def __init__(self, users: torch.Tensor, items: torch.Tensor, batch_size: int, *, shuffle: bool = True,
                 drop_last: bool = False, seed: int = 0) -> None:
        if users.shape != items.shape or users.dim() != 1:
            raise ValueError("ttamm: users and items must be 1-D tensors of one length")
        if users.dtype != torch.long or items.dtype != torch.long:
            raise ValueError("ttamm: interaction ids must be int64 (torch.long)")
        _lib.require_rocm(users, "interaction users")
        _lib.require_rocm(items, "interaction items")
        if batch_size <= 0:
            raise ValueError("batch_size should be a positive integer value")
        self.users, self.items = users.contiguous(), items.contiguous()
        self.batch_size = int(batch_size)
        self.shuffle, self.drop_last = bool(shuffle), bool(drop_last)
        self.seed = int(seed) & ((1 << 64) - 1)
        self.epoch = 0
        self.lib = _lib.load()

    def __len__(self) -> int:
        n = self.users.numel()
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size

    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)

    def batch(self, index: int, epoch: int | None = None) -> tuple[torch.Tensor, torch.Tensor]:
        """Batch ``index`` of ``epoch`` (default: the current one)."""
        n = self.users.numel()
        if not 0 <= index < len(self):
            raise IndexError("ttamm: batch index out of range")
        start = index * self.batch_size
        count = min(self.batch_size, n - start)
        out_u = torch.empty(count, dtype=torch.long, device=self.users.device)
        out_i = torch.empty(count, dtype=torch.long, device=self.users.device)
        _lib.check(self.lib.ttamm_epoch_batch(
            ctypes.c_void_p(self.users.data_ptr()), ctypes.c_void_p(self.items.data_ptr()), n,
            ctypes.c_uint64(self.seed), self.epoch if epoch is None else int(epoch), int(self.shuffle), start, count,
            ctypes.c_void_p(out_u.data_ptr()), ctypes.c_void_p(out_i.data_ptr()),
            _lib.stream_handle(self.users.device)))
        return out_u, out_i

    def __iter__(self):
        epoch = self.epoch
        for b in range(len(self)):
            yield self.batch(b, epoch)
        self.epoch = epoch + 1
