"""CPU restatement of ttamm's on-device epoch order (csrc/data.hip, ttamm.h ttamm_epoch_batch).

TEST INFRASTRUCTURE ONLY: tests/ use it as the checker of the HIP kernel; the product never
imports it.

The reference shuffles with torch.utils.data.DataLoader(shuffle=True) (training.py:260-264), i.e.
torch.randperm on the host RNG; that stream cannot be reproduced on the device, so ttamm defines
its own seeded bijection and this module is its specification:

    keys[q] = low32(splitmix64(seed ^ splitmix64(4 * epoch + q)))      q = 0..3
    h       = smallest h >= 1 with 4^h >= n
    F(x)    = 4 Feistel rounds on (l, r) = (x >> h, x & (2^h - 1)):
              (l, r) <- (r, l ^ (fmix32(low32(r) ^ keys[q]) & (2^h - 1)))
    perm(p) = F(p), then F again while the value is >= n (cycle-walking)

Parity is bit-exact (integer arithmetic).  The loader semantics (batches in order, the last one
short, drop_last=False) follow torch's DataLoader over InteractionDataset (datasets.py:12-45)."""

from __future__ import annotations

import numpy as np

M64 = (1 << 64) - 1
M32 = (1 << 32) - 1


def splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & M64
    z = x
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def round_keys(seed: int, epoch: int) -> list[int]:
    return [splitmix64((seed ^ splitmix64((epoch * 4 + q) & M64)) & M64) & M32 for q in range(4)]


def half_bits(n: int) -> int:
    h = 1
    while h < 32 and n > (1 << (2 * h)):
        h += 1
    return h


def _fmix32(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64)
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x85EBCA6B)) & np.uint64(M32)
    x ^= x >> np.uint64(13)
    x = (x * np.uint64(0xC2B2AE35)) & np.uint64(M32)
    x ^= x >> np.uint64(16)
    return x


def _feistel(x: np.ndarray, h: int, keys: list[int]) -> np.ndarray:
    mask = np.uint64((1 << h) - 1)
    sh = np.uint64(h)
    left, right = x >> sh, x & mask
    for k in keys:
        f = _fmix32((right & np.uint64(M32)) ^ np.uint64(k)) & mask
        left, right = right, left ^ f
    return (left << sh) | right


def epoch_order(n: int, seed: int, epoch: int, shuffle: bool = True) -> np.ndarray:
    """Source index of every position 0..n-1 in epoch `epoch` (int64)."""
    pos = np.arange(n, dtype=np.uint64)
    if not shuffle or n == 0:
        return pos.astype(np.int64)
    h, keys = half_bits(n), round_keys(seed, epoch)
    y = _feistel(pos, h, keys)
    out = y.copy()
    todo = out >= np.uint64(n)
    while todo.any():
        out[todo] = _feistel(out[todo], h, keys)
        todo = out >= np.uint64(n)
    return out.astype(np.int64)


def epoch_batches(users: np.ndarray, items: np.ndarray, batch_size: int, seed: int, epoch: int,
                  shuffle: bool = True) -> list[tuple[np.ndarray, np.ndarray]]:
    """The loader's batches of one epoch: DataLoader(..., batch_size, drop_last=False) order."""
    order = epoch_order(len(users), seed, epoch, shuffle)
    return [(users[order[i:i + batch_size]], items[order[i:i + batch_size]])
            for i in range(0, len(order), batch_size)]
