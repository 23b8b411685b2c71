"""Row grouping (ttamm_coalesce_rows): the coalescing every row-table update of the step runs —
unique rows in first-occurrence (or ascending) order, each row's batch positions ascending, as
torch's grad.coalesce() / index_add order them (_functional.py:44, training.py:822).  Index
work, so bit-exact against a numpy restatement (a stable argsort), including Zipf-hot rows far
longer than a register sort (the LDS bitmap ranking) and a hot row spanning more positions than
the bitmap holds (the counting fallback)."""

from __future__ import annotations

import numpy as np
import pytest
import torch

from ttamm import _lib as L

pytestmark = pytest.mark.gpu


def _expected(idx: np.ndarray, sorted_keys: bool):
    order = np.argsort(idx, kind="stable")  # positions ascending within each row
    keys = idx[order]
    uniq, start = np.unique(keys, return_index=True)
    bounds = list(start) + [len(idx)]
    segs = [(int(uniq[u]), order[bounds[u]:bounds[u + 1]]) for u in range(len(uniq))]
    if not sorted_keys:
        segs.sort(key=lambda kv: kv[1][0])  # by first occurrence
    k = np.concatenate([np.full(len(p), r, dtype=np.int32) for r, p in segs])
    p = np.concatenate([p for _, p in segs]).astype(np.int32)
    ss = np.cumsum([0] + [len(p) for _, p in segs]).astype(np.int32)
    return k, p, ss, len(segs)


def _run(idx: torch.Tensor, rows: int, sorted_keys: bool, ws: torch.Tensor | None = None):
    lib = L.load()
    n = idx.numel()
    need = int(lib.ttamm_coalesce_workspace_bytes(n, rows))
    if ws is None or ws.numel() < need:
        ws = torch.zeros(need, dtype=torch.uint8, device="cuda")
    keys = torch.empty(n, dtype=torch.int32, device="cuda")
    pos = torch.empty(n, dtype=torch.int32, device="cuda")
    ss = torch.empty(n + 1, dtype=torch.int32, device="cuda")
    nu = torch.empty(1, dtype=torch.int32, device="cuda")
    d = idx.cuda()
    L.check(lib.ttamm_coalesce_rows(d.data_ptr(), n, rows, int(sorted_keys), keys.data_ptr(), pos.data_ptr(),
                                    ss.data_ptr(), nu.data_ptr(), ws.data_ptr(), ws.numel(), L.stream_handle()))
    torch.cuda.synchronize()
    u = int(nu.item())
    return keys.cpu().numpy(), pos.cpu().numpy(), ss[: u + 1].cpu().numpy(), u, ws


def _zipf(n: int, rows: int, s: float, seed: int) -> torch.Tensor:
    g = np.random.default_rng(seed)
    r = np.minimum(g.zipf(s, n) - 1, rows - 1)
    perm = g.permutation(rows)
    return torch.from_numpy(perm[r].astype(np.int64))


CASES = [
    ("uniform", lambda: torch.randint(0, 2_000_000, (49_152,), generator=torch.Generator().manual_seed(1)), 2_000_000),
    ("zipf-c2-items", lambda: _zipf(49_152, 2_000_000, 1.3, 2), 2_000_000),
    ("zipf-very-hot", lambda: _zipf(60_000, 50_000, 1.05, 3), 50_000),
    ("one-row", lambda: torch.full((300_000,), 7, dtype=torch.long), 100),  # range > the LDS bitmap
    ("small", lambda: torch.tensor([3, 1, 3, 3, 0, 1], dtype=torch.long), 4),
]


@pytest.mark.parametrize("name,make,rows", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("sorted_keys", [False, True], ids=["first-occurrence", "ascending"])
def test_coalesce_rows_bit_exact(name, make, rows, sorted_keys):
    if sorted_keys and rows > 65536:
        pytest.skip("ascending grouping covers <= 65536 keys")
    idx = make()
    k, p, ss, u, ws = _run(idx, rows, sorted_keys)
    ek, ep, ess, eu = _expected(idx.numpy(), sorted_keys)
    assert u == eu
    assert np.array_equal(ss, ess)
    assert np.array_equal(k, ek)
    assert np.array_equal(p, ep)
    # the per-row scratch is zero again: a second call on the same workspace agrees
    k2, p2, ss2, u2, _ = _run(idx, rows, sorted_keys, ws)
    assert u2 == u and np.array_equal(p2, p) and np.array_equal(k2, k)
