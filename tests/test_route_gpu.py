"""ttamm_route_rows (csrc/route.hip) against its CPU restatement (oracle/route.py): the owner
grouping of the sharded step is a stable sort by id % world, so parity is bit-exact — slots,
(local row, key / payload) rows and counts — over block-boundary sizes, skewed and uniform
owners, world sizes up to the kernel's 1024, and both key and payload modes."""

from __future__ import annotations

import pytest
import torch

from oracle.route import route_rows
from ttamm import _lib
from ttamm.sharded import device_route

pytestmark = pytest.mark.gpu


def _check(world, id0, id1=None, payload=None, key0=0, key1=0):
    lib = _lib.load()
    got = device_route(lib, world, id0, id1, payload, key0, key1)
    torch.cuda.synchronize()
    want = route_rows(world, id0.cpu(), None if id1 is None else id1.cpu(),
                      None if payload is None else payload.cpu(), key0, key1)
    for g, w, name in zip(got, want, ("packed", "slot", "counts")):
        assert torch.equal(g.cpu(), w.cpu()), name


@pytest.mark.parametrize("world", [1, 2, 3, 8, 64, 1024])
@pytest.mark.parametrize("n", [1, 63, 2047, 2048, 2049, 49152])
def test_route_requests_matches_stable_sort(world, n):
    g = torch.Generator().manual_seed(world * 7919 + n)
    ids = torch.randint(0, 1 << 40, (n,), generator=g).cuda()
    n0 = n // 6
    _check(world, ids[:n0], ids[n0:], None, 12345, 10 ** 9 + 7)


@pytest.mark.parametrize("world", [2, 8])
def test_route_skewed_owners(world):
    """Every id owned by one rank (the others receive nothing), and a two-owner mix."""
    g = torch.Generator().manual_seed(5)
    ids = (torch.randint(0, 1000, (9000,), generator=g) * world + (world - 1)).cuda()
    _check(world, ids, None, None, 0, 0)
    mix = torch.where(torch.rand(9000, generator=g).cuda() < 0.9, ids, ids - (world - 1))
    _check(world, mix[:100], mix[100:], None, 3, 4)


@pytest.mark.parametrize("world", [1, 4, 8])
def test_route_pairs_payload(world):
    g = torch.Generator().manual_seed(11)
    users = torch.randint(0, 50000, (20000,), generator=g).cuda()
    items = torch.randint(0, 1 << 50, (20000,), generator=g).cuda()
    _check(world, users, None, items)


def test_route_large_batch():
    """The C4-sized request set of a sharded step (B 65536, 1 + 5 rows each) over 8 owners."""
    g = torch.Generator().manual_seed(2)
    ids = torch.randint(0, 10 ** 6, (65536 * 6,), generator=g).cuda()
    _check(8, ids[:65536], ids[65536:], None, 65536 * 3, 8 * 65536 + 65536 * 3 * 5)


def test_route_empty_and_bad_world():
    lib = _lib.load()
    e = torch.empty(0, dtype=torch.long, device="cuda")
    packed, slot, counts = device_route(lib, 4, e, e)
    assert packed.numel() == 0 and slot.numel() == 0 and counts.cpu().tolist() == [0, 0, 0, 0]
    with pytest.raises(ValueError):
        device_route(lib, 0, torch.ones(3, dtype=torch.long, device="cuda"))
    with pytest.raises(ValueError):
        device_route(lib, 1025, torch.ones(3, dtype=torch.long, device="cuda"))


@pytest.mark.parametrize("world", [1, 3, 8, 1024])
@pytest.mark.parametrize("n", [0, 2049, 49152])
def test_route_positive_counts_column(world, n):
    """counts_ld >= 3 (the compact exchange's count rows): column 2 = how many of each owner's
    ids came from id0 (the positives), beside the counts and the status word, and slot = each
    request's first unit of the compact exchange layout (oracle/route.py)."""
    lib = _lib.load()
    g = torch.Generator().manual_seed(world + n)
    ids = torch.randint(0, 1 << 40, (n,), generator=g).cuda()
    n0 = n // 6
    counts = torch.full((world, 3), -1, dtype=torch.long, device="cuda")
    status = torch.tensor([5], dtype=torch.int32, device="cuda")
    packed, slot, _ = device_route(lib, world, ids[:n0], ids[n0:], None, 7, 9, counts_out=counts, status=status)
    torch.cuda.synchronize()
    wc = torch.zeros((world, 3), dtype=torch.long)
    want = route_rows(world, ids[:n0].cpu(), ids[n0:].cpu(), None, 7, 9, counts_out=wc,
                      status=torch.tensor([5], dtype=torch.int32))
    assert torch.equal(packed.cpu(), want[0].cpu()) and torch.equal(slot.cpu(), want[1].cpu())
    c = counts.cpu()
    assert torch.equal(c, wc)
    assert torch.equal(c[:, 0], torch.bincount(ids.cpu() % world, minlength=world))
    assert c[:, 1].tolist() == [5] * world
    assert torch.equal(c[:, 2], torch.bincount(ids[:n0].cpu() % world, minlength=world))
