"""The sharded step's exchange layer on CPU: row ownership, request routing and the three
all-to-alls + all-reduce of ttamm/sharded.py, served by torch.distributed (gloo, world_size 2,
two processes) and by the in-process loopback — both must route every row to the right place
in the right order, including a rank that receives no requests.  The owner grouping itself is
ttamm_route_rows on the GPU (tests/test_route_gpu.py); here its CPU restatement
(oracle/route.py) stands in for it."""

from __future__ import annotations

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle.route import route_rows  # the CPU router (ttamm_route_rows runs on the GPU)
from ttamm.sharded import (AllGather, AllReduce, AllToAll, ReduceScatter, RowOwnership, TorchComm, Wait, route_pairs,
                           route_requests, run_loopback)


def test_row_ownership():
    for W in (1, 2, 3, 8):
        total = 0
        for r in range(W):
            own = RowOwnership(W, r)
            n = own.local_count(29)
            total += n
            ids = own.global_ids(torch.arange(n))
            assert torch.equal(own.owner(ids), torch.full_like(ids, r))
            assert torch.equal(own.local(ids), torch.arange(n))
            full = torch.arange(29 * 2).view(29, 2)
            assert torch.equal(own.shard(full)[:, 0] // 2, ids)
        assert total == 29
    with pytest.raises(ValueError):
        RowOwnership(2, 2)


def _requests(W: int, rank: int, case: str):
    g = torch.Generator().manual_seed(100 + rank)
    B, N = 5, 3
    R = B * (1 + N)
    if case == "skewed":  # every item owned by rank 0: the other ranks receive nothing
        items = torch.randint(0, 40, (R,), generator=g) * W
    else:
        items = torch.randint(0, 97, (R,), generator=g)
    Bg = W * B
    keys = torch.cat([torch.arange(B) + rank * B, torch.arange(B * N) + Bg + rank * B * N])
    return items, keys


def _exchange_program(W: int, rank: int, case: str):
    own = RowOwnership(W, rank)
    items, keys = _requests(W, rank, case)
    B, N = 5, 3
    route = yield from route_requests(own, route_rows, items[:B], items[B:], rank * B, W * B + rank * B * N)
    assert torch.equal(route.slot.sort().values, torch.arange(items.numel()))
    assert torch.equal(own.owner(own.global_ids(route.rows)), torch.full_like(route.rows, rank))
    # owner: payload rows (global id, request key, 7) for what it was asked
    payload = torch.stack([own.global_ids(route.rows).double(), route.keys.double(),
                           torch.full((route.rows.numel(),), 7.0, dtype=torch.float64)], dim=1)
    h = yield AllToAll(payload, route.recv_counts, route.send_counts, async_op=True)
    back = yield Wait(h)
    fwd = back[route.slot]  # request j's row sits at slot[j] of the owner-grouped buffer
    # requester: gradient rows keyed by its request positions, written at their slots
    grads = torch.stack([keys.double() * 3.0, items.double()], dim=1)
    grouped = torch.empty_like(grads)
    grouped[route.slot] = grads
    to_owner = yield AllToAll(grouped, route.send_counts, route.recv_counts)
    acc = torch.tensor([float(rank + 1), 2.0 ** -rank])
    yield AllReduce(acc)
    # in-batch negatives: all-gather [2, 3] rows, reduce-scatter [2W, 3] rows
    gathered = yield AllGather(torch.full((2, 3), float(rank)))
    scattered = yield ReduceScatter(torch.arange(2 * W * 3, dtype=torch.float64).reshape(2 * W, 3) * (rank + 1))
    return {"items": items, "keys": keys, "fwd": fwd, "route_rows": route.rows, "route_keys": route.keys,
            "to_owner": to_owner, "acc": acc, "recv": route.recv_counts, "gathered": gathered,
            "scattered": scattered}


def _check(W: int, outs: list[dict], case: str):
    for rank, o in enumerate(outs):
        # rows come back to the requester in request order
        assert torch.equal(o["fwd"][:, 0], o["items"].double())
        assert torch.equal(o["fwd"][:, 1], o["keys"].double())
        # each owner got, for every row it computed, the gradient of that very request
        assert torch.equal(o["to_owner"][:, 0], o["route_keys"].double() * 3.0)
        own = RowOwnership(W, rank)
        assert torch.equal(o["to_owner"][:, 1], own.global_ids(o["route_rows"]).double())
        assert torch.equal(o["acc"], torch.tensor([sum(range(1, W + 1)), sum(2.0 ** -r for r in range(W))],
                                                  dtype=o["acc"].dtype))
        if case == "skewed" and rank > 0:
            assert o["route_rows"].numel() == 0
        assert torch.equal(o["gathered"], torch.arange(W).repeat_interleave(2).double()[:, None].expand(2 * W, 3)
                           .to(o["gathered"].dtype))
        full = torch.arange(2 * W * 3, dtype=torch.float64).reshape(2 * W, 3) * (W * (W + 1) / 2)
        assert torch.equal(o["scattered"], full[2 * rank:2 * rank + 2])
    total = sum(o["route_rows"].numel() for o in outs)
    assert total == sum(o["items"].numel() for o in outs)


@pytest.mark.parametrize("W", [1, 2, 3])
@pytest.mark.parametrize("case", ["uniform", "skewed"])
def test_exchange_loopback(W, case):
    outs = run_loopback([_exchange_program(W, r, case) for r in range(W)])
    _check(W, outs, case)


def _worker(rank: int, world: int, port: int, case: str, q) -> None:
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = TorchComm().run(_exchange_program(world, rank, case))
        q.put((rank, {k: (v.tolist() if torch.is_tensor(v) else v) for k, v in out.items()},
               {k: str(v.dtype) for k, v in out.items() if torch.is_tensor(v)}))
    finally:
        dist.destroy_process_group()


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("case", ["uniform", "skewed"])
def test_exchange_gloo_world2(case):
    W = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, W, port, case, q)) for r in range(W)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(W):
        rank, out, dtypes = q.get(timeout=120)
        got[rank] = {k: (torch.tensor(v, dtype=getattr(torch, dtypes[k].split(".")[1])) if k in dtypes else v)
                     for k, v in out.items()}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    outs = [got[r] for r in range(W)]
    for o in outs:  # empty tensors lose their trailing shape in the round trip through lists
        for k in ("fwd", "to_owner", "gathered", "scattered"):
            o[k] = o[k].reshape(-1, 2 if k == "to_owner" else 3)
    _check(W, outs, case)
    # identical to the loopback schedule
    ref = run_loopback([_exchange_program(W, r, case) for r in range(W)])
    for a, b in zip(outs, ref):
        assert torch.equal(a["fwd"], b["fwd"]) and torch.equal(a["to_owner"], b["to_owner"])


@pytest.mark.parametrize("W", [1, 2, 3])
def test_route_pairs_to_user_owners(W):
    """The sharded epoch's pair routing: rank r ends up with exactly the pairs whose user it
    owns, source rank by source rank, each source's pairs in their original order."""
    streams = []
    for r in range(W):
        g = torch.Generator().manual_seed(40 + r)
        u = torch.randint(0, 50, (17,), generator=g)
        streams.append((u, u * 100 + torch.arange(17) + 10000 * r))

    def prog(r):
        got = yield from route_pairs(RowOwnership(W, r), route_rows, *streams[r])
        return got

    outs = run_loopback([prog(r) for r in range(W)])
    for r, (u, i, sizes) in enumerate(outs):
        want_u = torch.cat([su[su % W == r] for su, _ in streams])
        want_i = torch.cat([si[su % W == r] for su, si in streams])
        assert torch.equal(u, want_u // W) and torch.equal(i, want_i)  # local user rows
        assert sizes == [sum(int((su % W == d).sum()) for su, _ in streams) for d in range(W)]


def test_route_oracle_compact_units_tile_the_exchange_buffer():
    """oracle/route.py with [world, 3] count rows (the compact exchange layout, ttamm.h
    exchange_counts): the units of a rank's requests tile [0, requests + positives) exactly, each
    owner's group starting where the previous one ends, positives two units apart."""
    g = torch.Generator().manual_seed(3)
    for world in (1, 3, 8):
        ids = torch.randint(0, 10 ** 6, (600,), generator=g)
        counts = torch.zeros((world, 3), dtype=torch.long)
        _, units, _ = route_rows(world, ids[:100], ids[100:], None, 0, 0, counts_out=counts)
        width = torch.ones(600, dtype=torch.long)
        width[:100] = 2
        cover = torch.zeros(600 + 100, dtype=torch.long)
        for u, w in zip(units.tolist(), width.tolist()):
            cover[u:u + w] += 1
        assert torch.equal(cover, torch.ones_like(cover))
        assert counts[:, 2].sum() == 100 and counts[:, 0].sum() == 600
