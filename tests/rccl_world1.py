"""Rank program for tests/test_rccl_gpu.py: TorchComm's RCCL branch (backend "nccl") on one GPU.

Every collective request type the row-sharded step issues (AllToAll, async AllToAll + Wait,
AllGather, ReduceScatter, AllReduce) goes through torch.distributed with a world-1 RCCL group on
device tensors, the step's real call pattern (receive buffers given, async work waited), and the
results are checked against what a world-1 collective must return.  Prints "rccl ok" on success."""

from __future__ import annotations

import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "two-tower-augmented-with-adaptive-mimic-mechanism_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from ttamm.sharded import AllGather, AllReduce, AllToAll, ReduceScatter, TorchComm, Wait  # noqa: E402


def main() -> None:
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    comm = TorchComm()
    assert not comm.staged and dist.get_backend() == "nccl"
    dev = torch.device("cuda", local)
    g = torch.Generator(device=dev).manual_seed(1)
    rows = torch.randn((37, 192), device=dev, generator=g)
    # (t | a) rows into a caller-given receive buffer, synchronous and async + Wait
    out = torch.empty_like(rows)
    got = comm(AllToAll(rows, [37], [37], out=out))
    assert got.data_ptr() == out.data_ptr() and torch.equal(got, rows)
    out2 = torch.empty_like(rows)
    h = comm(AllToAll(rows * 2, [37], [37], async_op=True, out=out2))
    got2 = comm(Wait(h))
    torch.cuda.current_stream().synchronize()
    assert torch.equal(got2, rows * 2)
    # int64 (local row, key) pairs, new receive tensor
    pairs = torch.arange(20, device=dev, dtype=torch.long).view(10, 2)
    assert torch.equal(comm(AllToAll(pairs, [10], [10])), pairs)
    # all-gather of in-batch positives, reduce-scatter of dP, all-reduce of the gradient arena
    assert torch.equal(comm(AllGather(rows[:8])), rows[:8])
    assert torch.equal(comm(ReduceScatter(rows[:16])), rows[:16])
    arena = rows.reshape(-1).clone()
    assert torch.equal(comm(AllReduce(arena)), rows.reshape(-1))
    # status flags as the finish program all-reduces them
    flags = torch.tensor([0.0, 1.0, 0.0], device=dev)
    assert comm(AllReduce(flags)).tolist() == [0.0, 1.0, 0.0]
    torch.cuda.synchronize()
    dist.destroy_process_group()
    print("rccl ok", flush=True)


if __name__ == "__main__":
    main()
