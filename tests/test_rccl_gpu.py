"""TorchComm's RCCL branch on real hardware (one GPU: RCCL allows one rank per GPU, so the
multi-rank parity tests use gloo or the in-process loopback; this runs every request type the
row-sharded step issues through a world-1 "nccl" group, so the RCCL calls themselves — buffer
arguments, async work, dtypes — have executed before the driver's 8-GPU run)."""

from __future__ import annotations

import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu


def test_torchcomm_rccl_world_one():
    root = Path(__file__).resolve().parents[1]
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={port}", str(root / "tests" / "rccl_world1.py")]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=root, env=env)
    assert res.returncode == 0, res.stderr[-3000:]
    assert "rccl ok" in res.stdout
