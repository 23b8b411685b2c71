"""bench.py's launcher logic on CPU (no GPU call): `--gpus N` without WORLD_SIZE starts N ranks
through torch.distributed.run on 127.0.0.1 and forwards the arguments unchanged."""

import importlib.util
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_launch_command_starts_n_ranks_on_loopback():
    b = _bench()
    argv = ["--gpus", "8", "--steps", "20", "--warmup", "3"]
    cmd = b.launch_command(argv, 8, 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    assert cmd[-len(argv) - 1].endswith("bench.py") and cmd[-len(argv):] == argv


def test_free_port_is_bindable():
    import socket

    port = _bench().free_port()
    with socket.socket() as s:
        s.bind(("127.0.0.1", port))
