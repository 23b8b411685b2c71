#!/usr/bin/env python3
"""bench.py's 50M x 128 bulk gather sub-line alone (bench.gather_bulk), for rocprofv3 passes:
    rocprofv3 --kernel-trace --stats -- python3 tools/gather_bulk.py
    rocprofv3 --pmc FETCH_SIZE -- python3 tools/gather_bulk.py      (then WRITE_SIZE)
Prints the sub-line's JSON."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "two-tower-augmented-with-adaptive-mimic-mechanism_amd")]

import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    print(json.dumps(bench.gather_bulk(torch.device("cuda", 0), reps=int(sys.argv[1]) if len(sys.argv) > 1 else 10)))
