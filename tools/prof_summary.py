#!/usr/bin/env python3
"""Summarise rocprofv3 output directories into small files (run on the GPU box, so only the
summaries travel back), then drop the per-dispatch CSVs.

    python3 tools/prof_summary.py stats  <dir>                 # keeps run_kernel_stats.csv
    python3 tools/prof_summary.py pmc    <dir> <COUNTER> <out.json>

pmc: mean value of COUNTER per dispatch for every kernel (rocprofv3 reports FETCH_SIZE /
WRITE_SIZE in KiB; MI355X_MICROARCH.md: on gfx950 FETCH_SIZE is half the bytes of a wide
coalesced streaming read — the doubling is applied by the consumer, bench.load_traffic)."""

from __future__ import annotations

import csv
import json
import sys
from collections import defaultdict
from pathlib import Path


def _drop(d: Path, keep: set[str]) -> None:
    for f in d.iterdir():
        if f.is_file() and f.name not in keep:
            f.unlink()


def stats(d: Path) -> None:
    _drop(d, {"run_kernel_stats.csv", "run_domain_stats.csv", "run_agent_info.csv"})


def pmc(d: Path, counter: str, out: Path) -> None:
    per_kernel: dict[str, list[float]] = defaultdict(list)
    with open(d / "run_counter_collection.csv", newline="") as fh:
        for row in csv.DictReader(fh):
            if row.get("Counter_Name") != counter:
                continue
            per_kernel[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    summary = {k: {"dispatches": len(v), "mean": sum(v) / len(v), "min": min(v), "max": max(v)}
               for k, v in per_kernel.items()}
    out.write_text(json.dumps({"counter": counter, "unit": "KiB", "kernels": summary}, indent=1))
    _drop(d, {"run_agent_info.csv"})


if __name__ == "__main__":
    mode, path = sys.argv[1], Path(sys.argv[2])
    if mode == "stats":
        stats(path)
    else:
        pmc(path, sys.argv[3], Path(sys.argv[4]))
