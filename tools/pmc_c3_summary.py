#!/usr/bin/env python3
"""HBM bytes per launch of the C3 retrieval scan kernel from two rocprofv3 PMC passes
(FETCH_SIZE, WRITE_SIZE; tools/gpu/pmc_c3.sh) into profiles/pmc_traffic.json "c3".

    python3 tools/pmc_c3_summary.py <tag> [gpurun_out]
"""

from __future__ import annotations

import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))
from pmc_summary import per_kernel  # noqa: E402


def main() -> None:
    tag = sys.argv[1]
    src = Path(sys.argv[2]) if len(sys.argv) > 2 else ROOT / "gpurun_out"
    fetch = per_kernel(src / "pmc_c3_fetch.csv", "FETCH_SIZE")
    write = per_kernel(src / "pmc_c3_write.csv", "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, [0.0]), write.get(k, [0.0])
        kernels[k] = {"launches": len(f), "hbm_bytes_per_launch": round(sum(f) / len(f) * 1024 * 2 + sum(w) / len(w) * 1024)}
    scan = [k for k in kernels if k.startswith("retrieval_x_kernel") or k.startswith("retrieval_partial_kernel")]
    entry = {"tag": tag, "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, one pass each, "
             "tools/bench_retrieval.py --reps 2 --cpu-queries 0 (C3: 65,536 queries x 2M items x 96, K = 80, "
             "20 blocked per query); bytes = FETCH_SIZE*1024*2 + WRITE_SIZE*1024 (MI355X_MICROARCH.md HBM)",
             "kernels": kernels}
    if scan:
        k = max(scan, key=lambda n: kernels[n]["hbm_bytes_per_launch"])
        entry["retrieval_kernel"] = k
        entry["retrieval_bytes_per_launch"] = kernels[k]["hbm_bytes_per_launch"]
    path = ROOT / "profiles" / "pmc_traffic.json"
    allp = json.loads(path.read_text()) if path.exists() else {}
    allp["c3"] = entry
    path.write_text(json.dumps(allp, indent=1) + "\n")
    print(json.dumps({k: v for k, v in entry.items() if k != "kernels"}, indent=1))


if __name__ == "__main__":
    main()
