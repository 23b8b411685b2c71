#!/usr/bin/env python3
"""Per-kernel means of every counter in rocprofv3 --pmc counter_collection.csv files.

    python3 tools/pmc_kernel.py <csv> [<csv> ...] [--match SUBSTRING]

Prints one JSON object: {kernel: {counter: mean per launch, "launches": n}} (counters summed over
the dimensions of one dispatch first)."""

from __future__ import annotations

import csv
import json
import sys
from collections import defaultdict


def main() -> None:
    args = sys.argv[1:]
    match = None
    if "--match" in args:
        i = args.index("--match")
        match = args[i + 1]
        args = args[:i] + args[i + 2:]
    per: dict[tuple[str, str], float] = defaultdict(float)
    for path in args:
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].replace("ttamm::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            if match and match not in k:
                continue
            per[(k, r["Counter_Name"], path, r["Dispatch_Id"])] += float(r["Counter_Value"])
    out: dict[str, dict] = defaultdict(lambda: defaultdict(list))
    for (k, c, _, _), v in per.items():
        out[k][c].append(v)
    res = {}
    for k, cs in out.items():
        res[k] = {c: sum(v) / len(v) for c, v in cs.items()}
        res[k]["launches"] = max(len(v) for v in cs.values())
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
