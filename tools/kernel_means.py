#!/usr/bin/env python3
"""Mean duration per kernel name over a rocprofv3 kernel trace (all dispatches), optionally
side by side with a second trace:  python3 tools/kernel_means.py new.csv [old.csv]"""
import csv
import sys
from collections import defaultdict


def means(path):
    acc = defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"].replace("ttamm::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        a = acc[n]
        a[0] += 1
        a[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    return {k: (c, t / c) for k, (c, t) in acc.items()}


new = means(sys.argv[1])
old = means(sys.argv[2]) if len(sys.argv) > 2 else {}
for k, (c, m) in sorted(new.items(), key=lambda kv: -kv[1][0] * kv[1][1]):
    o = old.get(k)
    print(f"{k[:72]:72s} n {c:5d} mean {m:8.1f} us" + (f"   old {o[1]:8.1f} us  ({m - o[1]:+.1f})" if o else ""))
