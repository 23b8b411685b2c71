#!/usr/bin/env python3
"""Per-step timeline of a rocprofv3 kernel trace of bench.py: for the last timed step, every
dispatch with its stream, start offset and duration, plus the step's busy / idle time.
    python3 tools/trace_timeline.py gpurun_out/trace_c2_kernels.csv [marker_kernel]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
marker = sys.argv[2] if len(sys.argv) > 2 else None
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
rows.sort(key=lambda r: r["s"])
if marker is None:  # the step's first kernel: the fused prologue (round 3) or the sampler before it
    marker = next((m for m in ("step_prologue_kernel", "sample_negatives_kernel")
                   if any(m in r["Kernel_Name"] for r in rows)), "step_prologue_kernel")
starts = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
if len(starts) < 3:
    sys.exit(f"marker {marker} found {len(starts)} times")
i0, i1 = starts[-3], starts[-2]  # a full step in the timed region
step = rows[i0:i1]
t0 = step[0]["s"]
t1 = rows[i1]["s"]
print(f"step span {(t1 - t0) / 1e3:.1f} us, {len(step)} dispatches")
busy = 0
cur_s = cur_e = None
for r in step:
    if cur_e is None or r["s"] > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = r["s"], r["e"]
    else:
        cur_e = max(cur_e, r["e"])
busy += cur_e - cur_s
print(f"GPU busy (union) {busy / 1e3:.1f} us, idle {(t1 - t0 - busy) / 1e3:.1f} us")
agg = defaultdict(float)
for r in step:
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").replace("ttamm::", "").split("(")[0][:70]
    print(f"  q{r['Queue_Id']:>2} +{(r['s'] - t0) / 1e3:8.1f} {(r['e'] - r['s']) / 1e3:8.1f} us  {name}  grid={r['Grid_Size_X']}")
    agg[name] += (r["e"] - r["s"]) / 1e3
print("by kernel (sum of durations, us):")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1]):
    print(f"  {v:8.1f}  {k}")
