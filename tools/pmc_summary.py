#!/usr/bin/env python3
"""Summarise the rocprofv3 passes of tools/gpu/pmc_passes.sh into profiles/pmc_traffic.json.

    python3 tools/pmc_summary.py <config> <tag> [gpurun_out]

Per kernel (mean over its launches in the 40-step run): HBM bytes = FETCH_SIZE * 1024 * 2
(gfx950 reports half of a wide streaming read, MI355X_MICROARCH.md "HBM") + WRITE_SIZE * 1024,
each from its own pass.  The deferred table AdamW gets a VALU roofline: SQ_INSTS_VALU summed over
every replay_kernel launch of the run, per element-step replayed, against the chip's VALU issue
rate, timed by the kernel-trace --stats run of the bench command."""

from __future__ import annotations

import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

VALU_ISSUE_PER_S = 1024 * 2.4e9 / 2  # 256 CUs x 4 SIMD-32s, one wave64 VALU instruction per 2 cycles
# (MI355X_MICROARCH.md "Wave scheduling" and the v_fma_f32 row: 2 cycles per SIMD-32; one wave alone
# issues at half that, and v_sqrt / v_rcp cost more, so the replay cannot reach this upper bound)
SIMD_CYCLES_PER_S = 1024 * 2.4e9
# measured sustained issue costs with 8 waves per SIMD (csrc/tools/valu_bench.cpp,
# profiles/r03_valu_issue_rates.txt), SIMD cycles at 2.4 GHz per wave64 instruction
COST_TRANS = 8.43  # v_sqrt_f32 8.46, v_rcp_f32 8.39
COST_OTHER = 4.08  # v_fma_f32 (the cheapest measured; v_pk_mul_f32 4.78, v_pk_fma_f32 5.21)


def short(name: str) -> str:
    return name.replace("ttamm::(anonymous namespace)::", "").replace("void ", "").split("(")[0]


def per_kernel(path: Path, counter: str) -> dict[str, list[float]]:
    vals: dict[tuple[str, str], float] = defaultdict(float)
    for r in csv.DictReader(path.open()):
        if r["Counter_Name"] == counter:
            vals[(r["Dispatch_Id"], r["Kernel_Name"])] += float(r["Counter_Value"])
    out: dict[str, list[float]] = defaultdict(list)
    for (_, k), v in vals.items():
        out[short(k)].append(v)
    return out


def main() -> None:
    config, tag = sys.argv[1], sys.argv[2]
    src = Path(sys.argv[3]) if len(sys.argv) > 3 else ROOT / "gpurun_out"
    fetch = per_kernel(src / "pmc_fetch.csv", "FETCH_SIZE")
    write = per_kernel(src / "pmc_write.csv", "WRITE_SIZE")
    valu = per_kernel(src / "pmc_valu.csv", "SQ_INSTS_VALU")
    trans = per_kernel(src / "pmc_valu.csv", "SQ_INSTS_VALU_TRANS_F32")
    stats = {short(r["Name"]): r for r in csv.DictReader((src / "stats_kernel_stats.csv").open())}
    bench = json.loads((src / "stats_bench.json").read_text())

    import bench as B  # the config's shapes

    c = B.CONFIGS[config.split("_")[0]]  # "c2_inbatch": c2's shapes (bench.py --negatives in-batch)
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [0.0])
        w = write.get(k, [0.0])
        kernels[k] = {
            "launches": len(f),
            "hbm_bytes_per_launch": round(sum(f) / len(f) * 1024 * 2 + sum(w) / len(w) * 1024),
            "fetch_bytes_per_launch": round(sum(f) / len(f) * 1024 * 2),
            "write_bytes_per_launch": round(sum(w) / len(w) * 1024),
        }
    entry = {"tag": tag, "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE / --pmc SQ_INSTS_VALU "
             "SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_WAVES SQ_INSTS_SALU, one pass "
             "each, bench.py --steps 40 --warmup 3; bytes = FETCH_SIZE*1024*2 + "
             "WRITE_SIZE*1024 (MI355X_MICROARCH.md HBM); kernel times from rocprofv3 --kernel-trace --stats of "
             "the default bench command", "kernels": kernels}

    # the roofline kernel of bench.py: the grouped first feature-layer forward (EPI_HIDDEN = 1)
    l1 = [k for k in kernels if ("gemm_x_kernel" in k or "gemm_bf16_kernel" in k or "gemm_kernel" in k)
          and (k.endswith(", 1, 3>") or k.endswith(", 1, 1>") or k == "gemm_bf16_kernel<1>"
               or k.endswith(", 1, false>") or k.endswith(", 1, true>"))]
    if l1:
        k = max(l1, key=lambda n: kernels[n]["hbm_bytes_per_launch"])
        entry["l1_forward_gemm_kernel"] = k
        entry["l1_forward_gemm_bytes_per_launch"] = kernels[k]["hbm_bytes_per_launch"]
    # the wide weight-gradient launch: the split-K launch (XCfg<..., true, true, ...>, EPI_STORE = 0)
    # moving the most bytes (round 5: its tile width follows the layer widths, gemm.hip pick_tile_n)
    wg = [k for k in kernels if k.startswith("gemm_x_kernel<XCfg<") and ", true, true, " in k and
          k.split(">, ")[-1].startswith("0, ")]
    if wg:
        k = max(wg, key=lambda n: kernels[n]["hbm_bytes_per_launch"])
        entry["wgrad_wide_kernel"] = k
        entry["wgrad_wide_bytes_per_launch"] = kernels[k]["hbm_bytes_per_launch"]
    ib = [k for k in kernels if k.startswith("inbatch")]
    if ib:
        k = max(ib, key=lambda n: kernels[n]["hbm_bytes_per_launch"])
        entry["inbatch_bytes_per_launch"] = kernels[k]["hbm_bytes_per_launch"]

    # deferred table AdamW: VALU roofline over the whole run
    rep = [k for k in valu if k.startswith("replay_kernel")]
    if rep:
        instr = sum(sum(valu[k]) for k in rep)
        steps = 40 + 3  # bench --steps 40 --warmup 3: every step's g = 0 updates are replayed by the end
        B_, N_, U_, I_, D_ = c["B"], c["N"], c["U"], c["I"], c["D"]
        # rows a step touches get the real-gradient update instead (row_update_kernel): unique
        # users ~ B, unique items ~ B (1 + N) less repeats; taken as B + B (1 + N) (upper bound of
        # the touched rows, so a lower bound of the replayed element-steps)
        replayed = steps * ((U_ + I_) - (B_ + B_ * (1 + N_))) * D_
        per_es = instr * 64 / replayed  # lane-instructions per element-step
        st = stats.get(rep[0])
        step_ms = None
        if st:
            total_ns = sum(float(stats[k]["TotalDurationNs"]) for k in rep if k in stats)
            step_ms = total_ns / 1e6 / bench["steps"]
        es_per_step = ((U_ + I_) - (B_ + B_ * (1 + N_))) * D_
        hbm = sum(kernels[k]["hbm_bytes_per_launch"] * kernels[k]["launches"] for k in kernels
                  if k.startswith("replay_kernel"))
        out = {
            "kernel": "replay_kernel (deferred AdamW g=0: catch-up of touched rows + rolling slice + flushes)",
            "hbm_bytes_per_step": round(hbm / steps),
            "bound": "valu",
            "valu_lane_instr_per_element_step": round(per_es, 2),
            "element_steps_per_step": es_per_step,
            "replay_ms_per_step": round(step_ms, 4) if step_ms else None,
            "peak_wave_instr_per_s": VALU_ISSUE_PER_S,
        }
        if step_ms:
            achieved = es_per_step * per_es / 64 / (step_ms * 1e-3)
            out["achieved_wave_instr_per_s"] = round(achieved, 0)
            out["frac"] = round(achieved / VALU_ISSUE_PER_S, 4)
        if trans:
            # issue-cycle roofline: every VALU instruction priced at its measured sustained cost
            tr = sum(sum(trans[k]) for k in rep)
            cycles = tr * COST_TRANS + (instr - tr) * COST_OTHER
            out["valu_wave_instr_per_step"] = round(instr / steps)
            out["trans_wave_instr_per_step"] = round(tr / steps)
            out["issue_cycles_per_step"] = round(cycles / steps)
            out["issue_cost_model"] = {"trans_f32": COST_TRANS, "other": COST_OTHER,
                                       "source": "profiles/r03_valu_issue_rates.txt (csrc/tools/valu_bench.cpp)"}
            if step_ms:
                out["issue_frac"] = round(cycles / steps / (step_ms * 1e-3 * SIMD_CYCLES_PER_S), 4)
        entry["replay_valu_roofline"] = out

    path = ROOT / "profiles" / "pmc_traffic.json"
    allp = json.loads(path.read_text()) if path.exists() else {}
    allp[config] = entry
    path.write_text(json.dumps(allp, indent=1) + "\n")
    print(json.dumps({k: v for k, v in entry.items() if k != "kernels"}, indent=1))


if __name__ == "__main__":
    main()
