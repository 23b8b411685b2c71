#!/usr/bin/env python3
"""C4 embedding-gather benchmark (BASELINE configs[3], north_star target: >= 60 % of the HBM
read roofline on the 50M x 128 embedding gather).

    python tools/bench_gather.py [--rows 50000000] [--dim 128] [--batch 8192] [--neg 5]

The table is one rank's item-ID table at C4 size (50M x 128 fp32 = 25.6 GB; at 8 GPUs each
owner holds 6.25M rows, so the whole table on one GPU is the harder, cache-hostile case).  One
launch gathers what one owner serves per step, B(1+N) = 49,152 rows (the requests of a global
8 x 8192 batch spread over 8 owners), and a bulk launch of 2M rows shows the streaming rate.
Indices: uniform (every row a cold HBM read) and Zipf(1.05) through a fixed permutation (the
bench's interaction distribution).  Timed with HIP events on the launch stream over 50
launches; every launch's output is checked bit-exact against torch.index_select.

Algorithmic bytes per row: dim*4 read (the table row) + dim*4 written + 8 (int64 index).
`read_frac` prices the table-row reads alone against 8 TB/s (the north_star's "HBM-read
roofline"); `frac` prices all algorithmic bytes.  `bulk_read_only` is the product's read-only
gather of a 50M x 128 table: ttamm_candidate_topk scoring uniform random candidate rows by id
(the sampled-candidate evaluation), 4 B written per 512 B row read."""

from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "two-tower-augmented-with-adaptive-mimic-mechanism_amd"))

import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0


def zipf_rows(n: int, rows: int, s: float, gen: torch.Generator, device) -> torch.Tensor:
    """Zipf(s) ranks over `rows` (inverse-CDF on a float64 rank grid), then a fixed random
    permutation so hot rows are spread over the table."""
    # P(rank <= r) ~ H(r)/H(rows), approximated by the continuous integral r^(1-s)
    u = torch.rand(n, generator=gen, device=device, dtype=torch.float64)
    a = 1.0 - s
    top = float(rows) ** a
    r = torch.floor((u * (top - 1.0) + 1.0) ** (1.0 / a)).long().clamp_(1, rows) - 1
    perm_key = (r * 2654435761 + 97) % rows  # a fixed bijection-like scramble of the ranks
    return perm_key


def run(lib, L, table: torch.Tensor, idx: torch.Tensor, reps: int) -> dict:
    n, D = idx.numel(), table.shape[1]
    out = torch.empty((n, D), dtype=torch.float32, device=table.device)
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream

    def launch():
        L.check(lib.ttamm_gather_rows(table.data_ptr(), table.shape[0], D, idx.data_ptr(), n, out.data_ptr(), D, sp))

    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    ref = torch.index_select(table, 0, idx)
    exact = bool(torch.equal(out, ref))
    del ref
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for _ in range(reps):
        launch()
    ev1.record(stream)
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / reps
    read_b = n * D * 4
    total_b = n * (2 * D * 4 + 8)
    return {"rows": n, "avg_launch_us": round(ms * 1e3, 2), "read_GBps": round(read_b / ms / 1e6, 1),
            "read_frac": round(read_b / ms / 1e6 / HBM_PEAK_GBS, 4), "total_GBps": round(total_b / ms / 1e6, 1),
            "frac": round(total_b / ms / 1e6 / HBM_PEAK_GBS, 4), "bit_exact": exact}


def run_candidates(lib, L, table: torch.Tensor, nq: int, per_q: int, reps: int, gen: torch.Generator,
                   k: int = 20) -> dict:
    """ttamm_candidate_topk (the sampled-candidate evaluation, training.py:974-1009) over `nq`
    queries with `per_q` uniform candidate rows each: every candidate is one random row of the
    table read by index (its only HBM traffic besides 8 B of id), scored and ranked in LDS.
    Checked against torch: the top-k positions of a sample of queries."""
    dev = table.device
    rows, D = table.shape
    q = torch.randn((nq, D), generator=gen, device=dev, dtype=torch.float32)
    cand = torch.randint(0, rows, (nq * per_q,), generator=gen, device=dev)
    off = torch.arange(0, nq * per_q + 1, per_q, device=dev, dtype=torch.long)
    out_s = torch.empty((nq, k), dtype=torch.float32, device=dev)
    out_p = torch.empty((nq, k), dtype=torch.long, device=dev)
    sp = torch.cuda.current_stream().cuda_stream

    def launch():
        L.check(lib.ttamm_candidate_topk(q.data_ptr(), nq, D, table.data_ptr(), rows, D, D, off.data_ptr(),
                                         cand.data_ptr(), per_q, 0, k, out_s.data_ptr(), out_p.data_ptr(), sp))

    for _ in range(2):
        launch()
    torch.cuda.synchronize()
    sample = torch.arange(0, nq, max(1, nq // 512), device=dev)
    ref = (table[cand.view(nq, per_q)[sample]] * q[sample, None, :]).sum(-1)
    ref_top = torch.topk(ref, k, dim=1).values
    score_err = float((out_s[sample] - ref_top).abs().max() / ref_top.abs().max())
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(reps):
        launch()
    ev1.record()
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / reps
    read_b = nq * per_q * D * 4
    return {"queries": nq, "candidates_per_query": per_q, "rows_read": nq * per_q, "avg_launch_ms": round(ms, 4),
            "read_GBps": round(read_b / ms / 1e6, 1), "read_frac": round(read_b / ms / 1e6 / HBM_PEAK_GBS, 4),
            "topk_score_rel_err_vs_torch": score_err}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=50_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--neg", type=int, default=5)
    ap.add_argument("--bulk", type=int, default=2_000_000)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--cand-queries", type=int, default=200_000)
    ap.add_argument("--cand-per-query", type=int, default=101)
    args = ap.parse_args()

    from ttamm import _lib as L

    lib = L.load()
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234)
    table = torch.empty((args.rows, args.dim), dtype=torch.float32, device=dev)
    chunk = 1 << 22
    for lo in range(0, args.rows, chunk):  # N(0, 0.02) init (encoders.py:19-36), in chunks
        table[lo:lo + chunk].normal_(0.0, 0.02, generator=gen)
    step_rows = args.batch * (1 + args.neg)
    results = {}
    for name, n in (("step", step_rows), ("bulk", args.bulk)):
        uni = torch.randint(0, args.rows, (n,), generator=gen, device=dev)
        zipf = zipf_rows(n, args.rows, 1.05, gen, dev)
        results[name] = {"uniform": run(lib, L, table, uni, args.reps), "zipf": run(lib, L, table, zipf, args.reps)}
    results["bulk_read_only"] = {"candidate_topk_uniform": run_candidates(lib, L, table, args.cand_queries,
                                                                         args.cand_per_query, 5, gen)}
    line = {
        "metric": "C4 embedding row gather (ttamm_gather_rows), HBM read roofline",
        "config": {"table": f"{args.rows} x {args.dim} fp32", "step_rows": step_rows,
                   "step_rows_meaning": f"B(1+N) = {args.batch} x {1 + args.neg} rows an owner serves per step",
                   "bulk_rows": args.bulk},
        "roofline": {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "achieved": results["step"]["uniform"]["read_GBps"],
                     "frac": results["step"]["uniform"]["read_frac"],
                     "note": "table-row reads of one step-sized launch, uniform indices"},
        "results": results,
    }
    print(json.dumps(line))


if __name__ == "__main__":
    main()
