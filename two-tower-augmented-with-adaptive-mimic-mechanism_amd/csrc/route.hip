// Owner routing of a row-sharded step: group n ids by owner rank (id % world), stably, and
// emit each position's slot in that order plus the (local row, key) rows the owners receive.
// It replaces the host-side torch.argsort(owner, stable=True) / bincount / gathers of the
// sharded step (ttamm/sharded.py route_requests, route_pairs) with three small launches:
//   count    one block per 2048 positions: per-owner counts in LDS           -> blk[b][o]
//   scan     one block: counts[o], then blk[b][o] := first slot of (b, o)   (owner-major,
//            block-minor: the stable order)
//   scatter  one block per 2048 positions, 256 at a time in position order: a position's rank
//            among the equal-owner positions of its wave comes from ballots over the owner's
//            bits, the waves before it from per-wave counts in LDS.
// Integer-only, so the result is exactly the stable sort (oracle: tests/test_route_gpu.py).
#include "kernels.h"

namespace ttamm {

namespace {

constexpr int kRouteThreads = 256;
constexpr int kRouteRounds = 8;
constexpr int kRouteSpan = kRouteThreads * kRouteRounds;  // positions per block
constexpr int kRouteWaves = kRouteThreads / 64;

struct RouteIn {
    const int64_t* id0;
    int64_t n0;
    const int64_t* id1;
    int64_t n;  // n0 + n1
    const int64_t* payload;
    int64_t key0, key1;
    uint64_t world;
};

__device__ __forceinline__ uint64_t id_at(const RouteIn& a, int64_t j) {
    return (uint64_t)(j < a.n0 ? a.id0[j] : a.id1[j - a.n0]);
}

// blk[b][o]: ids of block b owned by o; blk0[b][o] (when given): of them from id0
__global__ __launch_bounds__(kRouteThreads) void route_count_kernel(RouteIn a, int32_t* __restrict__ blk,
                                                                    int32_t* __restrict__ blk0) {
    extern __shared__ int32_t hist[];
    const int W = (int)a.world;
    int32_t* hist0 = hist + W;
    for (int o = threadIdx.x; o < 2 * W; o += kRouteThreads) hist[o] = 0;
    __syncthreads();
    const int64_t lo = (int64_t)blockIdx.x * kRouteSpan;
    for (int r = 0; r < kRouteRounds; ++r) {
        const int64_t j = lo + r * kRouteThreads + threadIdx.x;
        if (j < a.n) {
            const int o = (int)(id_at(a, j) % a.world);
            atomicAdd(&hist[o], 1);
            if (blk0 && j < a.n0) atomicAdd(&hist0[o], 1);
        }
    }
    __syncthreads();
    for (int o = threadIdx.x; o < W; o += kRouteThreads) {
        blk[(int64_t)blockIdx.x * W + o] = hist[o];
        if (blk0) blk0[(int64_t)blockIdx.x * W + o] = hist0[o];
    }
}

__global__ __launch_bounds__(kRouteThreads) void route_scan_kernel(int32_t* __restrict__ blk, int nb, int W,
                                                                   int64_t* __restrict__ counts, int64_t ld,
                                                                   const uint32_t* __restrict__ status,
                                                                   const int32_t* __restrict__ blk0) {
    extern __shared__ int64_t tot[];
    for (int o = threadIdx.x; o < W; o += kRouteThreads) {
        int64_t t = 0, t0 = 0;
        for (int b = 0; b < nb; ++b) t += blk[(int64_t)b * W + o];
        if (ld >= 3)
            for (int b = 0; b < nb && blk0; ++b) t0 += blk0[(int64_t)b * W + o];
        tot[o] = t;
        counts[o * ld] = t;
        if (status) counts[o * ld + 1] = (int64_t)*status;
        if (ld >= 3) counts[o * ld + 2] = t0;  // of them from id0 (a step's positives)
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // exclusive scan over owners (W <= 1024)
        int64_t run = 0;
        for (int o = 0; o < W; ++o) {
            const int64_t t = tot[o];
            tot[o] = run;
            run += t;
        }
    }
    __syncthreads();
    for (int o = threadIdx.x; o < W; o += kRouteThreads) {
        int64_t run = tot[o];
        for (int b = 0; b < nb; ++b) {
            const int64_t x = blk[(int64_t)b * W + o];
            blk[(int64_t)b * W + o] = (int32_t)run;  // slots < n < 2^31 (checked by the launcher)
            run += x;
        }
    }
}

__global__ __launch_bounds__(kRouteThreads) void route_scatter_kernel(RouteIn a, const int32_t* __restrict__ blk,
                                                                      int owner_bits, int64_t* __restrict__ packed,
                                                                      int64_t* __restrict__ slot) {
    extern __shared__ int32_t lds[];
    const int W = (int)a.world;
    int32_t* off = lds;       // [W] next slot of each owner in this block
    int32_t* wc = lds + W;    // [kRouteWaves][W] this round's per-wave counts
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int o = threadIdx.x; o < W; o += kRouteThreads) off[o] = blk[(int64_t)blockIdx.x * W + o];
    const int64_t lo = (int64_t)blockIdx.x * kRouteSpan;
    const uint64_t below = (1ull << lane) - 1ull;
    for (int r = 0; r < kRouteRounds; ++r) {
        for (int i = threadIdx.x; i < kRouteWaves * W; i += kRouteThreads) wc[i] = 0;
        __syncthreads();
        const int64_t j = lo + r * kRouteThreads + threadIdx.x;
        const bool valid = j < a.n;
        uint64_t id = 0;
        int o = 0;
        if (valid) {
            id = id_at(a, j);
            o = (int)(id % a.world);
        }
        uint64_t m = __ballot(valid);  // lanes with the same owner as this one
        for (int k = 0; k < owner_bits; ++k) {
            const bool bit = (o >> k) & 1;
            const uint64_t bal = __ballot(valid && bit);
            m &= bit ? bal : ~bal;
        }
        const int rank = __popcll(m & below);
        if (valid && rank == 0) wc[w * W + o] = __popcll(m);
        __syncthreads();
        if (valid) {
            int32_t s = off[o] + rank;
            for (int q = 0; q < w; ++q) s += wc[q * W + o];
            slot[j] = s;
            packed[2 * (int64_t)s] = (int64_t)(id / a.world);
            packed[2 * (int64_t)s + 1] = a.payload ? a.payload[j] : (j < a.n0 ? a.key0 + j : a.key1 + (j - a.n0));
        }
        __syncthreads();
        for (int oo = threadIdx.x; oo < W; oo += kRouteThreads) {
            int32_t t = 0;
            for (int q = 0; q < kRouteWaves; ++q) t += wc[q * W + oo];
            off[oo] += t;
        }
        // the next round's zeroing of wc is ordered after these reads by its own barrier below
        __syncthreads();
    }
}

// Compact exchange units (ttamm.h ttamm_step_args.exchange_counts): groups o = 0 .. W-1 of
// counts[o * ld] rows each, the first counts[o * ld + 2] of them positives (two units) and the
// rest negatives (one unit).  Row s (s = slot[i] when slot is given, else i) starts at unit
//   s + (positives of the groups before o) + min(s - start(o), positives of o);
// mark_neg stores ~unit for a negative row (the owner's row maps carry the row class).
constexpr int kUnitThreads = 256;
__global__ __launch_bounds__(kUnitThreads) void exchange_units_kernel(const int64_t* __restrict__ counts, int64_t ld,
                                                                     int W, const int64_t* __restrict__ slot,
                                                                     int64_t n, int mark_neg, int64_t* __restrict__ out) {
    extern __shared__ int64_t tab[];  // start[W], pcum[W], pos[W]
    int64_t* start = tab;
    int64_t* pcum = tab + W;
    int64_t* pos = tab + 2 * W;
    if (threadIdx.x == 0) {
        int64_t r = 0, p = 0;
        for (int o = 0; o < W; ++o) {
            const int64_t c = counts[o * ld], q = counts[o * ld + 2];
            start[o] = r;
            pcum[o] = p;
            pos[o] = q;
            r += c;
            p += q;
        }
    }
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * kUnitThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kUnitThreads) {
        const int64_t s = slot ? slot[i] : i;
        int lo = 0, hi = W - 1;  // the last group starting at or before s (empty groups share starts)
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (start[mid] <= s) lo = mid;
            else hi = mid - 1;
        }
        const int64_t r = s - start[lo], p = pos[lo];
        const int64_t unit = s + pcum[lo] + (r < p ? r : p);
        out[i] = (mark_neg && r >= p) ? ~unit : unit;
    }
}

}  // namespace

int launch_exchange_units(const int64_t* counts, int64_t ld, int W, const int64_t* slot, int64_t n, int mark_neg,
                          int64_t* out, hipStream_t s) {
    TTAMM_REQUIRE(W >= 1 && W <= 1024 && ld >= 3 && counts, "exchange units: bad count rows");
    if (n <= 0) return TTAMM_OK;
    TTAMM_REQUIRE(out != nullptr, "exchange units: null output");
    const int64_t blocks = std::min<int64_t>(ceil_div(n, kUnitThreads), 4096);
    hipLaunchKernelGGL(exchange_units_kernel, dim3((unsigned)blocks), dim3(kUnitThreads), 3 * sizeof(int64_t) * W, s,
                       counts, ld, W, slot, n, mark_neg, out);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

size_t route_scratch_bytes(int64_t n, int world) {
    const int64_t nb = n > 0 ? ceil_div(n, kRouteSpan) : 0;
    return (size_t)(2 * nb * (world > 0 ? world : 0)) * sizeof(int32_t);  // blk, blk0
}

int launch_route_rows(const int64_t* id0, int64_t n0, const int64_t* id1, int64_t n1, const int64_t* payload,
                      int64_t key0, int64_t key1, int world, int64_t* packed, int64_t* slot, int64_t* counts,
                      int64_t counts_ld, const uint32_t* status, void* scratch, size_t scratch_bytes, hipStream_t s) {
    TTAMM_REQUIRE(world >= 1 && world <= 1024, "route: world must be in [1, 1024]");
    TTAMM_REQUIRE(n0 >= 0 && n1 >= 0 && n0 + n1 < (int64_t(1) << 31), "route: bad sizes");
    TTAMM_REQUIRE(counts != nullptr, "route: counts missing");
    TTAMM_REQUIRE(counts_ld >= 1 && (status == nullptr || counts_ld >= 2), "route: counts_ld must be >= 1 (>= 2 with status)");
    const int64_t n = n0 + n1;
    if (n == 0) {  // zero counts (and the status column): the scan over no blocks
        hipLaunchKernelGGL(route_scan_kernel, dim3(1), dim3(kRouteThreads), sizeof(int64_t) * world, s,
                           static_cast<int32_t*>(nullptr), 0, world, counts, counts_ld, status,
                           static_cast<const int32_t*>(nullptr));
        TTAMM_LAUNCH_CHECK();
        return TTAMM_OK;
    }
    TTAMM_REQUIRE((n0 == 0 || id0) && (n1 == 0 || id1) && packed && slot, "route: null pointer");
    TTAMM_REQUIRE(scratch && scratch_bytes >= route_scratch_bytes(n, world), "route: scratch too small");
    RouteIn a{id0, n0, id1, n, payload, key0, key1, (uint64_t)world};
    const int nb = (int)ceil_div(n, kRouteSpan);
    int bits = 0;
    while ((1 << bits) < world) ++bits;
    int32_t* blk = static_cast<int32_t*>(scratch);
    int32_t* blk0 = counts_ld >= 3 ? blk + (int64_t)nb * world : nullptr;
    hipLaunchKernelGGL(route_count_kernel, dim3(nb), dim3(kRouteThreads), 2 * sizeof(int32_t) * world, s, a, blk,
                       blk0);
    TTAMM_LAUNCH_CHECK();
    hipLaunchKernelGGL(route_scan_kernel, dim3(1), dim3(kRouteThreads), sizeof(int64_t) * world, s, blk, nb, world,
                       counts, counts_ld, status, static_cast<const int32_t*>(blk0));
    TTAMM_LAUNCH_CHECK();
    hipLaunchKernelGGL(route_scatter_kernel, dim3(nb), dim3(kRouteThreads),
                       sizeof(int32_t) * world * (1 + kRouteWaves), s, a, blk, bits, packed, slot);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

}  // namespace ttamm
