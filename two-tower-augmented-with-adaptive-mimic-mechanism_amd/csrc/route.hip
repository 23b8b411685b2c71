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
                                                                   const int32_t* __restrict__ blk0,
                                                                   int64_t* __restrict__ grp) {
    extern __shared__ int64_t tot[];  // [W] totals, then their exclusive scan
    int64_t* tot0 = tot + W;          // (blk0) [W] id0 totals
    for (int o = threadIdx.x; o < W; o += kRouteThreads) {
        int64_t t = 0, t0 = 0;
        for (int b = 0; b < nb; ++b) t += blk[(int64_t)b * W + o];
        if (ld >= 3)
            for (int b = 0; b < nb && blk0; ++b) t0 += blk0[(int64_t)b * W + o];
        tot[o] = t;
        if (blk0) tot0[o] = t0;
        counts[o * ld] = t;
        if (status) counts[o * ld + 1] = (int64_t)*status;
        if (ld >= 3) counts[o * ld + 2] = t0;  // of them from id0 (a step's positives)
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // exclusive scan over owners (W <= 1024)
        int64_t run = 0, run0 = 0;
        for (int o = 0; o < W; ++o) {
            const int64_t t = tot[o];
            tot[o] = run;
            run += t;
            if (grp) {  // the compact exchange units of owner o's group: (first row, id0 rows before, id0 rows)
                grp[3 * o] = tot[o];
                grp[3 * o + 1] = run0;
                grp[3 * o + 2] = tot0[o];
                run0 += tot0[o];
            }
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

// grp (compact exchange units, counts_ld >= 3): slot[j] = the request's first unit instead of its row
__global__ __launch_bounds__(kRouteThreads) void route_scatter_kernel(RouteIn a, const int32_t* __restrict__ blk,
                                                                      int owner_bits, int64_t* __restrict__ packed,
                                                                      int64_t* __restrict__ slot,
                                                                      const int64_t* __restrict__ grp) {
    extern __shared__ int32_t lds[];
    const int W = (int)a.world;
    int32_t* off = lds;       // [W] next slot of each owner in this block
    int32_t* wc = lds + W;    // [kRouteWaves][W] this round's per-wave counts
    int64_t* gt = reinterpret_cast<int64_t*>(lds + W * (1 + kRouteWaves + ((1 + kRouteWaves) & 1)));  // [3W]
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int o = threadIdx.x; o < W; o += kRouteThreads) off[o] = blk[(int64_t)blockIdx.x * W + o];
    if (grp)
        for (int e = threadIdx.x; e < 3 * W; e += kRouteThreads) gt[e] = grp[e];
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
            if (grp) {
                const int64_t r = s - gt[3 * o], p = gt[3 * o + 2];
                slot[j] = s + gt[3 * o + 1] + (r < p ? r : p);
            } else {
                slot[j] = s;
            }
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

}  // namespace

size_t route_scratch_bytes(int64_t n, int world) {
    const int64_t nb = n > 0 ? ceil_div(n, kRouteSpan) : 0;
    const int64_t w = world > 0 ? world : 0;
    return (size_t)(2 * nb * w) * sizeof(int32_t) + 8 + (size_t)(3 * w) * sizeof(int64_t);  // blk, blk0, grp
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
        hipLaunchKernelGGL(route_scan_kernel, dim3(1), dim3(kRouteThreads), 2 * sizeof(int64_t) * world, s,
                           static_cast<int32_t*>(nullptr), 0, world, counts, counts_ld, status,
                           static_cast<const int32_t*>(nullptr), static_cast<int64_t*>(nullptr));
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
    int64_t* grp = nullptr;  // [3 world], 8-B aligned after blk, blk0
    if (blk0) grp = reinterpret_cast<int64_t*>(align_up(reinterpret_cast<uintptr_t>(blk + 2 * (int64_t)nb * world), 8));
    hipLaunchKernelGGL(route_count_kernel, dim3(nb), dim3(kRouteThreads), 2 * sizeof(int32_t) * world, s, a, blk,
                       blk0);
    TTAMM_LAUNCH_CHECK();
    hipLaunchKernelGGL(route_scan_kernel, dim3(1), dim3(kRouteThreads), 2 * sizeof(int64_t) * world, s, blk, nb, world,
                       counts, counts_ld, status, static_cast<const int32_t*>(blk0), grp);
    TTAMM_LAUNCH_CHECK();
    // LDS: off [W], wc [waves][W] (int32, padded to 8 B), then grp's copy [3W] (int64)
    const size_t lds_i32 = (size_t)world * (1 + kRouteWaves + ((1 + kRouteWaves) & 1));
    hipLaunchKernelGGL(route_scatter_kernel, dim3(nb), dim3(kRouteThreads),
                       sizeof(int32_t) * lds_i32 + (grp ? sizeof(int64_t) * 3 * world : 0), s, a, blk, bits, packed,
                       slot, static_cast<const int64_t*>(grp));
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

}  // namespace ttamm
