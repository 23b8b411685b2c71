// Exact inner-product retrieval with per-query blocked items and top-k.
//
// Replaces the FAISS IndexFlatIP search + the candidate filter of `_evaluate_model`
// (training.py:944-970, index built at :645-679): for every query q, the k items with the
// highest <Q[q], X[i]> that are not in q's blocked set, ordered by score (descending) then item
// id (ascending).  FAISS's own tie order is an implementation detail of its heaps; this
// kernel's is the total order above.
//
// Pass 1 (retrieval_partial_kernel): a block owns 64 queries and one partition of the items.
// Four waves: (query half, item half) of each 64-item tile.  Scores come from fp32 MFMA
// 32x32x2 with items as M and queries as N, so every lane holds ONE query and 16 items of the
// tile.  A lane appends (score, id) to its query's candidate buffer only when the score reaches
// the query's running threshold (the k-th best so far); a wave compacts a query's buffer
// (blocked items dropped, bitonic sort in registers, keep k) before it could overflow.
// D <= 128 runs the same scheme on split-bf16 MFMA (retrieval_x_kernel: fp32-level scores at
// 2.6x the fp32 MFMA rate; TTAMM_RETRIEVAL_FP32=1 keeps the fp32 kernel for comparison).
// Pass 2 (retrieval_merge_kernel): one wave per query merges the partitions' top-k lists.
#include <cfloat>
#include <cstdlib>
#include <cstring>

#include "kernels.h"

namespace ttamm {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kRQ = 64;      // queries per block
constexpr int kRI = 64;      // items per tile
constexpr int kRCap = 256;   // candidate slots per query: k + kRI <= kRCap
constexpr int kMergeJ = 8;   // merge: up to 64 * 8 = 512 candidates per query
constexpr int kLinearBlocked = 64;  // blocked lists up to this long: one wave-wide scan

__device__ __forceinline__ bool better(float sa, int ia, float sb, int ib) {
    return sa > sb || (sa == sb && (unsigned)ia < (unsigned)ib);
}

// Sort the 64*J (score, id) pairs of a wave — element e = lane*J + j — best first.
template <int J>
__device__ void wave_bitonic_sort(float (&s)[J], int (&id)[J]) {
    const int lane = threadIdx.x & 63;
    constexpr int N = 64 * J;
#pragma unroll
    for (int size = 2; size <= N; size <<= 1) {
#pragma unroll
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            if (stride >= J) {
                const int ls = stride / J;
#pragma unroll
                for (int j = 0; j < J; ++j) {
                    const int e = lane * J + j;
                    const float ps = __shfl_xor(s[j], ls, 64);
                    const int pi = __shfl_xor(id[j], ls, 64);
                    const bool dir = (e & size) == 0;       // block sorted best-first
                    const bool lower = (e & stride) == 0;
                    const bool mine_better = better(s[j], id[j], ps, pi);
                    if (mine_better != (lower == dir)) {
                        s[j] = ps;
                        id[j] = pi;
                    }
                }
            } else {
#pragma unroll
                for (int j = 0; j < J; ++j) {
                    if (j & stride) continue;
                    const int e = lane * J + j;
                    const bool dir = (e & size) == 0;
                    const int k = j | stride;
                    if (better(s[k], id[k], s[j], id[j]) == dir) {
                        const float ts = s[j];
                        const int ti = id[j];
                        s[j] = s[k];
                        id[j] = id[k];
                        s[k] = ts;
                        id[k] = ti;
                    }
                }
            }
        }
    }
}

// Sort query q's buffered candidates, keep the best k, update its threshold.  With a blocked
// list (bval[blo, bhi), sorted; the split kernel defers the blocked test to here) candidates on
// it are dropped first: the wave loads the list 64 values at a time and every lane compares its
// four candidates against each value (one load round trip per 64 blocked items, instead of a
// dependent binary search per inserted candidate); lists longer than kLinearBlocked take one
// lower-bound search per candidate instead (cost log n, not n / 64 x 64).
__device__ int compact_core(float* __restrict__ bs, int* __restrict__ bi, int q, int n, int k, float* out_s,
                             int* out_i, int out_k, const int64_t* __restrict__ bval, int64_t blo, int64_t bhi,
                             float& tau_out) {
    const int lane = threadIdx.x & 63;
    float s[4];
    int id[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int e = lane * 4 + j;
        s[j] = e < n ? bs[q * kRCap + e] : -INFINITY;
        id[j] = e < n ? bi[q * kRCap + e] : -1;
    }
    if (bhi - blo > kLinearBlocked) {
        // a long list (a heavy user's history): a branchless lower bound per candidate, the four
        // searches of a lane interleaved — log2(n) rounds of four independent L2-resident loads
        // instead of n / 64 rounds of 64 compares per candidate.  The trip count depends on n
        // only, so the wave stays converged.
        int64_t base[4];
        const int64_t cnt = bhi - blo;
#pragma unroll
        for (int j = 0; j < 4; ++j) base[j] = blo;
        for (int64_t len = cnt; len > 1;) {
            const int64_t half = len >> 1;
            int64_t b[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) b[j] = bval[base[j] + half];
#pragma unroll
            for (int j = 0; j < 4; ++j) base[j] = b[j] <= (int64_t)id[j] ? base[j] + half : base[j];
            len -= half;
        }
        int kept = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (id[j] >= 0 && bval[base[j]] == (int64_t)id[j]) {
                s[j] = -INFINITY;
                id[j] = -1;
            }
            kept += __popcll(__ballot(lane * 4 + j < n && id[j] >= 0));
        }
        n = kept;
    } else if (bhi > blo) {
        bool drop[4] = {false, false, false, false};
        for (int64_t c0 = blo; c0 < bhi; c0 += 64) {
            const int64_t v = c0 + lane < bhi ? bval[c0 + lane] : int64_t(-1);
            const int m = bhi - c0 < 64 ? (int)(bhi - c0) : 64;
            const int vlo = (int)(uint32_t)v, vhi = (int)(v >> 32);
            for (int i = 0; i < m; ++i) {
                const int64_t b = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane(vhi, i) << 32) |
                                            (uint32_t)__builtin_amdgcn_readlane(vlo, i));
#pragma unroll
                for (int j = 0; j < 4; ++j) drop[j] |= id[j] >= 0 && (int64_t)id[j] == b;
            }
        }
        int kept = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (drop[j]) {
                s[j] = -INFINITY;  // sorts after every kept candidate (id -1 last among ties)
                id[j] = -1;
            }
            kept += __popcll(__ballot(lane * 4 + j < n && !drop[j]));
        }
        n = kept;
    }
    wave_bitonic_sort<4>(s, id);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int e = lane * 4 + j;
        if (e < k && e < n) {
            bs[q * kRCap + e] = s[j];
            bi[q * kRCap + e] = id[j];
        }
        if (out_s && e < out_k) {
            out_s[e] = e < n ? s[j] : -INFINITY;
            out_i[e] = e < n ? id[j] : -1;
        }
    }
    // the k-th best (element k - 1 = lane (k-1)/4, slot (k-1)%4) to every lane
    const int jk = (k - 1) & 3;
    const float sk = jk == 0 ? s[0] : jk == 1 ? s[1] : jk == 2 ? s[2] : s[3];
    const float kth = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sk), (k - 1) >> 2));
    tau_out = k <= n ? kth : -INFINITY;
    return n < k ? n : k;
}

__device__ void compact_query(float* __restrict__ bs, int* __restrict__ bi, int* cnt, float* tau, int q, int k,
                              float* out_s, int* out_i, int out_k, const int64_t* __restrict__ bval = nullptr,
                              int64_t blo = 0, int64_t bhi = 0) {
    float t;
    const int nc = compact_core(bs, bi, q, cnt[q], k, out_s, out_i, out_k, bval, blo, bhi, t);
    if ((threadIdx.x & 63) == 0) {
        cnt[q] = nc;
        tau[q] = t;
    }
}

// IT items per tile: wave (qw, iw) scores queries [32 qw, 32 qw + 32) against items
// [iw IT/2, (iw+1) IT/2) of the tile — IT/64 MFMA tiles sharing the query fragments.  The next
// tile's rows are loaded into registers while the current one is scored (PF float4 per thread).
template <int IT, int DMAX>
__global__ __launch_bounds__(256) void retrieval_partial_kernel(RetrievalArgs A) {
    constexpr int MT = IT / 64;                       // 32x32 MFMA tiles per wave
    constexpr int PF = (IT * DMAX / 4 + 255) / 256;   // prefetch float4 per thread
    extern __shared__ __attribute__((aligned(16))) float lds[];
    __shared__ int cnt[kRQ];
    __shared__ float tau[kRQ];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int qw = w & 1, iw = w >> 1, h = lane >> 5;
    const int D = A.D, LD = D + 4, D4 = D >> 2, Dh = D >> 1;
    const int64_t q0 = (int64_t)blockIdx.x * kRQ;
    const int64_t i_begin = (int64_t)blockIdx.y * A.items_per_part;
    const int64_t i_end = i_begin + A.items_per_part < A.ni ? i_begin + A.items_per_part : A.ni;
    float* Qs = lds;
    float* Xs = lds + kRQ * LD;
    for (int e = tid; e < kRQ * D4; e += 256) {
        const int r = e / D4, c = (e - r * D4) * 4;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (q0 + r < A.nq) v = *reinterpret_cast<const float4*>(A.Q + (q0 + r) * A.ldq + c);
        *reinterpret_cast<float4*>(Qs + r * LD + c) = v;
    }
    if (tid < kRQ) {
        cnt[tid] = 0;
        tau[tid] = -INFINITY;
    }
    const int64_t blk = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
    float* bs = A.buf_s + blk * kRQ * kRCap;
    int* bi = A.buf_i + blk * kRQ * kRCap;
    const int myq = qw * 32 + (lane & 31);
    const int64_t gq = q0 + myq;
    const bool qvalid = gq < A.nq;
    const float* qb = Qs + myq * LD + h * Dh;
    float4 pf[PF];
    auto load_tile = [&](int64_t t0) {
#pragma unroll
        for (int it = 0; it < PF; ++it) {
            const int e = tid + it * 256;
            const int r = e / D4, c = (e - r * D4) * 4;
            pf[it] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (e < IT * D4 && t0 + r < i_end) pf[it] = *reinterpret_cast<const float4*>(A.X + (t0 + r) * A.ldx + c);
        }
    };
    auto store_tile = [&]() {
#pragma unroll
        for (int it = 0; it < PF; ++it) {
            const int e = tid + it * 256;
            const int r = e / D4, c = (e - r * D4) * 4;
            if (e < IT * D4) *reinterpret_cast<float4*>(Xs + r * LD + c) = pf[it];
        }
    };
    if (i_begin < i_end) {
        load_tile(i_begin);
        store_tile();
    }
    for (int64_t t0 = i_begin; t0 < i_end; t0 += IT) {
        __syncthreads();  // tile t0 is in LDS; thresholds and counts are current
        if (t0 + IT < i_end && !(kDevKnobs && (A.ablate & 4))) load_tile(t0 + IT);
        const float my_tau = tau[myq];
        f32x16 acc[MT];
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[m][r] = 0.f;
        // lane half h sums k in [h*D/2, (h+1)*D/2) — the same k order for both operands
        const float* xa = Xs + (iw * (IT / 2) + (lane & 31)) * LD + h * Dh;
#pragma unroll 4
        for (int kk = 0; kk < Dh; kk += 4) {
            const float4 b4 = *reinterpret_cast<const float4*>(qb + kk);
            float4 a4[MT];
#pragma unroll
            for (int m = 0; m < MT; ++m) a4[m] = *reinterpret_cast<const float4*>(xa + m * 32 * LD + kk);
            // accumulators interleaved: consecutive MFMAs never depend on each other
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int m = 0; m < MT; ++m)
                    acc[m] = __builtin_amdgcn_mfma_f32_32x32x2f32(q == 0 ? a4[m].x : q == 1 ? a4[m].y : q == 2 ? a4[m].z : a4[m].w,
                                                                  q == 0 ? b4.x : q == 1 ? b4.y : q == 2 ? b4.z : b4.w,
                                                                  acc[m], 0, 0, 0);
        }
        // most tiles hold no score at or above the lane's threshold once it has warmed up: one max
        // over the lane's scores skips the per-score filter
        float mx = -INFINITY;
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int r = 0; r < 16; ++r) mx = fmaxf(mx, acc[m][r]);
        if (qvalid && mx >= my_tau) {
#pragma unroll
            for (int m = 0; m < MT; ++m)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int64_t item = t0 + iw * (IT / 2) + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                    const float sc = acc[m][r];
                    if (item < i_end && sc >= my_tau) {  // blocked items are dropped at compaction
                        const int slot = atomicAdd(&cnt[myq], 1);
                        bs[myq * kRCap + slot] = sc;  // slot < kRCap: cnt <= kRCap - IT before the tile
                        bi[myq * kRCap + slot] = (int)item;
                    }
                }
        }
        __syncthreads();  // all scores of the tile are in; Xs is free
        for (int q = w; q < kRQ; q += 4)
            if (cnt[q] > kRCap - IT) {
                const bool bl = A.boff && q0 + q < A.nq;
                compact_query(bs, bi, cnt, tau, q, A.k, nullptr, nullptr, 0, A.bval, bl ? A.boff[q0 + q] : 0,
                              bl ? A.boff[q0 + q + 1] : 0);
            }
        if (t0 + IT < i_end) store_tile();
    }
    __syncthreads();
    for (int q = w; q < kRQ; q += 4) {
        const int64_t g = q0 + q;
        if (g >= A.nq) continue;
        float* os = A.part_s + (g * A.parts + blockIdx.y) * A.k;
        int* oi = A.part_i + (g * A.parts + blockIdx.y) * A.k;
        const bool bl = A.boff != nullptr;
        compact_query(bs, bi, cnt, tau, q, A.k, os, oi, A.k, A.bval, bl ? A.boff[g] : 0, bl ? A.boff[g + 1] : 0);
    }
}

// Split-bf16 variant (D <= 128): every fp32 score as six v_mfma_f32_32x32x16_bf16 products of
// (hi, mid, lo) bf16 planes (x = hi + mid + lo exactly to ~24 bits; the small terms accumulated
// first, as the tower GEMMs of gemm.hip) — fp32-level accuracy, and exact whenever the operands
// are small integers (the hi plane holds them, the other planes are 0).  A block of 8 waves owns
// 256 queries, each wave 32 of them, their planes held in registers as MFMA B fragments for the
// whole padded K; the partition's items stream through double-buffered LDS planes in 64-item
// tiles (fp32 loads of the next tile in flight, split in registers, then written).  Query tiles
// 4x the fp32 kernel's cut the item re-reads (one pass over the partition per 256 queries).
constexpr int kXQ = 256;    // queries per block
constexpr int kXThreads = 512;

typedef __bf16 bf16x8r __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4r __attribute__((ext_vector_type(4)));
typedef float f32x4r __attribute__((ext_vector_type(4)));

// x -> (hi, mid, lo) bf16 quadruples (gemm.hip split_bf16<3>)
__device__ __forceinline__ void split3(float4 v, uint2 (&out)[3]) {
    const f32x4r x = {v.x, v.y, v.z, v.w};
    const bf16x4r hi = __builtin_convertvector(x, bf16x4r);
    const f32x4r r = x - __builtin_convertvector(hi, f32x4r);
    const bf16x4r mid = __builtin_convertvector(r, bf16x4r);
    const f32x4r r2 = r - __builtin_convertvector(mid, f32x4r);
    out[0] = __builtin_bit_cast(uint2, hi);
    out[1] = __builtin_bit_cast(uint2, mid);
    out[2] = __builtin_bit_cast(uint2, __builtin_convertvector(r2, bf16x4r));
}

// byte offset of k values [c, c + 4) (c < 16) of item row `row` in a 32-B-row plane: 16-B halves
// swapped on rows with bit 3 set, so the 16 rows of a ds_read_b128 lane group hit distinct bank
// quads (gemm.hip mn_off<32>)
__device__ __forceinline__ int xoff(int row, int c) { return row * 32 + (((c >> 3) ^ ((row >> 3) & 1)) << 4) + (c & 4) * 2; }

template <int KS, int IT>
__global__ __launch_bounds__(kXThreads) void retrieval_x_kernel(RetrievalArgs A) {
    constexpr int MT = IT / 32;           // 32-item MFMA tiles per wave
    constexpr int PLANE = IT * 32;        // one k-step plane: IT rows x 16 bf16
    constexpr int BUF = 3 * KS * PLANE;   // (hi, mid, lo) x k-steps
    constexpr int C4 = 4 * KS;            // float4 chunks per padded row
    constexpr int LOADS = (IT * C4 + kXThreads - 1) / kXThreads;
    extern __shared__ __attribute__((aligned(16))) float lds_f[];  // 2 * BUF bytes
    unsigned char* lds = reinterpret_cast<unsigned char*>(lds_f);
    __shared__ int cnt[kXQ];
    __shared__ float tau[kXQ];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
    const int D = A.D;
    const int64_t q0 = (int64_t)blockIdx.x * kXQ;
    const int64_t i_begin = (int64_t)blockIdx.y * A.items_per_part;
    const int64_t i_end = i_begin + A.items_per_part < A.ni ? i_begin + A.items_per_part : A.ni;
    const int64_t blk = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
    float* bs = A.buf_s + blk * kXQ * kRCap;
    int* bi = A.buf_i + blk * kXQ * kRCap;
    if (tid < kXQ) {
        cnt[tid] = 0;
        tau[tid] = -INFINITY;
    }
    const int myq = w * 32 + (lane & 31);
    const int64_t gq = q0 + myq;
    const bool qvalid = gq < A.nq;
    int64_t blo = 0, bhi = 0;
    if (A.boff && qvalid) {
        blo = A.boff[gq];
        bhi = A.boff[gq + 1];
    }
    // this lane's B fragments: query myq, k = 16 ks + 8 h + [0, 8), zero past D
    bf16x8r qf[3][KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        uint2 lo3[3], hi3[3];
        const int k0 = 16 * ks + 8 * h;
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
        if (qvalid && k0 < D) a = *reinterpret_cast<const float4*>(A.Q + gq * A.ldq + k0);
        if (qvalid && k0 + 4 < D) b = *reinterpret_cast<const float4*>(A.Q + gq * A.ldq + k0 + 4);
        split3(a, lo3);
        split3(b, hi3);
#pragma unroll
        for (int p = 0; p < 3; ++p) qf[p][ks] = __builtin_bit_cast(bf16x8r, make_uint4(lo3[p].x, lo3[p].y, hi3[p].x, hi3[p].y));
    }
    // item tile staging: chunk e -> (row e / C4, k 4 (e % C4)); zero past D and past the partition
    float4 pf[LOADS];
    auto load_tile = [&](int64_t t0) {
#pragma unroll
        for (int it = 0; it < LOADS; ++it) {
            const int e = tid + it * kXThreads;
            const int r = e / C4, c = (e - r * C4) * 4;
            pf[it] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (e < IT * C4 && c < D && t0 + r < i_end) pf[it] = *reinterpret_cast<const float4*>(A.X + (t0 + r) * A.ldx + c);
        }
    };
    auto store_tile = [&](int buf) {
        unsigned char* base = lds + buf * BUF;
#pragma unroll
        for (int it = 0; it < LOADS; ++it) {
            const int e = tid + it * kXThreads;
            if (e >= IT * C4) continue;
            const int r = e / C4, c = (e - r * C4) * 4;
            uint2 v[3];
            split3(pf[it], v);
            const int off = (c >> 4) * PLANE + xoff(r, c & 15);
#pragma unroll
            for (int p = 0; p < 3; ++p) *reinterpret_cast<uint2*>(base + p * KS * PLANE + off) = v[p];
        }
    };
    int buf = 0;
    if (i_begin < i_end) {
        load_tile(i_begin);
        store_tile(0);
    }
    for (int64_t t0 = i_begin; t0 < i_end; t0 += IT) {
        __syncthreads();  // tile t0 is in LDS buffer `buf`; thresholds and counts are current
        if (t0 + IT < i_end && !(kDevKnobs && (A.ablate & 4))) load_tile(t0 + IT);
        const float my_tau = tau[myq];
        const unsigned char* base = lds + buf * BUF;
        f32x16 acc[MT];
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[m][r] = 0.f;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            if (kDevKnobs && (A.ablate & 2)) break;
#pragma unroll
            for (int m = 0; m < MT; ++m) {
                bf16x8r af[3];
#pragma unroll
                for (int p = 0; p < 3; ++p)
                    af[p] = *reinterpret_cast<const bf16x8r*>(base + (p * KS + ks) * PLANE +
                                                              xoff(32 * m + (lane & 31), 8 * h));
                acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1], qf[1][ks], acc[m], 0, 0, 0);
                acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[2], qf[0][ks], acc[m], 0, 0, 0);
                acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0], qf[2][ks], acc[m], 0, 0, 0);
                acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1], qf[0][ks], acc[m], 0, 0, 0);
                acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0], qf[1][ks], acc[m], 0, 0, 0);
                acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0], qf[0][ks], acc[m], 0, 0, 0);
            }
        }
        // hierarchical filter: a wave enters a 32-item group only when one of its lanes has a
        // score >= tau there, then tests that group's scores one by one (steady state: one or
        // two passing scores per wave and tile, so most groups are skipped after one compare)
        float mm[MT];
#pragma unroll
        for (int m = 0; m < MT; ++m) {
            mm[m] = acc[m][0];
#pragma unroll
            for (int r = 1; r < 16; ++r) mm[m] = fmaxf(mm[m], acc[m][r]);
        }
        const bool full = t0 + IT <= i_end;
        if (!(kDevKnobs && (A.ablate & 1)) && qvalid) {
#pragma unroll
            for (int m = 0; m < MT; ++m) {
                if (mm[m] >= my_tau) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const float sc = acc[m][r];
                        if (sc >= my_tau) {
                            const int64_t item = t0 + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                            if (full || item < i_end) {  // blocked items are dropped at compaction
                                const int slot = atomicAdd(&cnt[myq], 1);
                                bs[myq * kRCap + slot] = sc;  // slot < kRCap: cnt <= kRCap - IT before the tile
                                bi[myq * kRCap + slot] = (int)item;
                            }
                        }
                    }
                }
            }
        }
        // compaction of this wave's own 32 queries (their candidates come only from this wave's
        // lanes, so no block barrier): one LDS read per lane and a ballot, then only the buffers
        // near capacity are sorted, in ascending q.  The other LDS buffer is already free: every
        // wave finished reading it before this tile's barrier.
        __threadfence_block();  // this wave's candidate stores before its own compaction loads
        {
            uint64_t need = __ballot(lane < 32 && cnt[w * 32 + lane] > kRCap - IT);
            while (need) {
                const int j = __builtin_ctzll(need);
                need &= need - 1;
                compact_query(bs, bi, cnt, tau, w * 32 + j, A.k, nullptr, nullptr, 0, A.bval, __shfl(blo, j, 64),
                              __shfl(bhi, j, 64));
            }
        }
        if (t0 + IT < i_end && !(kDevKnobs && (A.ablate & 4))) store_tile(buf ^ 1);
        buf ^= 1;
    }
    __syncthreads();  // an empty partition skips the loop: counts and thresholds were set by waves 0-3
    for (int j = 0; j < 32; ++j) {  // this wave's queries: their buffers are written only by it
        const int q = w * 32 + j;
        const int64_t g = q0 + q;
        const int64_t qlo = __shfl(blo, j, 64), qhi = __shfl(bhi, j, 64);
        if (g >= A.nq) continue;
        float* os = A.part_s + (g * A.parts + blockIdx.y) * A.k;
        int* oi = A.part_i + (g * A.parts + blockIdx.y) * A.k;
        compact_query(bs, bi, cnt, tau, q, A.k, os, oi, A.k, A.bval, qlo, qhi);
    }
}

__global__ __launch_bounds__(64) void retrieval_merge_kernel(RetrievalArgs A, float* __restrict__ out_s,
                                                             int64_t* __restrict__ out_i) {
    const int lane = threadIdx.x;
    const int64_t q = blockIdx.x;
    const int n = A.parts * A.k;
    float s[kMergeJ];
    int id[kMergeJ];
#pragma unroll
    for (int j = 0; j < kMergeJ; ++j) {
        const int e = lane * kMergeJ + j;
        s[j] = e < n ? A.part_s[q * n + e] : -INFINITY;
        id[j] = e < n ? A.part_i[q * n + e] : -1;
        if (id[j] < 0) s[j] = -INFINITY;  // empty slots sort last
    }
    wave_bitonic_sort<kMergeJ>(s, id);
#pragma unroll
    for (int j = 0; j < kMergeJ; ++j) {
        const int e = lane * kMergeJ + j;
        if (e < A.k) {
            const bool ok = id[j] >= 0;
            out_s[q * A.k + e] = ok ? s[j] : -INFINITY;
            out_i[q * A.k + e] = ok ? (int64_t)id[j] : -1;
        }
    }
}

int pick_parts(int64_t nq, int64_t ni, int k, int qb = kRQ) {
    const int64_t qtiles = (nq + qb - 1) / qb;
    // the fp32 kernel: >= 2048 blocks (8 per CU).  The split kernel holds one block per CU (144 KB
    // of LDS): one block per CU is enough, and every extra partition costs each query another
    // k ln(items / (parts k)) candidate insertions and their compactions
    const int64_t target = qb == kXQ ? 256 : 2048;
    int64_t parts = (target + qtiles - 1) / qtiles;
    if (const char* e = dev_env("TTAMM_RETRIEVAL_PARTS")) parts = std::atoi(e);  // sweeps only
    const int64_t by_items = (ni + 4 * kRI - 1) / (4 * kRI);  // >= 4 tiles per partition
    if (parts > by_items) parts = by_items;
    const int64_t by_merge = (64 * kMergeJ) / k;
    if (parts > by_merge) parts = by_merge;
    return parts < 1 ? 1 : (int)parts;
}

// faiss.normalize_L2 (faiss/utils/distances.cpp fvec_renorm_L2), applied to the item matrix
// and the queries when the model's similarity is cosine (training.py:670-672, :954-955): each
// row is scaled by 1 / sqrt(sum x^2) in fp32; rows of norm 0 stay as they are.  One wave per
// row, the squares summed lane-strided then by a butterfly.
__global__ __launch_bounds__(256) void normalize_rows_kernel(float* __restrict__ x, int64_t n, int dim, int64_t ld) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n) return;
    float* r = x + row * ld;
    float ss = 0.f;
    for (int c = lane; c < dim; c += 64) ss = fmaf(r[c], r[c], ss);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
    if (ss > 0.f) {
        const float inv = 1.0f / sqrtf(ss);
        for (int c = lane; c < dim; c += 64) r[c] *= inv;
    }
}

// Sampled-candidate retrieval (_retrieve_with_sampling, training.py:974-1009): one block per
// query scores its candidates (one wave per candidate, lanes over D), cosine when `cosine`
// (F.normalize on both sides, :999-1003), then ranks them: a candidate's rank is the number of
// candidates with a larger score, or an equal score at an earlier list position (torch.topk
// order, sorted=True); ranks < k are written.  Candidate lists are at most kCandCap long.
constexpr int kCandCap = 4096;

__global__ __launch_bounds__(256) void candidate_topk_kernel(const float* __restrict__ Q, int64_t ldq,
                                                             const float* __restrict__ X, int64_t ni, int64_t ldx,
                                                             int dim, const int64_t* __restrict__ coff,
                                                             const int64_t* __restrict__ crow, int cosine, int k,
                                                             float* __restrict__ out_s, int64_t* __restrict__ out_p) {
    __shared__ float sc[kCandCap];
    __shared__ float qn;
    const int64_t q = blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t c0 = coff[q];
    const int nc = (int)(coff[q + 1] - c0);
    const float* qr = Q + q * ldq;
    if (wave == 0) {  // ||query||
        float ss = 0.f;
        for (int d = lane; d < dim; d += 64) ss = fmaf(qr[d], qr[d], ss);
        ss = wave_sum(ss);
        if (lane == 0) qn = fmaxf(sqrtf(ss), 1e-12f);
    }
    __syncthreads();
    for (int c = wave; c < nc; c += 4) {
        const int64_t r = crow[c0 + c];
        float dot = 0.f, ss = 0.f;
        if (r >= 0 && r < ni) {
            const float* xr = X + r * ldx;
            for (int d = lane; d < dim; d += 64) {
                dot = fmaf(qr[d], xr[d], dot);
                ss = fmaf(xr[d], xr[d], ss);
            }
        }
        dot = wave_sum(dot);
        ss = wave_sum(ss);
        if (lane == 0) sc[c] = cosine ? dot / (qn * fmaxf(sqrtf(ss), 1e-12f)) : dot;
    }
    __syncthreads();
    for (int c = threadIdx.x; c < nc; c += blockDim.x) {
        const float v = sc[c];
        int rank = 0;
        for (int o = 0; o < nc; ++o) {
            const float w = sc[o];
            rank += (w > v || (w == v && o < c)) ? 1 : 0;
        }
        if (rank < k) {
            out_s[q * k + rank] = v;
            out_p[q * k + rank] = c;
        }
    }
    for (int r = nc + threadIdx.x; r < k; r += blockDim.x) {  // fewer candidates than k
        out_s[q * k + r] = -INFINITY;
        out_p[q * k + r] = -1;
    }
}

// The same scores with G lanes per candidate row and NV float4 columns per lane (dim = 4 G NV),
// U candidates per lane group in flight: each row is 16-B loads by G lanes, reduced over
// log2 G lanes.  The block's 256 / G groups keep 256 U / G random rows in flight — the rows
// are the HBM traffic of this kernel (a gather of the item-vector table by candidate id).
template <int G, int NV>
__global__ __launch_bounds__(256) void candidate_topk_v_kernel(const float* __restrict__ Q, int64_t ldq,
                                                               const float* __restrict__ X, int64_t ni, int64_t ldx,
                                                               const int64_t* __restrict__ coff,
                                                               const int64_t* __restrict__ crow, int cosine, int k,
                                                               float* __restrict__ out_s, int64_t* __restrict__ out_p) {
    constexpr int GPB = 256 / G, U = 2;
    __shared__ float sc[kCandCap];
    const int s = threadIdx.x % G, grp = threadIdx.x / G;
    const int64_t q = blockIdx.x;
    const int64_t c0 = coff[q];
    const int nc = (int)(coff[q + 1] - c0);
    float4 qv[NV];
    float qq = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        qv[i] = *reinterpret_cast<const float4*>(Q + q * ldq + 4 * (s + G * i));
        qq += qv[i].x * qv[i].x + qv[i].y * qv[i].y + qv[i].z * qv[i].z + qv[i].w * qv[i].w;
    }
    for (int o = G / 2; o > 0; o >>= 1) qq += __shfl_xor(qq, o, 64);
    const float qn = fmaxf(sqrtf(qq), 1e-12f);
    for (int cb = grp; cb < nc; cb += GPB * U) {
        int64_t r[U];
        float4 x[U][NV];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int c = cb + u * GPB;
            r[u] = c < nc ? crow[c0 + c] : -1;
            if (r[u] >= ni) r[u] = -1;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int i = 0; i < NV; ++i)
                x[u][i] = r[u] >= 0 ? *reinterpret_cast<const float4*>(X + r[u] * ldx + 4 * (s + G * i))
                                    : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            float dot = 0.f, ss = 0.f;
#pragma unroll
            for (int i = 0; i < NV; ++i) {
                dot += qv[i].x * x[u][i].x + qv[i].y * x[u][i].y + qv[i].z * x[u][i].z + qv[i].w * x[u][i].w;
                ss += x[u][i].x * x[u][i].x + x[u][i].y * x[u][i].y + x[u][i].z * x[u][i].z + x[u][i].w * x[u][i].w;
            }
            for (int o = G / 2; o > 0; o >>= 1) {
                dot += __shfl_xor(dot, o, 64);
                ss += __shfl_xor(ss, o, 64);
            }
            const int c = cb + u * GPB;
            if (s == 0 && c < nc) sc[c] = cosine ? dot / (qn * fmaxf(sqrtf(ss), 1e-12f)) : dot;
        }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < nc; c += blockDim.x) {
        const float v = sc[c];
        int rank = 0;
        for (int o = 0; o < nc; ++o) {
            const float w = sc[o];
            rank += (w > v || (w == v && o < c)) ? 1 : 0;
        }
        if (rank < k) {
            out_s[q * k + rank] = v;
            out_p[q * k + rank] = c;
        }
    }
    for (int r = nc + threadIdx.x; r < k; r += blockDim.x) {
        out_s[q * k + r] = -INFINITY;
        out_p[q * k + r] = -1;
    }
}

}  // namespace

int launch_candidate_topk(const float* Q, int64_t nq, int64_t ldq, const float* X, int64_t ni, int64_t ldx, int dim,
                          const int64_t* coff, const int64_t* crow, int max_candidates, int cosine, int k, float* out_s,
                          int64_t* out_p, hipStream_t s) {
    TTAMM_REQUIRE(nq >= 0 && ni >= 0 && dim > 0 && ldq >= dim && ldx >= dim, "candidate_topk: bad shape");
    TTAMM_REQUIRE(k >= 1, "candidate_topk: k must be >= 1");
    TTAMM_REQUIRE(max_candidates >= 0 && max_candidates <= kCandCap, "candidate_topk: at most 4096 candidates per query");
    if (nq == 0) return TTAMM_OK;
    TTAMM_REQUIRE(Q && coff && out_s && out_p && (crow || max_candidates == 0), "candidate_topk: null pointer");
    const bool al = ((uintptr_t)Q | (uintptr_t)X) % 16 == 0 && ldq % 4 == 0 && ldx % 4 == 0;
    const dim3 g((unsigned)nq), t(256);
#define TTAMM_CAND(G, NV) \
    hipLaunchKernelGGL((candidate_topk_v_kernel<G, NV>), g, t, 0, s, Q, ldq, X, ni, ldx, coff, crow, cosine, k, out_s, out_p)
    if (al && dim == 32) TTAMM_CAND(8, 1);
    else if (al && dim == 64) TTAMM_CAND(8, 2);
    else if (al && dim == 96) TTAMM_CAND(8, 3);
    else if (al && dim == 128) TTAMM_CAND(8, 4);
    else if (al && dim == 256) TTAMM_CAND(16, 4);
    else if (al && dim == 512) TTAMM_CAND(16, 8);
    else
        hipLaunchKernelGGL(candidate_topk_kernel, g, t, 0, s, Q, ldq, X, ni, ldx, dim, coff, crow, cosine, k, out_s,
                           out_p);
#undef TTAMM_CAND
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

int launch_normalize_rows(float* x, int64_t n, int dim, int64_t ld, hipStream_t s) {
    TTAMM_REQUIRE(n >= 0 && dim > 0 && ld >= dim, "normalize_rows: bad shape");
    if (n == 0) return TTAMM_OK;
    TTAMM_REQUIRE(x != nullptr, "normalize_rows: null rows");
    hipLaunchKernelGGL(normalize_rows_kernel, dim3((unsigned)ceil_div(n, 4)), dim3(256), 0, s, x, n, dim, ld);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

template <int KS, int IT>
int launch_x(const RetrievalArgs& A, dim3 grid, hipStream_t s) {
    constexpr int lds = 2 * 3 * KS * IT * 32;
    static bool attr_set = false;
    if (!attr_set) {
        TTAMM_HIP(hipFuncSetAttribute((const void*)retrieval_x_kernel<KS, IT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      lds));
        attr_set = true;
    }
    hipLaunchKernelGGL((retrieval_x_kernel<KS, IT>), grid, dim3(kXThreads), lds, s, A);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

template <int KS>
int launch_x_ks(const RetrievalArgs& A, dim3 grid, bool wide, hipStream_t s) {
    if constexpr (KS <= 6) {
        if (wide) return launch_x<KS, 128>(A, grid, s);
    }
    return launch_x<KS, 64>(A, grid, s);
}

// the split-bf16 kernel's query block (dim <= 128), else the fp32 kernel's
bool retrieval_split(int dim) { return dim <= 128 && product_env("TTAMM_RETRIEVAL_FP32") == nullptr; }
int retrieval_qb(int dim) { return retrieval_split(dim) ? kXQ : kRQ; }

size_t retrieval_workspace_bytes(int64_t nq, int64_t ni, int dim, int k) {
    if (nq <= 0 || k <= 0) return 256;
    const int qb = retrieval_qb(dim);
    const int parts = pick_parts(nq, ni, k, qb);
    const int64_t blocks = ((nq + qb - 1) / qb) * parts;
    const size_t buf = (size_t)blocks * qb * kRCap * (sizeof(float) + sizeof(int));
    const size_t part = (size_t)nq * parts * k * (sizeof(float) + sizeof(int));
    return buf + part + 4 * 256;
}

int launch_retrieval_topk(const float* Q, int64_t nq, int64_t ldq, const float* X, int64_t ni, int64_t ldx, int dim,
                          const int64_t* boff, const int64_t* bval, int k, float* out_s, int64_t* out_i, void* ws,
                          size_t ws_bytes, hipStream_t s) {
    TTAMM_REQUIRE(nq >= 0 && ni >= 0, "retrieval: negative sizes");
    TTAMM_REQUIRE(k >= 1 && k <= kRCap - kRI, "retrieval: k must be in [1, 192]");
    TTAMM_REQUIRE(dim > 0 && dim % 8 == 0 && dim <= 256, "retrieval: embedding dim must be a multiple of 8, <= 256");
    TTAMM_REQUIRE(ldq >= dim && ldx >= dim && ldq % 4 == 0 && ldx % 4 == 0 &&
                      ((uintptr_t)Q | (uintptr_t)X) % 16 == 0,
                  "retrieval: rows must be 16-byte aligned (leading dims % 4 == 0)");
    TTAMM_REQUIRE(ni < (int64_t(1) << 31), "retrieval: at most 2^31 - 1 items");
    if (nq == 0) return TTAMM_OK;
    TTAMM_REQUIRE(out_s && out_i, "retrieval: outputs missing");
    TTAMM_REQUIRE(ws_bytes >= retrieval_workspace_bytes(nq, ni, dim, k), "retrieval: workspace too small");
    RetrievalArgs A;
    std::memset(&A, 0, sizeof(A));
    A.Q = Q;
    A.ldq = ldq;
    A.nq = nq;
    A.X = X;
    A.ldx = ldx;
    A.ni = ni;
    A.D = dim;
    A.boff = boff;
    A.bval = bval;
    A.k = k;
    if (const char* e = dev_env("TTAMM_RETRIEVAL_ABLATE")) A.ablate = std::atoi(e);
    const int qb = retrieval_qb(dim);
    A.parts = pick_parts(nq, ni, k, qb);
    A.items_per_part = ni > 0 ? ((ni + A.parts - 1) / A.parts + 127) / 128 * 128 : 0;
    const int64_t qtiles = (nq + qb - 1) / qb;
    const int64_t blocks = qtiles * A.parts;
    char* p = static_cast<char*>(ws);
    auto take = [&](size_t bytes) {
        char* r = p;
        p += (bytes + 255) / 256 * 256;
        return r;
    };
    A.buf_s = reinterpret_cast<float*>(take((size_t)blocks * qb * kRCap * sizeof(float)));
    A.buf_i = reinterpret_cast<int*>(take((size_t)blocks * qb * kRCap * sizeof(int)));
    A.part_s = reinterpret_cast<float*>(take((size_t)nq * A.parts * k * sizeof(float)));
    A.part_i = reinterpret_cast<int*>(take((size_t)nq * A.parts * k * sizeof(int)));
    if (retrieval_split(dim)) {
        const dim3 grid((unsigned)qtiles, (unsigned)A.parts);
        // 128-item tiles (twice the MFMA work per barrier and per load latency) when the candidate
        // buffer (k <= 128) and the LDS (two buffers of 3 x 128 x 16 KS bf16: KS <= 6) allow
        const bool wide = k <= kRCap - 128;
        int rc = TTAMM_OK;
        switch ((dim + 15) / 16) {
            case 1: rc = launch_x_ks<1>(A, grid, wide, s); break;
            case 2: rc = launch_x_ks<2>(A, grid, wide, s); break;
            case 3: rc = launch_x_ks<3>(A, grid, wide, s); break;
            case 4: rc = launch_x_ks<4>(A, grid, wide, s); break;
            case 5: rc = launch_x_ks<5>(A, grid, wide, s); break;
            case 6: rc = launch_x_ks<6>(A, grid, wide, s); break;
            case 7: rc = launch_x_ks<7>(A, grid, wide, s); break;
            default: rc = launch_x_ks<8>(A, grid, wide, s); break;
        }
        if (rc) return rc;
    } else {
        // 128-item tiles (twice the MFMA work per barrier) when the LDS and the buffer allow
        const bool wide = dim <= 128 && k <= kRCap - 128;
        const int IT = wide ? 128 : kRI;
        const size_t lds = (size_t)(kRQ + IT) * (dim + 4) * sizeof(float);
        auto kern = wide ? (const void*)retrieval_partial_kernel<128, 128> : (const void*)retrieval_partial_kernel<64, 256>;
        static bool attr_set[2] = {false, false};
        if (!attr_set[wide]) {
            TTAMM_HIP(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 1024));
            attr_set[wide] = true;
        }
        if (wide)
            hipLaunchKernelGGL((retrieval_partial_kernel<128, 128>), dim3((unsigned)qtiles, (unsigned)A.parts), dim3(256),
                               lds, s, A);
        else
            hipLaunchKernelGGL((retrieval_partial_kernel<64, 256>), dim3((unsigned)qtiles, (unsigned)A.parts), dim3(256),
                               lds, s, A);
        TTAMM_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(retrieval_merge_kernel, dim3((unsigned)nq), dim3(64), 0, s, A, out_s, out_i);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

}  // namespace ttamm
