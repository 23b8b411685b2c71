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
// the query's running threshold (the k-th best so far) and the item is not blocked; a wave
// compacts a query's buffer (bitonic sort in registers, keep k) before it could overflow.
// Pass 2 (retrieval_merge_kernel): one wave per query merges the partitions' top-k lists.
#include <cfloat>
#include <cstring>

#include "kernels.h"

namespace ttamm {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kRQ = 64;      // queries per block
constexpr int kRI = 64;      // items per tile
constexpr int kRCap = 256;   // candidate slots per query: k + kRI <= kRCap
constexpr int kMergeJ = 8;   // merge: up to 64 * 8 = 512 candidates per query

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

__device__ __forceinline__ bool is_blocked(const int64_t* __restrict__ vals, int64_t lo, int64_t hi, int64_t item) {
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        const int64_t v = vals[mid];
        if (v == item) return true;
        if (v < item)
            lo = mid + 1;
        else
            hi = mid;
    }
    return false;
}

// Sort query q's buffered candidates, keep the best `keep`, update its threshold.
__device__ void compact_query(float* __restrict__ bs, int* __restrict__ bi, int* cnt, float* tau, int q, int k,
                              float* out_s, int* out_i, int out_k) {
    const int lane = threadIdx.x & 63;
    const int n = cnt[q];
    float s[4];
    int id[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int e = lane * 4 + j;
        s[j] = e < n ? bs[q * kRCap + e] : -INFINITY;
        id[j] = e < n ? bi[q * kRCap + e] : -1;
    }
    wave_bitonic_sort<4>(s, id);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int e = lane * 4 + j;
        if (e < k && e < n) {
            bs[q * kRCap + e] = s[j];
            bi[q * kRCap + e] = id[j];
        }
        if (e == k - 1) tau[q] = e < n ? s[j] : -INFINITY;
        if (out_s && e < out_k) {
            out_s[e] = e < n ? s[j] : -INFINITY;
            out_i[e] = e < n ? id[j] : -1;
        }
    }
    if (lane == 0) cnt[q] = n < k ? n : k;
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
    int64_t blo = 0, bhi = 0;
    if (A.boff && qvalid) {
        blo = A.boff[gq];
        bhi = A.boff[gq + 1];
    }
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
        if (t0 + IT < i_end) load_tile(t0 + IT);
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
        if (qvalid) {
#pragma unroll
            for (int m = 0; m < MT; ++m)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int64_t item = t0 + iw * (IT / 2) + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                    const float sc = acc[m][r];
                    if (item < i_end && sc >= my_tau && !(bhi > blo && is_blocked(A.bval, blo, bhi, item))) {
                        const int slot = atomicAdd(&cnt[myq], 1);
                        bs[myq * kRCap + slot] = sc;  // slot < kRCap: cnt <= kRCap - IT before the tile
                        bi[myq * kRCap + slot] = (int)item;
                    }
                }
        }
        __syncthreads();  // all scores of the tile are in; Xs is free
        for (int q = w; q < kRQ; q += 4)
            if (cnt[q] > kRCap - IT) compact_query(bs, bi, cnt, tau, q, A.k, nullptr, nullptr, 0);
        if (t0 + IT < i_end) store_tile();
    }
    __syncthreads();
    for (int q = w; q < kRQ; q += 4) {
        const int64_t g = q0 + q;
        if (g >= A.nq) continue;
        float* os = A.part_s + (g * A.parts + blockIdx.y) * A.k;
        int* oi = A.part_i + (g * A.parts + blockIdx.y) * A.k;
        compact_query(bs, bi, cnt, tau, q, A.k, os, oi, A.k);
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

int pick_parts(int64_t nq, int64_t ni, int k) {
    const int64_t qtiles = (nq + kRQ - 1) / kRQ;
    int64_t parts = (2048 + qtiles - 1) / qtiles;  // aim for >= 2048 blocks (8 per CU)
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

}  // namespace

int launch_candidate_topk(const float* Q, int64_t nq, int64_t ldq, const float* X, int64_t ni, int64_t ldx, int dim,
                          const int64_t* coff, const int64_t* crow, int max_candidates, int cosine, int k, float* out_s,
                          int64_t* out_p, hipStream_t s) {
    TTAMM_REQUIRE(nq >= 0 && ni >= 0 && dim > 0 && ldq >= dim && ldx >= dim, "candidate_topk: bad shape");
    TTAMM_REQUIRE(k >= 1, "candidate_topk: k must be >= 1");
    TTAMM_REQUIRE(max_candidates >= 0 && max_candidates <= kCandCap, "candidate_topk: at most 4096 candidates per query");
    if (nq == 0) return TTAMM_OK;
    TTAMM_REQUIRE(Q && coff && out_s && out_p && (crow || max_candidates == 0), "candidate_topk: null pointer");
    hipLaunchKernelGGL(candidate_topk_kernel, dim3((unsigned)nq), dim3(256), 0, s, Q, ldq, X, ni, ldx, dim, coff, crow,
                       cosine, k, out_s, out_p);
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

size_t retrieval_workspace_bytes(int64_t nq, int64_t ni, int dim, int k) {
    (void)dim;
    if (nq <= 0 || k <= 0) return 256;
    const int parts = pick_parts(nq, ni, k);
    const int64_t blocks = ((nq + kRQ - 1) / kRQ) * parts;
    const size_t buf = (size_t)blocks * kRQ * kRCap * (sizeof(float) + sizeof(int));
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
    A.parts = pick_parts(nq, ni, k);
    A.items_per_part = ni > 0 ? ((ni + A.parts - 1) / A.parts + 127) / 128 * 128 : 0;
    const int64_t qtiles = (nq + kRQ - 1) / kRQ;
    const int64_t blocks = qtiles * A.parts;
    char* p = static_cast<char*>(ws);
    auto take = [&](size_t bytes) {
        char* r = p;
        p += (bytes + 255) / 256 * 256;
        return r;
    };
    A.buf_s = reinterpret_cast<float*>(take((size_t)blocks * kRQ * kRCap * sizeof(float)));
    A.buf_i = reinterpret_cast<int*>(take((size_t)blocks * kRQ * kRCap * sizeof(int)));
    A.part_s = reinterpret_cast<float*>(take((size_t)nq * A.parts * k * sizeof(float)));
    A.part_i = reinterpret_cast<int*>(take((size_t)nq * A.parts * k * sizeof(int)));
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
    hipLaunchKernelGGL(retrieval_merge_kernel, dim3((unsigned)nq), dim3(64), 0, s, A, out_s, out_i);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

}  // namespace ttamm
