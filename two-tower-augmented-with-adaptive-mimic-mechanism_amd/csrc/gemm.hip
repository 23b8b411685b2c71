// fp32 MFMA GEMMs for the tower MLP and fusion gate (gfx950).
//
// Forward / data-gradient kernel:  C[M,N] = epilogue( A[M,K] . op(B) )
//   - A rows may be gathered by an int64 index (feature rows by user/item id,
//     training.py:741-747,775) so the gathered [rows, F] matrix is never materialised.
//   - B is either an nn.Linear weight [N,K] (forward, y = x W^T) or [K,N] (dgrad, dX = dY W).
//   - Epilogues fuse bias, ReLU, Dropout, Sigmoid gate mixing and the adaptive-mimic
//     augmentation (encoders.py:126-168, adaptive_mimic.py:88-95).
// Weight-gradient kernel:  dW[m,n] = sum_r dY[r,m] X[r,n], split over row chunks, with the
//   bias gradient riding along as an implicit all-ones column n == N; partial slabs are
//   summed in a fixed order (deterministic).
//
// Matrix core: v_mfma_f32_32x32x2_f32 (exact fp32, one fma per product).  Each lane of a
// wave supplies one A and one B value per instruction; lane half h = lane>>5 owns k-slot h.
// Within a 16-deep k-tile, lane half h walks k = 8h .. 8h+7, so its A/B fragments for four
// consecutive MFMAs are one contiguous float4 in LDS (ds_read_b128).
#include "kernels.h"

namespace ttamm {

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

// Kernel-argument (constant address space) view of a struct.
#define KArg(T) __attribute__((address_space(4))) T

constexpr int BK = 16;
constexpr int SK = BK + 4;  // LDS row stride (floats): 80 B rows keep ds_read_b128 conflict-free
constexpr int kThreads = 256;

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }

__device__ __forceinline__ bool aligned16(const void* p) {
    return (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
}

// Load 4 consecutive k elements of row `rp` starting at k (masked by K).
__device__ __forceinline__ float4 load4_k(const float* rp, int k, int K, bool vec) {
    if (rp == nullptr) return make_float4(0.f, 0.f, 0.f, 0.f);
    if (vec && k + 3 < K) return *reinterpret_cast<const float4*>(rp + k);
    float4 v;
    v.x = (k + 0 < K) ? rp[k + 0] : 0.f;
    v.y = (k + 1 < K) ? rp[k + 1] : 0.f;
    v.z = (k + 2 < K) ? rp[k + 2] : 0.f;
    v.w = (k + 3 < K) ? rp[k + 3] : 0.f;
    return v;
}

template <int BM, int BN, int WAVES_M, int WAVES_N>
struct GemmCfg {
    static constexpr int TM = BM / WAVES_M;
    static constexpr int TN = BN / WAVES_N;
    static constexpr int I = TM / 32;
    static constexpr int J = TN / 32;
    static constexpr int A_LOADS = (BM * 4 + kThreads - 1) / kThreads;
    static constexpr int B_LOADS = (BN * 4 + kThreads - 1) / kThreads;
    static_assert(WAVES_M * WAVES_N == 4, "4 waves per block");
    static_assert(TM % 32 == 0 && TN % 32 == 0, "wave tile must be a multiple of 32");
};

__device__ __forceinline__ uint32_t keep_threshold(float keep_prob) {
    double t = (double)keep_prob * 4294967296.0;
    return t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
}

// Epilogue for one MFMA accumulator set.  acc[i][j] register r of lane (li, h) holds
// C[row = i*32 + (r&3) + 8*(r>>2) + 4h][col = j*32 + li] of the wave tile.
template <int E, int I, int J, int TM, int TN, int WAVES_N>
__device__ __forceinline__ void epilogue(const KArg(GemmProblem) & P, f32x16 (&acc)[I][J], int m0, int n0, int wm,
                                         int wn, int li, int h) {
    const int M = P.M, N = P.N;
    const bool use_rng = (E == EPI_HIDDEN) && P.keep_mask == nullptr && P.keep_prob < 1.0f;
    const uint32_t thresh = keep_threshold(P.keep_prob);
#pragma unroll
    for (int i = 0; i < I; ++i) {
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const int col = n0 + wn * TN + j * 32 + li;
            const bool col_ok = col < N;
            float bias = 0.f;
            if (E == EPI_STORE || E == EPI_HIDDEN || E == EPI_GATE_HIDDEN || E == EPI_GATE_OUT)
                if (P.bias && col_ok) bias = P.bias[col];
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4) {
                const int rbase = m0 + wm * TM + i * 32 + 8 * g4 + 4 * h;
                u32x4 rnd = {0u, 0u, 0u, 0u};
                if (use_rng)
                    rnd = philox4x32(u32x4{(uint32_t)rbase, (uint32_t)col, P.rng_c2, P.rng_c3}, P.rng_k0, P.rng_k1);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int row = rbase + e;
                    float v = acc[i][j][4 * g4 + e];
                    if (row < M && col_ok) {
                        const int64_t off = (int64_t)row * P.ldc + col;
                        if (E == EPI_STORE) {
                            P.C[off] = v + bias;
                        } else if (E == EPI_HIDDEN) {
                            v = v + bias;
                            v = v > 0.f ? v : 0.f;
                            if (P.keep_prob < 1.0f) {
                                bool keep;
                                if (P.keep_mask) {
                                    keep = P.keep_mask[(int64_t)row * N + col] != 0;
                                } else {
                                    const uint32_t w = e == 0 ? rnd.x : e == 1 ? rnd.y : e == 2 ? rnd.z : rnd.w;
                                    keep = w < thresh;
                                }
                                v = v * (keep ? P.inv_keep : 0.f);
                            }
                            P.C[off] = v;
                        } else if (E == EPI_GATE_HIDDEN) {
                            v = v + bias;
                            P.C[off] = v > 0.f ? v : 0.f;
                        } else if (E == EPI_GATE_OUT) {
                            v = v + bias;
                            const float g = sigmoidf_(v);
                            const float* efr = P.aux0 + (int64_t)row * P.ld_aux0;
                            const float ev = efr[col], fv = efr[N + col];
                            const float t = g * ev + (1.0f - g) * fv;
                            const int64_t oo = (int64_t)row * P.ld_out + col;
                            P.out1[oo] = g;
                            P.out2[oo] = t;
                            float aug = t;
                            if (P.table) {
                                const float a = P.table[P.idx[row] * (int64_t)N + col];
                                P.out3[oo] = a;
                                aug = t + a;
                            }
                            P.C[off] = aug;
                        } else if (E == EPI_DGRAD_RELU) {
                            const float z = P.aux0[(int64_t)row * P.ld_aux0 + col];
                            P.C[off] = z > 0.f ? v : 0.f;
                        } else if (E == EPI_DGRAD_GATE_EF) {
                            const int D = N >> 1;
                            const int c = col < D ? col : col - D;
                            const float dt = P.aux1[(int64_t)row * P.ld_aux1 + c];
                            const float g = P.aux2[(int64_t)row * P.ld_aux1 + c];
                            P.C[off] = col < D ? v + dt * g : v + dt * (1.0f - g);
                        } else if (E == EPI_DGRAD_HIDDEN) {
                            const float hv = P.aux0[(int64_t)row * P.ld_aux0 + col];
                            P.C[off] = hv > 0.f ? v * P.inv_keep : 0.f;
                        }
                    }
                }
            }
        }
    }
}

template <int BM, int BN, int WAVES_M, int WAVES_N>
__global__ __launch_bounds__(kThreads) void gemm_kernel(GemmBatch batch) {
    using Cfg = GemmCfg<BM, BN, WAVES_M, WAVES_N>;
    constexpr int I = Cfg::I, J = Cfg::J, TM = Cfg::TM, TN = Cfg::TN;

    __shared__ __attribute__((aligned(16))) float As[2][BM][SK];
    __shared__ __attribute__((aligned(16))) float Bs[2][BN][SK];

    // ---- locate problem / tile --------------------------------------------------------
    // The problem table is read straight from the kernarg segment with a wave-uniform index
    // (scalar loads); indexing the by-value argument would copy it to scratch.
    const KArg(GemmBatch)* kb = (const KArg(GemmBatch)*)(__builtin_amdgcn_kernarg_segment_ptr());
    int tile = blockIdx.x;
    int pi = 0;
    if (kb->count > 1 && tile >= kb->p[1].tile_begin) pi = 1;
    const KArg(GemmProblem)& P = kb->p[pi];
    tile -= P.tile_begin;
    const int tm = tile / P.tiles_n, tn = tile - tm * P.tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const int M = P.M, N = P.N, K = P.K;

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    const int li = lane & 31, h = lane >> 5;

    const bool a_vec = (P.lda % 4 == 0) && aligned16(P.A);
    const bool b_vec = (P.ldb % 4 == 0) && aligned16(P.B);

    // ---- per-thread A row pointers (gather resolved once) -----------------------------
    const float* a_rp[Cfg::A_LOADS];
    int a_row[Cfg::A_LOADS], a_c4[Cfg::A_LOADS];
#pragma unroll
    for (int it = 0; it < Cfg::A_LOADS; ++it) {
        const int lin = tid + it * kThreads;
        a_row[it] = lin >> 2;
        a_c4[it] = lin & 3;
        const int gr = m0 + a_row[it];
        a_rp[it] = nullptr;
        if (lin < BM * 4 && gr < M) {
            const int64_t src = P.a_idx ? P.a_idx[gr] : (int64_t)gr;
            a_rp[it] = P.A + src * P.lda;
        }
    }

    float4 ra[Cfg::A_LOADS];
    float4 rb[Cfg::B_LOADS];

    auto load_tile = [&](int k0) {
#pragma unroll
        for (int it = 0; it < Cfg::A_LOADS; ++it) ra[it] = load4_k(a_rp[it], k0 + a_c4[it] * 4, K, a_vec);
#pragma unroll
        for (int it = 0; it < Cfg::B_LOADS; ++it) {
            const int lin = tid + it * kThreads;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (lin < BN * 4) {
                if (!P.b_kn) {
                    const int n = n0 + (lin >> 2), k = k0 + (lin & 3) * 4;
                    if (n < N) v = load4_k(P.B + (int64_t)n * P.ldb, k, K, b_vec);
                } else {
                    constexpr int NV = BN / 4;
                    const int kr = lin / NV, nv = lin - kr * NV;
                    const int k = k0 + kr, n = n0 + nv * 4;
                    if (k < K) v = load4_k(P.B + (int64_t)k * P.ldb, n, N, b_vec);
                }
            }
            rb[it] = v;
        }
    };
    auto store_tile = [&](int buf) {
#pragma unroll
        for (int it = 0; it < Cfg::A_LOADS; ++it) {
            const int lin = tid + it * kThreads;
            if (lin < BM * 4) *reinterpret_cast<float4*>(&As[buf][a_row[it]][a_c4[it] * 4]) = ra[it];
        }
#pragma unroll
        for (int it = 0; it < Cfg::B_LOADS; ++it) {
            const int lin = tid + it * kThreads;
            if (lin < BN * 4) {
                if (!P.b_kn) {
                    *reinterpret_cast<float4*>(&Bs[buf][lin >> 2][(lin & 3) * 4]) = rb[it];
                } else {
                    constexpr int NV = BN / 4;
                    const int kr = lin / NV, nv = lin - kr * NV;
                    Bs[buf][nv * 4 + 0][kr] = rb[it].x;
                    Bs[buf][nv * 4 + 1][kr] = rb[it].y;
                    Bs[buf][nv * 4 + 2][kr] = rb[it].z;
                    Bs[buf][nv * 4 + 3][kr] = rb[it].w;
                }
            }
        }
    };

    f32x16 acc[I][J];
#pragma unroll
    for (int i = 0; i < I; ++i)
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int nk = (K + BK - 1) / BK;
    load_tile(0);
    store_tile(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) load_tile((kt + 1) * BK);
#pragma unroll
        for (int s4 = 0; s4 < 2; ++s4) {
            float4 af[I], bf[J];
#pragma unroll
            for (int i = 0; i < I; ++i)
                af[i] = *reinterpret_cast<const float4*>(&As[buf][wm * TM + i * 32 + li][8 * h + 4 * s4]);
#pragma unroll
            for (int j = 0; j < J; ++j)
                bf[j] = *reinterpret_cast<const float4*>(&Bs[buf][wn * TN + j * 32 + li][8 * h + 4 * s4]);
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int i = 0; i < I; ++i)
#pragma unroll
                    for (int j = 0; j < J; ++j) {
                        const float a = q == 0 ? af[i].x : q == 1 ? af[i].y : q == 2 ? af[i].z : af[i].w;
                        const float b = q == 0 ? bf[j].x : q == 1 ? bf[j].y : q == 2 ? bf[j].z : bf[j].w;
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i][j], 0, 0, 0);
                    }
        }
        if (kt + 1 < nk) store_tile(buf ^ 1);
        __syncthreads();
    }

    // ---- epilogue (dispatched once; each variant fully unrolled so acc stays in registers)
    switch (P.epi) {
        case EPI_STORE: epilogue<EPI_STORE, I, J, TM, TN, WAVES_N>(P, acc, m0, n0, wm, wn, li, h); break;
        case EPI_HIDDEN: epilogue<EPI_HIDDEN, I, J, TM, TN, WAVES_N>(P, acc, m0, n0, wm, wn, li, h); break;
        case EPI_GATE_HIDDEN: epilogue<EPI_GATE_HIDDEN, I, J, TM, TN, WAVES_N>(P, acc, m0, n0, wm, wn, li, h); break;
        case EPI_GATE_OUT: epilogue<EPI_GATE_OUT, I, J, TM, TN, WAVES_N>(P, acc, m0, n0, wm, wn, li, h); break;
        case EPI_DGRAD_RELU: epilogue<EPI_DGRAD_RELU, I, J, TM, TN, WAVES_N>(P, acc, m0, n0, wm, wn, li, h); break;
        case EPI_DGRAD_GATE_EF:
            epilogue<EPI_DGRAD_GATE_EF, I, J, TM, TN, WAVES_N>(P, acc, m0, n0, wm, wn, li, h);
            break;
        case EPI_DGRAD_HIDDEN: epilogue<EPI_DGRAD_HIDDEN, I, J, TM, TN, WAVES_N>(P, acc, m0, n0, wm, wn, li, h); break;
        default: break;
    }
}

// ---------------------------------------------------------------------------------------
// Weight gradient: per block a 64x64 tile of dW (+ bias column) over one chunk of rows.
// ---------------------------------------------------------------------------------------
constexpr int WBM = 64, WBN = 64, WBK = 16;

__global__ __launch_bounds__(kThreads) void wgrad_kernel(WgradBatch batch) {
    __shared__ __attribute__((aligned(16))) float Ys[2][WBK][WBM];
    __shared__ __attribute__((aligned(16))) float Xs[2][WBK][WBN];

    const KArg(WgradBatch)* kb = (const KArg(WgradBatch)*)(__builtin_amdgcn_kernarg_segment_ptr());
    int blk = blockIdx.x;
    int pi = 0;
#pragma unroll 1
    for (int q = 1; q < kb->count; ++q)
        if (blk >= kb->p[q].tile_begin) pi = q;
    const KArg(WgradProblem)& P = kb->p[pi];
    blk -= P.tile_begin;
    const int tiles = P.tiles_m * P.tiles_n;
    const int split = blk / tiles;
    const int t2 = blk - split * tiles;
    const int tm = t2 / P.tiles_n, tn = t2 - tm * P.tiles_n;
    const int m0 = tm * WBM, n0 = tn * WBN;
    const int r0 = split * P.rows_per_split;
    const int r1 = min(P.R, r0 + P.rows_per_split);
    const int M = P.M, NN = P.N + 1;  // implicit ones column at n == N

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int li = lane & 31, h = lane >> 5;

    const bool y_vec = (P.ld_dy % 4 == 0) && aligned16(P.dY);
    const bool x_vec = (P.ld_x % 4 == 0) && aligned16(P.X);

    // thread -> (row in k-tile, float4 column)
    const int lr = tid >> 4, lc = (tid & 15) * 4;
    float4 ry, rx;

    auto load_tile = [&](int rr) {
        const int r = rr + lr;
        ry = make_float4(0.f, 0.f, 0.f, 0.f);
        rx = make_float4(0.f, 0.f, 0.f, 0.f);
        if (r < r1) {
            const float* yp = P.dY + (int64_t)r * P.ld_dy;
            ry = load4_k(yp, m0 + lc, M, y_vec);
            const int64_t src = P.x_idx ? P.x_idx[r] : (int64_t)r;
            const float* xp = P.X + src * P.ld_x;
            const int n = n0 + lc;
            if (x_vec && n + 3 < P.N) {
                rx = *reinterpret_cast<const float4*>(xp + n);
            } else {
                float t[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int ne = n + e;
                    t[e] = ne < P.N ? xp[ne] : (ne == P.N ? 1.0f : 0.f);
                }
                rx = make_float4(t[0], t[1], t[2], t[3]);
            }
        }
    };
    auto store_tile = [&](int buf) {
        *reinterpret_cast<float4*>(&Ys[buf][lr][lc]) = ry;
        *reinterpret_cast<float4*>(&Xs[buf][lr][lc]) = rx;
    };

    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;

    const int nk = (r1 - r0 + WBK - 1) / WBK;
    if (nk > 0) {
        load_tile(r0);
        store_tile(0);
    }
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) load_tile(r0 + (kt + 1) * WBK);
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const float a = Ys[buf][8 * h + s][wm * 32 + li];
            const float b = Xs[buf][8 * h + s][wn * 32 + li];
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
        }
        if (kt + 1 < nk) store_tile(buf ^ 1);
        __syncthreads();
    }

    float* slab = P.slab + (int64_t)split * M * NN;
    const int col = n0 + wn * 32 + li;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row < M && col < NN) slab[(int64_t)row * NN + col] = acc[r];
    }
}

__global__ void wgrad_reduce_kernel(WgradBatch batch, int64_t total) {
    const KArg(WgradBatch)* kb = (const KArg(WgradBatch)*)(__builtin_amdgcn_kernarg_segment_ptr());
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= total) return;
    int64_t off = gid;
    int pi = 0;
    for (; pi < kb->count; ++pi) {
        const int64_t sz = (int64_t)kb->p[pi].M * (kb->p[pi].N + 1);
        if (off < sz) break;
        off -= sz;
    }
    const KArg(WgradProblem)& P = kb->p[pi];
    const int NN = P.N + 1;
    const int64_t plane = (int64_t)P.M * NN;
    float s = 0.f;
    for (int sp = 0; sp < P.splits; ++sp) s += P.slab[sp * plane + off];
    const int m = (int)(off / NN), n = (int)(off - (int64_t)m * NN);
    if (n < P.N) {
        P.grad_w[(int64_t)m * P.N + n] = s;
    } else if (P.grad_b) {
        P.grad_b[m] = s;
    }
}

template <int BM, int BN, int WM, int WN>
int launch_cfg(GemmBatch& b, hipStream_t s) {
    int tiles = 0;
    for (int i = 0; i < b.count; ++i) {
        GemmProblem& p = b.p[i];
        p.tiles_n = (int)ceil_div(p.N, BN);
        p.tile_begin = tiles;
        tiles += (int)ceil_div(p.M, BM) * p.tiles_n;
    }
    b.total_tiles = tiles;
    if (tiles == 0) return TTAMM_OK;
    hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN>), dim3(tiles), dim3(kThreads), 0, s, b);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

}  // namespace

int launch_gemm(GemmBatch& b, hipStream_t s) {
    int maxN = 0;
    for (int i = 0; i < b.count; ++i) {
        const GemmProblem& p = b.p[i];
        TTAMM_REQUIRE(p.M >= 0 && p.N > 0 && p.K > 0, "gemm: bad shape");
        maxN = p.N > maxN ? p.N : maxN;
    }
    if (maxN > 96) return launch_cfg<128, 192, 2, 2>(b, s);
    return launch_cfg<128, 96, 4, 1>(b, s);
}

int wgrad_rows_per_split(int R) {
    (void)R;
    return 512;
}

size_t wgrad_slab_floats(int R, int M, int N) {
    const int rps = wgrad_rows_per_split(R);
    const int splits = R > 0 ? (int)ceil_div(R, rps) : 1;
    return (size_t)splits * M * (N + 1);
}

int launch_wgrad(WgradBatch& b, hipStream_t s) {
    int blocks = 0;
    int64_t total = 0;
    for (int i = 0; i < b.count; ++i) {
        WgradProblem& p = b.p[i];
        p.rows_per_split = wgrad_rows_per_split(p.R);
        p.splits = p.R > 0 ? (int)ceil_div(p.R, p.rows_per_split) : 1;
        p.tiles_m = (int)ceil_div(p.M, WBM);
        p.tiles_n = (int)ceil_div(p.N + 1, WBN);
        p.tile_begin = blocks;
        blocks += p.splits * p.tiles_m * p.tiles_n;
        total += (int64_t)p.M * (p.N + 1);
    }
    b.total_blocks = blocks;
    if (blocks == 0) return TTAMM_OK;
    hipLaunchKernelGGL(wgrad_kernel, dim3(blocks), dim3(kThreads), 0, s, b);
    TTAMM_LAUNCH_CHECK();
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)ceil_div(total, 256)), dim3(256), 0, s, b, total);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

}  // namespace ttamm
