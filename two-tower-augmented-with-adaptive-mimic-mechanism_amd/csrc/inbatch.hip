// In-batch negatives (ttamm's in-batch mode, BASELINE configs C2/C4; definition in
// oracle/cpu_reference.py train_step(in_batch=True) — not reference behaviour, which scores
// sampled negatives only, training.py:770-798):
//
//   S  = U P^T              [B, Bc]  users x every positive of the (global) batch, fp32 MFMA
//   dS = (sigmoid(S) - Y) / T        Y(b, j) = (j == row_base + b), T = logits in the BCE mean
//   dU = dS P   [B, D]               dP = dS^T U   [Bc, D]        + the BCE sum of S
//
// Nothing B x Bc is stored.  One launch holds two roles over the same code: "user" blocks own
// 128 user rows and a split of the columns (items) and accumulate dU; "item" blocks own 128
// positive rows and a split of the users and accumulate dP, recomputing S^T.  A block's 4 waves
// each keep their 32 rows' operand fragments in registers for the whole launch; the column
// operand streams through LDS in 64-row tiles (double buffered).  Per tile a wave computes its
// 32 x 64 score block (v_mfma_f32_32x32x2_f32, K = D), turns it into dS in registers, parks dS in
// its LDS slice and multiplies it back against the same LDS tile (K = 64).  Blocks write
// partial rows to slabs that ib_reduce_kernel sums in split order (deterministic).
#include <algorithm>

#include "kernels.h"

namespace ttamm {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kIbRows = 128;  // rows per block (4 waves x 32)
constexpr int kIbTile = 64;   // column tile
constexpr int kIbDsLd = kIbTile + 4;

__device__ __forceinline__ float ib_bce(float x, float y) {  // ATen BCEWithLogits term (rows.hip bce_logit)
    const float m = fmaxf(-x, 0.f);
    return (1.0f - y) * x + m + logf(expf(-m) + expf(-x - m));
}
__device__ __forceinline__ float f4at(const float4& v, int q) { return q == 0 ? v.x : q == 1 ? v.y : q == 2 ? v.z : v.w; }

template <int DP>
__global__ __launch_bounds__(256) void inbatch_kernel(InBatchArgs A) {
    constexpr int NB = DP / 32;   // 32-wide output column blocks
    constexpr int G = DP / 8;     // k groups of the score product (a lane reads 4 of each 8)
    constexpr int SD = DP + 4;    // LDS row stride of the column tile
    constexpr int TF4 = kIbTile * DP / 4;
    constexpr int LOADS = (TF4 + 255) / 256;
    __shared__ __attribute__((aligned(16))) float ct[2][kIbTile * SD];
    __shared__ __attribute__((aligned(16))) float dsb[4][32 * kIbDsLd];
    __shared__ float red[4];

    int blk = blockIdx.x;
    const int nu = A.rblk_u * A.splits_u;
    const bool role_u = blk < nu;
    if (!role_u) blk -= nu;
    const int splits = role_u ? A.splits_u : A.splits_p;
    const int rb = blk / splits, sp = blk - (blk / splits) * splits;
    const float* R = role_u ? A.U : A.P;
    const int64_t ldr = role_u ? A.ldu : A.ldp, nr = role_u ? A.B : A.Bc;
    const float* C = role_u ? A.P : A.U;
    const int64_t ldc = role_u ? A.ldp : A.ldu, nc = role_u ? A.Bc : A.B;
    const int64_t per = role_u ? A.cols_u : A.cols_p;
    const int64_t c_begin = min(nc, (int64_t)sp * per), c_end = min(nc, c_begin + per);
    const int D = A.D;

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 31, h = lane >> 5;
    const int64_t r0 = (int64_t)rb * kIbRows + 32 * w;

    // this lane's row fragments: R[r0 + li][8g + 4h .. +3], zero past D / nr
    float4 rf[G];
    {
        const int64_t row = r0 + li;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int col = 8 * g + 4 * h;
            rf[g] = (row < nr && col < D) ? *reinterpret_cast<const float4*>(R + row * ldr + col)
                                          : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    f32x16 acc[NB];
#pragma unroll
    for (int n = 0; n < NB; ++n)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[n][r] = 0.f;
    float bce = 0.f;

    // column tile -> registers (zero past c_end / D, so masked rows contribute exact zeros)
    float4 st[LOADS];
    auto load = [&](int64_t c0) {
#pragma unroll
        for (int it = 0; it < LOADS; ++it) {
            const int lin = tid + it * 256;
            const int row = lin / (DP / 4), col = (lin - row * (DP / 4)) * 4;
            const int64_t gc = c0 + row;
            st[it] = (lin < TF4 && gc < c_end && col < D) ? *reinterpret_cast<const float4*>(C + gc * ldc + col)
                                                          : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int it = 0; it < LOADS; ++it) {
            const int lin = tid + it * 256;
            if (lin >= TF4) continue;
            const int row = lin / (DP / 4), col = (lin - row * (DP / 4)) * 4;
            *reinterpret_cast<float4*>(&ct[buf][row * SD + col]) = st[it];
        }
    };

    const int ntiles = c_end > c_begin ? (int)((c_end - c_begin + kIbTile - 1) / kIbTile) : 0;
    if (ntiles > 0) {
        load(c_begin);
        store(0);
    }
    __syncthreads();
    float* my_ds = dsb[w];
    for (int t = 0; t < ntiles; ++t) {
        const int buf = t & 1;
        const int64_t c0 = c_begin + (int64_t)t * kIbTile;
        if (t + 1 < ntiles) load(c0 + kIbTile);  // in flight during this tile's MFMAs
        const float* tile = ct[buf];
        // ---- S block: 32 rows x 64 columns, K = DP --------------------------------------------
        f32x16 s[2];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) s[j][r] = 0.f;
#pragma unroll
        for (int g = 0; g < G; ++g) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const float4 b = *reinterpret_cast<const float4*>(tile + (32 * j + li) * SD + 8 * g + 4 * h);
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    s[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4at(rf[g], q), f4at(b, q), s[j], 0, 0, 0);
            }
        }
        // ---- dS in registers -> this wave's LDS slice ------------------------------------------
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int lr = (r & 3) + 8 * (r >> 2) + 4 * h;
                const int64_t gr = r0 + lr, gc = c0 + 32 * j + li;
                const bool ok = gr < nr && gc < c_end;
                const int64_t gu = role_u ? gr : gc, gi = role_u ? gc : gr;  // user row, positive column
                const float y = (gi == A.row_base + gu) ? 1.0f : 0.0f;
                const float x = s[j][r];
                const float d = ok ? (1.0f / (1.0f + expf(-x)) - y) * A.inv_T : 0.f;
                if (role_u && ok) bce += ib_bce(x, y);
                my_ds[lr * kIbDsLd + 32 * j + li] = d;
            }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the slice is written
        __builtin_amdgcn_wave_barrier();
        // ---- rows' gradient += dS . tile, K = 64 -----------------------------------------------
#pragma unroll
        for (int g = 0; g < kIbTile / 8; ++g) {
            const float4 a = *reinterpret_cast<const float4*>(my_ds + li * kIbDsLd + 8 * g + 4 * h);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float* brow = tile + (8 * g + 4 * h + q) * SD + li;
#pragma unroll
                for (int n = 0; n < NB; ++n)
                    acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4at(a, q), brow[32 * n], acc[n], 0, 0, 0);
            }
        }
        // the other buffer was last read in tile t - 1, before that tile's barrier
        if (t + 1 < ntiles) store(buf ^ 1);
        __syncthreads();
    }
    // ---- partial rows -> this split's slab ------------------------------------------------------
    float* slab = role_u ? A.slab_u + (int64_t)sp * A.B * D : A.slab_p + (int64_t)sp * A.Bc * D;
#pragma unroll
    for (int n = 0; n < NB; ++n)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int lr = (r & 3) + 8 * (r >> 2) + 4 * h;
            const int64_t gr = r0 + lr;
            const int col = 32 * n + li;
            if (gr < nr && col < D) slab[gr * D + col] = acc[n][r];
        }
    if (role_u) {
        bce = wave_sum(bce);
        if (lane == 0) red[w] = bce;
        __syncthreads();
        if (tid == 0) A.loss_part[blk] = (red[0] + red[1]) + (red[2] + red[3]);
    }
}

// dU = sum of the user slabs, dP = sum of the item slabs, in split order.
__global__ void ib_reduce_kernel(InBatchArgs A) {
    const int64_t nu = A.B * A.D, total = nu + A.Bc * A.D;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const bool u = i < nu;
        const int64_t e = u ? i : i - nu;
        const int64_t r = e / A.D;
        const int c = (int)(e - r * A.D);
        const float* slab = u ? A.slab_u : A.slab_p;
        const int64_t plane = (u ? A.B : A.Bc) * A.D;
        const int splits = u ? A.splits_u : A.splits_p;
        float s = 0.f;
        for (int k = 0; k < splits; ++k) s += slab[k * plane + e];
        if (u) A.dU[r * A.ld_du + c] = s;
        else A.dP[r * A.ld_dp + c] = s;
    }
}

}  // namespace

void inbatch_plan(int64_t B, int64_t Bc, InBatchArgs& a) {
    a.rblk_u = (int)ceil_div(B, kIbRows);
    a.rblk_p = (int)ceil_div(Bc, kIbRows);
    // ~4 blocks per CU over both roles: split the columns so each role has >= ~512 blocks
    const int64_t want = 512;
    a.splits_u = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(Bc, kIbTile), ceil_div(want, a.rblk_u)));
    a.splits_p = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(B, kIbTile), ceil_div(want, a.rblk_p)));
    a.cols_u = ceil_div(ceil_div(Bc, a.splits_u), kIbTile) * kIbTile;
    a.cols_p = ceil_div(ceil_div(B, a.splits_p), kIbTile) * kIbTile;
    a.splits_u = (int)std::max<int64_t>(1, ceil_div(Bc, a.cols_u));
    a.splits_p = (int)std::max<int64_t>(1, ceil_div(B, a.cols_p));
}

size_t inbatch_workspace_floats(int64_t B, int64_t Bc, int D, size_t* slab_u, size_t* slab_p, size_t* parts) {
    InBatchArgs a{};
    inbatch_plan(B, Bc, a);
    *slab_u = (size_t)a.splits_u * B * D;
    *slab_p = (size_t)a.splits_p * Bc * D;
    *parts = (size_t)a.rblk_u * a.splits_u;
    return *slab_u + *slab_p + *parts;
}

int launch_inbatch(InBatchArgs& a, hipStream_t s) {
    TTAMM_REQUIRE(a.D > 0 && a.D % 4 == 0 && a.D <= 128, "in-batch negatives: embedding dim must be a multiple of 4, <= 128");
    TTAMM_REQUIRE(a.B > 0 && a.Bc > 0 && a.B < (int64_t(1) << 31) && a.Bc < (int64_t(1) << 31), "in-batch: bad batch");
    TTAMM_REQUIRE(a.ldu % 4 == 0 && a.ldp % 4 == 0 && ((uintptr_t)a.U | (uintptr_t)a.P) % 16 == 0,
                  "in-batch: rows must be 16-byte aligned");
    inbatch_plan(a.B, a.Bc, a);
    const unsigned blocks = (unsigned)(a.rblk_u * a.splits_u + a.rblk_p * a.splits_p);
    const int dp = (a.D + 31) / 32 * 32;
    switch (dp) {
        case 32: hipLaunchKernelGGL(inbatch_kernel<32>, dim3(blocks), dim3(256), 0, s, a); break;
        case 64: hipLaunchKernelGGL(inbatch_kernel<64>, dim3(blocks), dim3(256), 0, s, a); break;
        case 96: hipLaunchKernelGGL(inbatch_kernel<96>, dim3(blocks), dim3(256), 0, s, a); break;
        default: hipLaunchKernelGGL(inbatch_kernel<128>, dim3(blocks), dim3(256), 0, s, a); break;
    }
    TTAMM_LAUNCH_CHECK();
    const int64_t total = (a.B + a.Bc) * a.D;
    hipLaunchKernelGGL(ib_reduce_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(total, 256), 8192)), dim3(256), 0, s,
                       a);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

}  // namespace ttamm
