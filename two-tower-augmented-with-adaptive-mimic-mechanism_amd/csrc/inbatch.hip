// In-batch negatives (ttamm's in-batch mode, BASELINE configs C2/C4; definition in
// oracle/cpu_reference.py train_step(in_batch=True) — not reference behaviour, which scores
// sampled negatives only, training.py:770-798):
//
//   S  = U P^T              [B, Bc]  users x every positive of the (global) batch, fp32-accurate MFMA
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
// partial rows to slabs that ib_reduce_kernel sums in split order (deterministic).  This fp32-MFMA
// kernel runs with TTAMM_FP32_MFMA=exact; the default is the split-bf16 inbatch_x_kernel below.
#include <algorithm>
#include <cstdlib>
#include <cstring>

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

// ---- split-bf16 variant (default) ---------------------------------------------------------------
// The same roles, splits and slabs, on v_mfma_f32_32x32x16_bf16: every fp32 operand x is split
// into bf16 planes hi = bf16(x), mid = bf16(x - hi), lo = bf16(x - hi - mid) (RNE, exact
// differences) and a product is formed by six MFMAs (hh, hm, mh, hl, lh, mm; the dropped terms
// are below 2^-24 relative), as in gemm.hip's split kernel: fp32-accurate at 6/16 of the fp32
// MFMA's cycles.
//   Product 1 (per wave, per 64-column tile): S^T[c][u] = C_tile[c][:] . R[u][:]  — the tile as
//     the A operand (row reads), the wave's 32 rows as the B operand (register fragments).  S^T
//     lands with the row u on the lane and the tile column c in registers.
//   dS^T = (sigmoid(S^T) - Y) / T in registers.
//   Product 2: dR[u][:] += sum_c dS^T[c][u] . C_tile[c][:] — dS^T is the A operand straight from
//     its accumulator registers (a 32x32x16 MFMA summing over the accumulator's row index takes
//     it with no lane movement; k order 16s + 8(j>>2) + 4h + (j&3)), the tile the B operand read
//     column-wise with ds_read_b64_tr_b16 in that k order.
// The tile's three planes share one LDS image that serves both the row reads (ds_read_b128) and
// the transposed reads: 256-B rows (128 bf16, columns past D zero and never multiplied) with the
// 16-B chunks XOR-permuted by the row, conflict-free for both.  Single LDS buffer, the next tile
// in flight in registers; two blocks per CU.
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4e_t __attribute__((ext_vector_type(4)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;

constexpr int kIbxRowBytes = 256;                  // LDS image row: 128 bf16
constexpr int kIbxPlane = kIbTile * kIbxRowBytes;  // one plane of a 64-row tile

__device__ __forceinline__ int ibx_off(int row, int ch) {  // byte offset of 16-B chunk ch of row
    return row * kIbxRowBytes + ((ch ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 4);
}
// x -> hi, mid, lo (4 bf16 each)
__device__ __forceinline__ void ibx_split(float4 v, uint2 out[3]) {
    const f32x4e_t x = {v.x, v.y, v.z, v.w};
    const bf16x4_t h = __builtin_convertvector(x, bf16x4_t);
    const f32x4e_t r = x - __builtin_convertvector(h, f32x4e_t);
    const bf16x4_t m = __builtin_convertvector(r, bf16x4_t);
    const f32x4e_t r2 = r - __builtin_convertvector(m, f32x4e_t);
    out[0] = __builtin_bit_cast(uint2, h);
    out[1] = __builtin_bit_cast(uint2, m);
    out[2] = __builtin_bit_cast(uint2, __builtin_convertvector(r2, bf16x4_t));
}
__device__ __forceinline__ bf16x8_t ibx_cat(uint2 a, uint2 b) {
    return __builtin_bit_cast(bf16x8_t, uint4{a.x, a.y, b.x, b.y});
}
// bf16 partial products per fp32 product: 5 (hh, hm, mh, hl, lh; round 6, the default) or, in
// developer measurement builds, 6 (+ mm), 4 (hh hm mh mm) or 3 (hh hm mh).  Measured against the
// chunked float64 definition at the C4 rank-of-8 shape (profiles/r06_inbatch_products.txt):
// 6: dU 9.8e-7, dP 2.9e-6, 3.24 ms; 5: 9.7e-7, 2.9e-6, 2.97 ms; 4: 5.6e-6, 7.3e-6, 2.27 ms;
// 3: 5.7e-6, 7.0e-6, 2.00 ms (bound 1e-5) — mm (<= 2^-18 relative) is below the fp32 noise,
// hl / lh (<= 2^-17 each) are not, so 5 keeps the 6-product accuracy
#ifndef TTAMM_IB_PRODUCTS
#define TTAMM_IB_PRODUCTS 5
#endif
__device__ __forceinline__ f32x16 ibx_mfma6(const bf16x8_t a[3], const bf16x8_t b[3], f32x16 c) {
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], c, 0, 0, 0);
    if constexpr (TTAMM_IB_PRODUCTS == 6 || TTAMM_IB_PRODUCTS == 5) {
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], c, 0, 0, 0);
    }
    if constexpr (TTAMM_IB_PRODUCTS == 6 || TTAMM_IB_PRODUCTS == 4)
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], c, 0, 0, 0);
    return c;
}

// MINB blocks per CU of NW waves (32 rows each); DBUF: two LDS tile buffers (one barrier per
// tile, the next tile split and stored right after this one's MFMAs)
template <int DP, int MINB, int NW, bool DBUF>
__global__ __launch_bounds__(64 * NW, MINB) void inbatch_x_kernel(InBatchArgs A) {
    constexpr int NT = 64 * NW;                      // threads
    constexpr int NB = DP / 32;                      // 32-wide output column blocks
    constexpr int KS = DP / 16;                      // k steps of product 1
    constexpr int TF4 = kIbTile * DP / 4;            // float4 per column tile
    constexpr int LOADS = TF4 / NT;
    static_assert(TF4 % NT == 0, "whole staging rounds");
    __shared__ __attribute__((aligned(16))) unsigned char tiles[DBUF ? 2 : 1][3 * kIbxPlane];
    __shared__ float red[NW];

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
    const int64_t r0 = (int64_t)rb * (32 * NW) + 32 * w;

    // this lane's row fragments (B operand of product 1): R[r0 + li][16 s + 8 h + j], zero past D / nr
    bf16x8_t rf[KS][3];
    {
        const int64_t row = r0 + li;
        const bool rok = row < nr;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int col = 16 * s + 8 * h;
            const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
            const float4 a = (rok && col < D) ? *reinterpret_cast<const float4*>(R + row * ldr + col) : z;
            const float4 b = (rok && col + 4 < D) ? *reinterpret_cast<const float4*>(R + row * ldr + col + 4) : z;
            uint2 pa[3], pb[3];
            ibx_split(a, pa);
            ibx_split(b, pb);
#pragma unroll
            for (int q = 0; q < 3; ++q) rf[s][q] = ibx_cat(pa[q], pb[q]);
        }
    }
    f32x16 acc[NB];
#pragma unroll
    for (int n = 0; n < NB; ++n)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[n][r] = 0.f;
    float bce = 0.f, bce_lin = 0.f, bce_log2 = 0.f;

    // column tile -> registers (zero past c_end / D, so masked rows contribute exact zeros)
    float4 st[LOADS];
    auto load = [&](int64_t c0) {
#pragma unroll
        for (int it = 0; it < LOADS; ++it) {
            const int lin = tid + it * NT;
            const int row = lin / (DP / 4), col = (lin - row * (DP / 4)) * 4;
            const int64_t gc = c0 + row;
            st[it] = (gc < c_end && col < D) ? *reinterpret_cast<const float4*>(C + gc * ldc + col)
                                             : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto store = [&](unsigned char* dst) {
#pragma unroll
        for (int it = 0; it < LOADS; ++it) {
            const int lin = tid + it * NT;
            const int row = lin / (DP / 4), c4 = lin - row * (DP / 4);
            const int o = ibx_off(row, c4 >> 1) + 8 * (c4 & 1);
            uint2 pl[3];
            ibx_split(st[it], pl);
#pragma unroll
            for (int q = 0; q < 3; ++q) *reinterpret_cast<uint2*>(dst + q * kIbxPlane + o) = pl[q];
        }
    };

    const int ntiles = c_end > c_begin ? (int)((c_end - c_begin + kIbTile - 1) / kIbTile) : 0;
    // the next tile in flight in registers while this one is multiplied (narrow D); at D > 64 the
    // registers go to the operands and the second block of the CU hides the load instead
    constexpr bool PREFETCH = DP <= 64 || MINB == 1;
    if (DBUF) {  // tile 0 in buffer 0, tile 1 in flight in registers
        if (ntiles > 0) {
            load(c_begin);
            store(tiles[0]);
            if (ntiles > 1) load(c_begin + kIbTile);
        }
        __syncthreads();
    } else if (PREFETCH && ntiles > 0) {
        load(c_begin);
    }
    // tr-read lane roles: 16-lane group g, lane 4q + p of the group
    const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
    const int64_t gr = r0 + li;
    for (int t = 0; t < ntiles; ++t) {
        const int64_t c0 = c_begin + (int64_t)t * kIbTile;
        unsigned char* const tile = tiles[DBUF ? (t & 1) : 0];
        if (!DBUF) {
            if (!PREFETCH) load(c0);
            __syncthreads();  // every wave is done with the previous tile
            store(tile);
            __syncthreads();
            if (PREFETCH && t + 1 < ntiles) load(c0 + kIbTile);  // in flight during this tile's MFMAs
        }
        // the label Y = 1 sits at tile column diag of this lane's row: user u's own positive is
        // column row_base + u (user role), positive i's user is row i - row_base (item role)
        const int64_t dl = role_u ? A.row_base + gr - c0 : gr - A.row_base - c0;
        const int diag = (dl >= 0 && dl < kIbTile) ? (int)dl : -1;
        const int cols_here = (int)min((int64_t)kIbTile, c_end - c0);
        const bool row_ok = gr < nr;
        // wave-uniform: the whole 32 x 64 block is interior and label-free (most tiles)
        const bool fast = cols_here == kIbTile && __builtin_amdgcn_ballot_w64(diag >= 0 || !row_ok) == 0;
#pragma unroll
        for (int jc = 0; jc < 2; ++jc) {  // tile rows 32 jc .. 32 jc + 31
            // ---- product 1: S^T block [32 c x 32 u] --------------------------------------------------
            f32x16 s2;
#pragma unroll
            for (int r = 0; r < 16; ++r) s2[r] = 0.f;
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const int o = ibx_off(32 * jc + li, 2 * s + h);
                bf16x8_t a[3];
#pragma unroll
                for (int q = 0; q < 3; ++q) a[q] = *reinterpret_cast<const bf16x8_t*>(tile + q * kIbxPlane + o);
                s2 = ibx_mfma6(a, rf[s], s2);
            }
            // ---- dS^T in registers (lane: row u = r0 + li; register r: tile column c) -----------
            // hardware exp2 / log2 / rcp (<= 1-2 ulp): this elementwise pass, not the MFMAs, bounds
            // the kernel with IEEE expf / logf / division.  Sigmoid and the ATen BCE term from one
            // exp: t = exp(-|x|); for x >= 0 exp(-max(-x,0)) = 1 and exp(-x-max(-x,0)) = t, for x < 0
            // the reverse.
            if (fast) {
                // every row and column in range, no label in this wave's block: y = 0, so the BCE
                // term is max(x, 0) + ln(1 + t) (x + max(-x, 0) == max(x, 0) exactly), summed as
                // two lane sums (the log2 terms scaled by ln 2 once at the end)
                if (role_u) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const float x = s2[r];
                        const float tx = __builtin_amdgcn_exp2f(-fabsf(x) * 1.4426950408889634f);
                        const float d1 = 1.0f + tx;
                        const float inv = __builtin_amdgcn_rcpf(d1);
                        const float sg = x >= 0.f ? inv : tx * inv;
                        bce_lin += fmaxf(x, 0.f);
                        bce_log2 += __builtin_amdgcn_logf(d1);
                        s2[r] = sg * A.inv_T;
                    }
                } else {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const float x = s2[r];
                        const float tx = __builtin_amdgcn_exp2f(-fabsf(x) * 1.4426950408889634f);
                        const float inv = __builtin_amdgcn_rcpf(1.0f + tx);
                        const float sg = x >= 0.f ? inv : tx * inv;
                        s2[r] = sg * A.inv_T;
                    }
                }
            } else {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int lc = 32 * jc + (r & 3) + 8 * (r >> 2) + 4 * h;
                    const bool ok = row_ok && lc < cols_here;
                    const float y = lc == diag ? 1.0f : 0.0f;
                    const float x = s2[r];
                    const float tx = __builtin_amdgcn_exp2f(-fabsf(x) * 1.4426950408889634f);
                    const float inv = __builtin_amdgcn_rcpf(1.0f + tx);
                    const float sg = x >= 0.f ? inv : tx * inv;
                    if (role_u && ok) bce += (1.0f - y) * x + fmaxf(-x, 0.f) + __builtin_amdgcn_logf(1.0f + tx) * 0.6931471805599453f;
                    s2[r] = ok ? (sg - y) * A.inv_T : 0.f;
                }
            }
            // ---- product 2: acc[n] (rows u, columns 32 n ..) += dS . tile ---------------------------
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                bf16x8_t a[3];
                {
                    const float4 x0 = make_float4(s2[8 * s + 0], s2[8 * s + 1], s2[8 * s + 2], s2[8 * s + 3]);
                    const float4 x1 = make_float4(s2[8 * s + 4], s2[8 * s + 5], s2[8 * s + 6], s2[8 * s + 7]);
                    uint2 pa[3], pb[3];
                    ibx_split(x0, pa);
                    ibx_split(x1, pb);
#pragma unroll
                    for (int q = 0; q < 3; ++q) a[q] = ibx_cat(pa[q], pb[q]);
                }
                // B: tile rows 32 jc + 16 s + 4 h + q (elements 0..3) and + 8 (elements 4..7)
                const int brow = 32 * jc + 16 * s + 4 * h + q4;
#pragma unroll
                for (int n = 0; n < NB; ++n) {
                    const int ch = 4 * n + 2 * (g & 1) + (p4 >> 1);
                    const int o0 = ibx_off(brow, ch) + 8 * (p4 & 1), o1 = ibx_off(brow + 8, ch) + 8 * (p4 & 1);
                    bf16x8_t b[3];
#pragma unroll
                    for (int q = 0; q < 3; ++q) {
                        const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(tile + q * kIbxPlane + o0));
                        const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(tile + q * kIbxPlane + o1));
                        const s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                        b[q] = __builtin_bit_cast(bf16x8_t, v);
                    }
                    acc[n] = ibx_mfma6(a, b, acc[n]);
                }
            }
        }
        if (DBUF) {
            // tile t + 1 (landed in registers during this tile's MFMAs) into the other buffer, last
            // read in tile t - 1 before that tile's barrier; tile t + 2 in flight
            if (t + 1 < ntiles) {
                store(tiles[(t + 1) & 1]);
                if (t + 2 < ntiles) load(c0 + 2 * kIbTile);
            }
            __syncthreads();
        }
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
        bce = wave_sum(bce + (bce_lin + bce_log2 * 0.6931471805599453f));
        if (lane == 0) red[w] = bce;
        __syncthreads();
        if (tid == 0) {
            float sum = 0.f;
#pragma unroll
            for (int i = 0; i < NW; i += 2) sum += red[i] + red[i + 1];
            A.loss_part[blk] = sum;
        }
    }
}

// ---- software-pipelined variant (default): one wave per SIMD ---------------------------------------
// The split kernel above at two waves per SIMD spills at D = 128 (the row fragments, 96 registers,
// and the dR accumulators, 64, leave too little of a 256-register budget), and its VALU work (the
// sigmoid / BCE pass and the dS splits) only overlaps the MFMAs across the two waves.  Here one
// 256-thread block per CU (one wave per SIMD, up to 512 registers: no spills) runs each role in a
// launch of its own (ROLE_U compile-time: the BCE terms only in the user role's code) and pipelines
// a 64-column tile inside the wave, in one basic block per tile:
//   S1 = P1(cols 0..31);  S2 = P1(cols 32..63)  ||  dS(S1);  P2(S1)  ||  dS(S2);  P2(S2)  ||  next tile -> LDS
// so the 8-cycle-issue MFMAs of one product cover the elementwise VALU of the other half.  The
// column tile is double buffered in LDS (one barrier per tile), the tile after next in flight in
// registers.  Same roles, splits, slabs, operand images and arithmetic as inbatch_x_kernel.
#ifndef IB_VALU_PER_MFMA
#define IB_VALU_PER_MFMA 5
#endif
template <int DP, bool ROLE_U>
__global__ __launch_bounds__(256, 1) void inbatch_p_kernel(InBatchArgs A) {
    constexpr int NB = DP / 32;
    constexpr int KS = DP / 16;
    constexpr int TF4 = kIbTile * DP / 4;
    constexpr int LOADS = TF4 / 256;
    static_assert(TF4 % 256 == 0, "whole staging rounds");
    __shared__ __attribute__((aligned(16))) unsigned char tiles[2][3 * kIbxPlane];
    __shared__ float red[4];

    const int blk = blockIdx.x;
    const int splits = ROLE_U ? A.splits_u : A.splits_p;
    const int rb = blk / splits, sp = blk - (blk / splits) * splits;
    const float* R = ROLE_U ? A.U : A.P;
    const int64_t ldr = ROLE_U ? A.ldu : A.ldp, nr = ROLE_U ? A.B : A.Bc;
    const float* C = ROLE_U ? A.P : A.U;
    const int64_t ldc = ROLE_U ? A.ldp : A.ldu, nc = ROLE_U ? A.Bc : A.B;
    const int64_t per = ROLE_U ? A.cols_u : A.cols_p;
    const int64_t c_begin = min(nc, (int64_t)sp * per), c_end = min(nc, c_begin + per);
    const int D = A.D;
    const float inv_T = A.inv_T;

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 31, h = lane >> 5;
    const int64_t r0 = (int64_t)rb * kIbRows + 32 * w;

    bf16x8_t rf[KS][3];
    {
        const int64_t row = r0 + li;
        const bool rok = row < nr;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int col = 16 * s + 8 * h;
            const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
            const float4 a = (rok && col < D) ? *reinterpret_cast<const float4*>(R + row * ldr + col) : z;
            const float4 b = (rok && col + 4 < D) ? *reinterpret_cast<const float4*>(R + row * ldr + col + 4) : z;
            uint2 pa[3], pb[3];
            ibx_split(a, pa);
            ibx_split(b, pb);
#pragma unroll
            for (int q = 0; q < 3; ++q) rf[s][q] = ibx_cat(pa[q], pb[q]);
        }
    }
    f32x16 acc[NB];
#pragma unroll
    for (int n = 0; n < NB; ++n)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[n][r] = 0.f;
    float bce = 0.f, bce_lin = 0.f, bce_log2 = 0.f;

    float4 st[LOADS];
    auto load = [&](int64_t c0) {
#pragma unroll
        for (int it = 0; it < LOADS; ++it) {
            const int lin = tid + it * 256;
            const int row = lin / (DP / 4), col = (lin - row * (DP / 4)) * 4;
            const int64_t gc = c0 + row;
            st[it] = (gc < c_end && col < D) ? *reinterpret_cast<const float4*>(C + gc * ldc + col)
                                             : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto store = [&](unsigned char* dst) {
#pragma unroll
        for (int it = 0; it < LOADS; ++it) {
            const int lin = tid + it * 256;
            const int row = lin / (DP / 4), c4 = lin - row * (DP / 4);
            const int o = ibx_off(row, c4 >> 1) + 8 * (c4 & 1);
            uint2 pl[3];
            ibx_split(st[it], pl);
#pragma unroll
            for (int q = 0; q < 3; ++q) *reinterpret_cast<uint2*>(dst + q * kIbxPlane + o) = pl[q];
        }
    };
    const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
    const int64_t gr = r0 + li;
    const bool row_ok = gr < nr;

    // product 1: S^T block of tile rows 32 jc .. 32 jc + 31 x this wave's 32 rows
    auto p1 = [&](const unsigned char* tile, int jc) {
        f32x16 s2;
#pragma unroll
        for (int r = 0; r < 16; ++r) s2[r] = 0.f;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int o = ibx_off(32 * jc + li, 2 * s + h);
            bf16x8_t a[3];
#pragma unroll
            for (int q = 0; q < 3; ++q) a[q] = *reinterpret_cast<const bf16x8_t*>(tile + q * kIbxPlane + o);
            s2 = ibx_mfma6(a, rf[s], s2);
        }
        return s2;
    };
    // dS^T in registers: the label-free interior form, or the general one (labels, edges)
    auto ds_general = [&](f32x16& s2, int jc, int diag, int cols_here) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int lc = 32 * jc + (r & 3) + 8 * (r >> 2) + 4 * h;
            const bool ok = row_ok && lc < cols_here;
            const float y = lc == diag ? 1.0f : 0.0f;
            const float x = s2[r];
            const float tx = __builtin_amdgcn_exp2f(-fabsf(x) * 1.4426950408889634f);
            const float inv = __builtin_amdgcn_rcpf(1.0f + tx);
            const float sg = x >= 0.f ? inv : tx * inv;
            if (ROLE_U && ok) bce += (1.0f - y) * x + fmaxf(-x, 0.f) + __builtin_amdgcn_logf(1.0f + tx) * 0.6931471805599453f;
            s2[r] = ok ? (sg - y) * inv_T : 0.f;
        }
    };
    // product 2: acc[n] += dS . tile rows 32 jc ..
    auto p2 = [&](const unsigned char* tile, const f32x16& s2, int jc) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            bf16x8_t a[3];
            {
                const float4 x0 = make_float4(s2[8 * s + 0], s2[8 * s + 1], s2[8 * s + 2], s2[8 * s + 3]);
                const float4 x1 = make_float4(s2[8 * s + 4], s2[8 * s + 5], s2[8 * s + 6], s2[8 * s + 7]);
                uint2 pa[3], pb[3];
                ibx_split(x0, pa);
                ibx_split(x1, pb);
#pragma unroll
                for (int q = 0; q < 3; ++q) a[q] = ibx_cat(pa[q], pb[q]);
            }
            const int brow = 32 * jc + 16 * s + 4 * h + q4;
#pragma unroll
            for (int n = 0; n < NB; ++n) {
                const int ch = 4 * n + 2 * (g & 1) + (p4 >> 1);
                const int o0 = ibx_off(brow, ch) + 8 * (p4 & 1), o1 = ibx_off(brow + 8, ch) + 8 * (p4 & 1);
                bf16x8_t b[3];
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(tile + q * kIbxPlane + o0));
                    const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(tile + q * kIbxPlane + o1));
                    const s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                    b[q] = __builtin_bit_cast(bf16x8_t, v);
                }
                acc[n] = ibx_mfma6(a, b, acc[n]);
            }
        }
    };

    // one element of ds_fast (the interleaved form; same operations)
    auto ds_fast_elem = [&](f32x16& s2, int r) {
        const float x = s2[r];
        const float tx = __builtin_amdgcn_exp2f(-fabsf(x) * 1.4426950408889634f);
        const float d1 = 1.0f + tx;
        const float inv = __builtin_amdgcn_rcpf(d1);
        const float sg = x >= 0.f ? inv : tx * inv;
        if (ROLE_U) {
            bce_lin += fmaxf(x, 0.f);
            bce_log2 += __builtin_amdgcn_logf(d1);
        }
        s2[r] = sg * inv_T;
    };
    // staging round i (of LOADS) of the next tile: its three planes into dst
    auto store_part = [&](unsigned char* dst, int it) {
        if (it >= LOADS) return;
        const int lin = tid + it * 256;
        const int row = lin / (DP / 4), c4 = lin - row * (DP / 4);
        const int o = ibx_off(row, c4 >> 1) + 8 * (c4 & 1);
        uint2 pl[3];
        ibx_split(st[it], pl);
#pragma unroll
        for (int q = 0; q < 3; ++q) *reinterpret_cast<uint2*>(dst + q * kIbxPlane + o) = pl[q];
    };
    // product 2 with side work f(i) after its i-th 6-MFMA group (i = 0 .. 2 NB - 1); the staging
    // rounds past 2 NB (LOADS > 2 NB) run after the last group
    auto split8 = [&](const f32x16& s2, int s, bf16x8_t a[3]) {
        const float4 x0 = make_float4(s2[8 * s + 0], s2[8 * s + 1], s2[8 * s + 2], s2[8 * s + 3]);
        const float4 x1 = make_float4(s2[8 * s + 4], s2[8 * s + 5], s2[8 * s + 6], s2[8 * s + 7]);
        uint2 pa[3], pb[3];
        ibx_split(x0, pa);
        ibx_split(x1, pb);
#pragma unroll
        for (int q = 0; q < 3; ++q) a[q] = ibx_cat(pa[q], pb[q]);
    };
    auto p2_il = [&](const unsigned char* tile, const f32x16& s2, int jc, auto&& f) {
        bf16x8_t aa[2][3];
        split8(s2, 0, aa[0]);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const bf16x8_t* a = aa[s];
            const int brow = 32 * jc + 16 * s + 4 * h + q4;
#pragma unroll
            for (int n = 0; n < NB; ++n) {
                const int ch = 4 * n + 2 * (g & 1) + (p4 >> 1);
                const int o0 = ibx_off(brow, ch) + 8 * (p4 & 1), o1 = ibx_off(brow + 8, ch) + 8 * (p4 & 1);
                bf16x8_t b[3];
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(tile + q * kIbxPlane + o0));
                    const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(tile + q * kIbxPlane + o1));
                    const s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                    b[q] = __builtin_bit_cast(bf16x8_t, v);
                }
                acc[n] = ibx_mfma6(a, b, acc[n]);
                if (s == 0 && n == 0) split8(s2, 1, aa[1]);  // the second half's planes under these MFMAs
                f(s * NB + n);
            }
        }
    };

    const int ntiles = c_end > c_begin ? (int)((c_end - c_begin + kIbTile - 1) / kIbTile) : 0;
    if (ntiles > 0) {
        load(c_begin);
        store(tiles[0]);
        if (ntiles > 1) load(c_begin + kIbTile);
    }
    __syncthreads();
    for (int t = 0; t < ntiles; ++t) {
        const int64_t c0 = c_begin + (int64_t)t * kIbTile;
        const unsigned char* const tile = tiles[t & 1];
        unsigned char* const next = tiles[(t + 1) & 1];
        const bool more = t + 1 < ntiles;
        const int64_t dl = ROLE_U ? A.row_base + gr - c0 : gr - A.row_base - c0;
        const int diag = (dl >= 0 && dl < kIbTile) ? (int)dl : -1;
        const int cols_here = (int)min((int64_t)kIbTile, c_end - c0);
        const bool fast = cols_here == kIbTile && __builtin_amdgcn_ballot_w64(diag >= 0 || !row_ok) == 0;
        // tile t + 1 goes into the other buffer (last read in tile t - 1, before that tile's
        // barrier; after the last tile the store is harmless), tile t + 2 into flight (masked to
        // zeros past the split's columns) — unconditionally, so each body is one basic block
        (void)more;
        if (fast) {
            // written in issue order: every MFMA group of one product carries a slice of the
            // other half's elementwise work
            f32x16 s_a = p1(tile, 0);
            f32x16 s_b;
#pragma unroll
            for (int r = 0; r < 16; ++r) s_b[r] = 0.f;
            // S(cols 32..63) || dS(cols 0..31), two elements per k-step
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const int o = ibx_off(32 + li, 2 * ks + h);
                bf16x8_t a[3];
#pragma unroll
                for (int q = 0; q < 3; ++q) a[q] = *reinterpret_cast<const bf16x8_t*>(tile + q * kIbxPlane + o);
                s_b = ibx_mfma6(a, rf[ks], s_b);
#pragma unroll
                for (int e = (ks * 16) / KS; e < ((ks + 1) * 16) / KS; ++e) ds_fast_elem(s_a, e);
            }
            // dR += dS(cols 0..31) . tile || dS(cols 32..63), 16 / (2 NB) elements per 6-MFMA group
            p2_il(tile, s_a, 0, [&](int i) {
#pragma unroll
                for (int e = (i * 16) / (2 * NB); e < ((i + 1) * 16) / (2 * NB); ++e) ds_fast_elem(s_b, e);
            });
            // dR += dS(cols 32..63) . tile || the next tile's planes into the other buffer
            p2_il(tile, s_b, 1, [&](int i) { store_part(next, i); });
            load(c0 + 2 * kIbTile);
        } else {
            f32x16 s_a = p1(tile, 0);
            f32x16 s_b = p1(tile, 1);
            ds_general(s_a, 0, diag, cols_here);
            p2(tile, s_a, 0);
            ds_general(s_b, 1, diag, cols_here);
            p2(tile, s_b, 1);
            store(next);
            load(c0 + 2 * kIbTile);
        }
        __syncthreads();
    }
    float* slab = ROLE_U ? A.slab_u + (int64_t)sp * A.B * D : A.slab_p + (int64_t)sp * A.Bc * D;
#pragma unroll
    for (int n = 0; n < NB; ++n)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int lr = (r & 3) + 8 * (r >> 2) + 4 * h;
            const int64_t grr = r0 + lr;
            const int col = 32 * n + li;
            if (grr < nr && col < D) slab[grr * D + col] = acc[n][r];
        }
    if (ROLE_U) {
        bce = wave_sum(bce + (bce_lin + bce_log2 * 0.6931471805599453f));
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

// The BCE sum over the user-role blocks' partial sums, in block order (fp64 accumulation):
// the standalone entry's loss (the fused step folds the parts into loss_finalize_kernel).
__global__ void ib_loss_sum_kernel(const float* __restrict__ parts, int n, double* __restrict__ out) {
    __shared__ double red[256];
    double s = 0.0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) s += (double)parts[i];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[0] = red[0];
}

}  // namespace

// Waves per block of the split-bf16 kernel: 4 (128 rows per block, two blocks per CU, one tile
// buffer), or TTAMM_IB_WAVES=8 (256 rows, one block per CU, double-buffered: the column tile staged
// once for twice the rows, but the tile prefetch registers push D = 128 into spills — 9.3 vs
// 3.15 ms at the C4 rank shape, profiles/r04_inbatch_variants.txt); the fp32-MFMA kernel
// (TTAMM_FP32_MFMA=exact) always uses 4.
int inbatch_waves() {
    const char* mf = product_env("TTAMM_FP32_MFMA");
    if (mf && std::strcmp(mf, "exact") == 0) return 4;
    const char* env = dev_env("TTAMM_IB_WAVES");
    return (env && std::atoi(env) == 8) ? 8 : 4;
}

// TTAMM_IB_KERNEL=p: the software-pipelined one-wave-per-SIMD kernel (inbatch_p_kernel), one
// launch per role
bool inbatch_pipelined() {
    const char* mf = product_env("TTAMM_FP32_MFMA");
    if (mf && std::strcmp(mf, "exact") == 0) return false;
    const char* env = dev_env("TTAMM_IB_KERNEL");
    return env && std::strcmp(env, "p") == 0;
}

void inbatch_plan(int64_t B, int64_t Bc, InBatchArgs& a) {
    const int rows = inbatch_pipelined() ? kIbRows : 32 * inbatch_waves();
    a.rblk_u = (int)ceil_div(B, rows);
    a.rblk_p = (int)ceil_div(Bc, rows);
    // ~256 blocks per role (one resident round over both roles at two blocks per CU, each block
    // twice the columns of the former 512: C4 0.952 -> 0.924 ms/step, C2 in-batch 0.658 -> 0.625,
    // the C4 rank-of-8 shape unchanged, profiles/r04_s43_inbatch_blocks.txt); developer knob
    // TTAMM_IB_BLOCKS = blocks per role
    static const int64_t want_env = [] {
        const char* e = dev_env("TTAMM_IB_BLOCKS");
        return e ? (int64_t)std::atoi(e) : (int64_t)0;
    }();
    // (the all-gathered columns of a sharded step, Bc > 2B, keep 512: 3.63 vs 3.74 ms per step at
    // the emulated C4 rank of 8, profiles/r04_s43_inbatch_blocks.txt)
    const int64_t want = want_env > 0 ? want_env : (Bc > 2 * B ? 512 : 256);
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
    // TTAMM_FP32_MFMA=exact: the v_mfma_f32_32x32x2_f32 kernel (as gemm.hip's developer switch)
    const char* env = product_env("TTAMM_FP32_MFMA");
    if (env && std::strcmp(env, "exact") == 0) {
        switch (dp) {
            case 32: hipLaunchKernelGGL(inbatch_kernel<32>, dim3(blocks), dim3(256), 0, s, a); break;
            case 64: hipLaunchKernelGGL(inbatch_kernel<64>, dim3(blocks), dim3(256), 0, s, a); break;
            case 96: hipLaunchKernelGGL(inbatch_kernel<96>, dim3(blocks), dim3(256), 0, s, a); break;
            default: hipLaunchKernelGGL(inbatch_kernel<128>, dim3(blocks), dim3(256), 0, s, a); break;
        }
    } else {
        if (inbatch_pipelined()) {
            const unsigned bu = (unsigned)(a.rblk_u * a.splits_u), bp = (unsigned)(a.rblk_p * a.splits_p);
            switch (dp) {
                case 32:
                    hipLaunchKernelGGL((inbatch_p_kernel<32, true>), dim3(bu), dim3(256), 0, s, a);
                    hipLaunchKernelGGL((inbatch_p_kernel<32, false>), dim3(bp), dim3(256), 0, s, a);
                    break;
                case 64:
                    hipLaunchKernelGGL((inbatch_p_kernel<64, true>), dim3(bu), dim3(256), 0, s, a);
                    hipLaunchKernelGGL((inbatch_p_kernel<64, false>), dim3(bp), dim3(256), 0, s, a);
                    break;
                case 96:
                    hipLaunchKernelGGL((inbatch_p_kernel<96, true>), dim3(bu), dim3(256), 0, s, a);
                    hipLaunchKernelGGL((inbatch_p_kernel<96, false>), dim3(bp), dim3(256), 0, s, a);
                    break;
                default:
                    hipLaunchKernelGGL((inbatch_p_kernel<128, true>), dim3(bu), dim3(256), 0, s, a);
                    hipLaunchKernelGGL((inbatch_p_kernel<128, false>), dim3(bp), dim3(256), 0, s, a);
                    break;
            }
        } else if (inbatch_waves() == 8) {
            switch (dp) {
                case 32: hipLaunchKernelGGL((inbatch_x_kernel<32, 1, 8, true>), dim3(blocks), dim3(512), 0, s, a); break;
                case 64: hipLaunchKernelGGL((inbatch_x_kernel<64, 1, 8, true>), dim3(blocks), dim3(512), 0, s, a); break;
                case 96: hipLaunchKernelGGL((inbatch_x_kernel<96, 1, 8, true>), dim3(blocks), dim3(512), 0, s, a); break;
                default: hipLaunchKernelGGL((inbatch_x_kernel<128, 1, 8, true>), dim3(blocks), dim3(512), 0, s, a); break;
            }
        } else {
            switch (dp) {
                case 32: hipLaunchKernelGGL((inbatch_x_kernel<32, 2, 4, false>), dim3(blocks), dim3(256), 0, s, a); break;
                case 64: hipLaunchKernelGGL((inbatch_x_kernel<64, 2, 4, false>), dim3(blocks), dim3(256), 0, s, a); break;
                case 96: hipLaunchKernelGGL((inbatch_x_kernel<96, 2, 4, false>), dim3(blocks), dim3(256), 0, s, a); break;
                // D = 128 at two blocks per CU spills ~20 registers and still beats one block per CU
                // (C4: 0.41 vs 0.50 ms per launch)
                default: hipLaunchKernelGGL((inbatch_x_kernel<128, 2, 4, false>), dim3(blocks), dim3(256), 0, s, a); break;
            }
        }
    }
    TTAMM_LAUNCH_CHECK();
    const int64_t total = (a.B + a.Bc) * a.D;
    hipLaunchKernelGGL(ib_reduce_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(total, 256), 8192)), dim3(256), 0, s,
                       a);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

size_t inbatch_standalone_workspace_bytes(int64_t B, int64_t Bc, int D) {
    size_t su, sp, parts;
    inbatch_workspace_floats(B, Bc, D, &su, &sp, &parts);
    return sizeof(float) * (su + sp + parts);
}

int inbatch_standalone(const float* U, int64_t B, int64_t ldu, const float* P, int64_t Bc, int64_t ldp, int D,
                       int64_t row_base, float inv_T, float* dU, int64_t ld_du, float* dP, int64_t ld_dp,
                       double* loss_sum, void* ws, size_t ws_bytes, hipStream_t s) {
    TTAMM_REQUIRE(U && P && dU && dP && loss_sum && ws, "inbatch_bce: null argument");
    TTAMM_REQUIRE(B > 0 && Bc > 0 && D > 0 && ldu >= D && ldp >= D && ld_du >= D && ld_dp >= D,
                  "inbatch_bce: bad shape");
    TTAMM_REQUIRE(row_base >= 0 && row_base + B <= Bc,
                  "inbatch_bce: row_base must place the B users' labels inside the Bc columns (0 <= row_base, "
                  "row_base + B <= Bc)");
    TTAMM_REQUIRE(ws_bytes >= inbatch_standalone_workspace_bytes(B, Bc, D), "inbatch_bce: workspace too small");
    InBatchArgs a{};
    a.U = U, a.ldu = ldu, a.B = B, a.P = P, a.ldp = ldp, a.Bc = Bc, a.D = D;
    a.row_base = row_base, a.inv_T = inv_T;
    size_t su, sp, parts;
    inbatch_workspace_floats(B, Bc, D, &su, &sp, &parts);
    float* w = static_cast<float*>(ws);
    a.slab_u = w, a.slab_p = w + su, a.loss_part = w + su + sp;
    a.dU = dU, a.ld_du = ld_du, a.dP = dP, a.ld_dp = ld_dp;
    const int rc = launch_inbatch(a, s);
    if (rc != TTAMM_OK) return rc;
    hipLaunchKernelGGL(ib_loss_sum_kernel, dim3(1), dim3(256), 0, s, a.loss_part, a.rblk_u * a.splits_u, loss_sum);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

}  // namespace ttamm
