// fp32 MFMA GEMMs of the tower MLP and fusion gate (gfx950).
//
//   C[M,N] = epilogue( sum_k A(m,k) * B(k,n) )
//
// Operands are staged HBM -> registers -> LDS (double buffered, one barrier per k-tile) in the
// orientation they have in memory:
//   MN-major  ([m][k] rows, k contiguous: an activation row or an nn.Linear weight row) —
//             LDS [mn][BK+4]; a lane reads its 4 next k values with one ds_read_b128.
//   K-major   ([k][m] rows, m contiguous: dgrad's weight, and both operands of the weight
//             gradient where k runs over batch rows) — LDS [BK][mn]; one ds_read_b32 per k.
// The operand whose memory rows are indexed by m (forward A) or by k (weight-gradient A)
// may be gathered through an int64 index, so gathered feature rows
// (training.py:741-747,775) are never materialised.
//
// Matrix core: v_mfma_f32_32x32x2_f32 (exact fp32: one rounding per product, like an fma
// chain).  Lane half h = lane>>5 owns k-slot h; inside a BK = 16 tile it walks k = 8h..8h+7.
// bf16 variant (BF = true; ttamm_tower.matmul_bf16, BASELINE config C5): the same LDS image
// and fragment reads — a lane's 8 k values 8h..8h+7 are exactly the A/B fragment of
// v_mfma_f32_32x32x16_bf16 (lane l: row l&31, k = 8(l>>5) + j) — rounded to bf16 (RNE,
// v_cvt_pk_bf16_f32) in registers; one bf16 MFMA replaces the eight fp32 ones per k-tile.
// Accumulation, epilogues and every stored tensor stay fp32.
//
// Epilogue: the accumulators go through LDS (in row slices) and 256 threads apply the fused
// elementwise tail with float4 loads/stores: bias, ReLU, dropout (encoders.py:132-138),
// ReLU', sigmoid gate mix + adaptive-mimic augment (encoders.py:164-168,
// adaptive_mimic.py:88-95), gate-mix backward.
//
// Weight gradients: dW^T[n_in, m_out] = X^T . dY, split over row chunks, written to fp32
// slabs and summed in a fixed order by wgrad_reduce_kernel; the bias gradient rides along as
// an implicit all-ones column of X.
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "kernels.h"

#ifndef TTAMM_GEMM_ABLATE
#define TTAMM_GEMM_ABLATE 0
#endif
#ifndef TTAMM_B16_ABLATE
#define TTAMM_B16_ABLATE 0
#endif

namespace ttamm {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

namespace {

// Kernel-argument (constant address space) view of a struct: indexing the by-value problem
// table with a block-uniform index then compiles to scalar loads instead of a scratch copy.

constexpr int BK = 16;
constexpr int SK = BK + 4;  // MN-major LDS row stride (floats): keeps ds_read_b128 conflict-free
constexpr int kThreads = 256;
// rows of one weight-gradient split: their gather indices are staged in LDS (Cfg::KIDX)
constexpr int kWgradMaxRowsPerSplit = 1024;

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }
__device__ __forceinline__ bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }
// 8 consecutive k values of one lane -> one bf16 MFMA fragment (round to nearest even)
__device__ __forceinline__ bf16x8 pack_bf16(float4 a, float4 b) {
    const f32x8 v = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    return __builtin_convertvector(v, bf16x8);
}
__device__ __forceinline__ float f4get(const float4& v, int q) {
    return q == 0 ? v.x : q == 1 ? v.y : q == 2 ? v.z : v.w;
}

// Operand fetch in two halves so the prefetch of a k-tile is never waited on early:
//   raw4:  one unconditional float4 load at a clamped in-bounds column (c <= ld - 4);
//   mask4: applied only when the tile is written to LDS (after the MFMAs of the current
//          tile): zeroes out-of-range elements, inserts the implicit all-ones column
//          (bias gradient) and drops the whole fetch when `ok` is false.
__device__ __forceinline__ int clamp_col(int c, int ld) { return max(0, min(c, ld - 4)); }
__device__ __forceinline__ float4 raw4(const float* rp, int c, int ld) {
    return *reinterpret_cast<const float4*>(rp + clamp_col(c, ld));
}
__device__ __forceinline__ float4 mask4(float4 v, int c, int lim, int ld, int ones, bool ok) {
    const bool same = clamp_col(c, ld) == c;
    float t[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int ce = c + e;
        t[e] = (ok && same && ce < lim) ? t[e] : ((ok && ce == ones) ? 1.0f : 0.f);
    }
    return make_float4(t[0], t[1], t[2], t[3]);
}

// MF: MFMA block edge — 32 (v_mfma_f32_32x32x2_f32 / 32x32x16_bf16) or 16
// (v_mfma_f32_16x16x4_f32, fp32 only): the 16-row granularity lets a tile height divide the
// step's row count into exactly two tiles per CU (C2: 57344 = 512 x 112).
template <int BM_, int BN_, int WAVES_M_, int WAVES_N_, bool A_KMAJ_, bool B_KMAJ_, int MF_ = 32>
struct Cfg {
    static constexpr int BM = BM_, BN = BN_, WAVES_M = WAVES_M_, WAVES_N = WAVES_N_, MF = MF_;
    static constexpr bool A_KMAJ = A_KMAJ_, B_KMAJ = B_KMAJ_;
    static constexpr int TM = BM / WAVES_M, TN = BN / WAVES_N;
    static constexpr int I = TM / MF, J = TN / MF;
    static constexpr int NR = MF == 32 ? 16 : 4;  // accumulator registers per MFMA block
    static constexpr int A_F4 = BM * BK / 4, B_F4 = BN * BK / 4;
    static constexpr int A_LOADS = (A_F4 + kThreads - 1) / kThreads;
    static constexpr int B_LOADS = (B_F4 + kThreads - 1) / kThreads;
    static constexpr int A_STAGE = A_KMAJ ? BK * BM : BM * SK;  // floats per buffer
    static constexpr int B_STAGE = B_KMAJ ? BK * BN : BN * SK;
    static constexpr int STAGE = 2 * (A_STAGE + B_STAGE);
    static constexpr int CLD = BN + 4;                           // epilogue tile row stride
    // epilogue row slices (whole MFMA row blocks): halves of the tile by wave rows, or by
    // row blocks when one wave row spans the tile
    static constexpr int EPI_ROWS = WAVES_M >= 2 ? BM / 2 : (I > 1 ? (I + 1) / 2 * MF : BM);
    static constexpr int EPI_PHASES = (BM + EPI_ROWS - 1) / EPI_ROWS;
    static constexpr int EPI = EPI_ROWS * CLD;
    static constexpr int KIDX = A_KMAJ ? 2 * kWgradMaxRowsPerSplit : 0;  // int64 gather rows (floats)
    static constexpr int LDS = (STAGE + KIDX) > EPI ? (STAGE + KIDX) : EPI;
    static_assert(WAVES_M * WAVES_N == 4, "4 waves per block");
    static_assert(MF == 32 || MF == 16, "MFMA block edge");
    static_assert(TM % MF == 0 && TN % MF == 0, "wave tile must be a multiple of the MFMA block");
    static_assert(WAVES_M == 1 || WAVES_M % EPI_PHASES == 0, "epilogue slices must hold whole wave rows");
};

// ---- the fused elementwise tail on 4 consecutive columns of one row ----------------------
// N % 4 == 0 (every layer width is a multiple of 4), so a column group is always whole and
// every operand access is one float4.  `bias4` is the group's bias (zero if none).
__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
// epilogue outputs are read by later kernels: streaming stores (common.h store_nt; measured
// neutral on the step, a plain-store build ran within noise of it)
__device__ __forceinline__ void st4(float* p, float4 v) { store_nt(p, v); }

// Feature-MLP activations (encoders.py:68-78, ttamm.h TTAMM_ACT_*), as ATen computes them on the
// CPU: ReLU; GELU (approximate='none') x / 2 (1 + erf(x / sqrt 2)), d = cdf + x pdf; Tanh, d = 1 - t^2;
// SELU scale (x > 0 ? x : alpha (exp(x) - 1)), d = x > 0 ? scale : scale alpha exp(x).  Non-ReLU
// layers keep their pre-activation (GemmProblem::pre) for the backward.
constexpr float kSeluAlpha = 1.6732632423543772848170429916717f;
constexpr float kSeluScale = 1.0507009873554804934193349852946f;
__device__ __forceinline__ float act_fwd(int act, float z) {
    switch (act) {
        case TTAMM_ACT_GELU: return z * 0.5f * (1.0f + erff(z * 0.70710678118654752440f));
        case TTAMM_ACT_TANH: return tanhf(z);
        case TTAMM_ACT_SELU: return z > 0.f ? z * kSeluScale : (expf(z) - 1.0f) * (kSeluAlpha * kSeluScale);
        default: return z > 0.f ? z : 0.f;
    }
}
__device__ __forceinline__ float act_grad(int act, float z) {
    switch (act) {
        case TTAMM_ACT_GELU: {
            const float cdf = 0.5f * (1.0f + erff(z * 0.70710678118654752440f));
            const float pdf = expf(-0.5f * z * z) * 0.39894228040143267794f;  // 1 / sqrt(2 pi)
            return cdf + z * pdf;
        }
        case TTAMM_ACT_TANH: {
            const float t = tanhf(z);
            return 1.0f - t * t;
        }
        case TTAMM_ACT_SELU: return z > 0.f ? kSeluScale : expf(z) * (kSeluAlpha * kSeluScale);
        default: return z > 0.f ? 1.f : 0.f;
    }
}

template <int E>
__device__ __forceinline__ void epilogue4(const KArg(GemmProblem) & P, float4 v, float4 bias4, int split, int row,
                                          int col) {
    const int N = P.N;
    float x[4] = {v.x + bias4.x, v.y + bias4.y, v.z + bias4.z, v.w + bias4.w};
    static_assert(E != EPI_HIDDEN, "EPI_HIDDEN runs through epilogue8_hidden");
    if (E == EPI_GATE_HIDDEN) {
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = x[e] > 0.f ? x[e] : 0.f;
    } else if (E == EPI_GATE_OUT) {
        const float* efr = P.aux0 + (int64_t)row * P.ld_aux0;
        const float4 ev = ld4(efr + col), fv = ld4(efr + N + col);
        const float e4[4] = {ev.x, ev.y, ev.z, ev.w}, f4[4] = {fv.x, fv.y, fv.z, fv.w};
        float g[4], t[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            g[e] = sigmoidf_(x[e]);
            t[e] = g[e] * e4[e] + (1.0f - g[e]) * f4[e];
        }
        const int64_t oo = (int64_t)row * P.ld_out2 + col;
        st4(P.out1 + (int64_t)row * P.ld_out + col, make_float4(g[0], g[1], g[2], g[3]));
        st4(P.out2 + oo, make_float4(t[0], t[1], t[2], t[3]));
        if (P.table) {
            const float4 a = ld4(P.table + P.idx[row] * (int64_t)N + col);
            st4(P.out3 + oo, a);
            x[0] = t[0] + a.x, x[1] = t[1] + a.y, x[2] = t[2] + a.z, x[3] = t[3] + a.w;
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) x[e] = t[e];
        }
    } else if (E == EPI_DGRAD_RELU) {
        const float4 z = ld4(P.aux0 + (int64_t)row * P.ld_aux0 + col);
        x[0] = z.x > 0.f ? x[0] : 0.f, x[1] = z.y > 0.f ? x[1] : 0.f;
        x[2] = z.z > 0.f ? x[2] : 0.f, x[3] = z.w > 0.f ? x[3] : 0.f;
    } else if (E == EPI_DGRAD_GATE_EF) {
        const int D = N >> 1;
        const int cc = col < D ? col : col - D;  // a group never straddles D (D % 4 == 0)
        const float4 dt = ld4(P.aux1 + (int64_t)row * P.ld_aux1 + cc);
        const float4 g = ld4(P.aux2 + (int64_t)row * P.ld_aux2 + cc);
        if (col < D) {
            x[0] += dt.x * g.x, x[1] += dt.y * g.y, x[2] += dt.z * g.z, x[3] += dt.w * g.w;
        } else {
            x[0] += dt.x * (1.0f - g.x), x[1] += dt.y * (1.0f - g.y);
            x[2] += dt.z * (1.0f - g.z), x[3] += dt.w * (1.0f - g.w);
        }
    } else if (E == EPI_DGRAD_HIDDEN) {
        const float4 hv = ld4(P.aux0 + (int64_t)row * P.ld_aux0 + col);
        if (P.act == TTAMM_ACT_RELU) {  // aux0 = the stored hidden output: > 0 iff ReLU passed and kept
            x[0] = hv.x > 0.f ? x[0] * P.inv_keep : 0.f, x[1] = hv.y > 0.f ? x[1] * P.inv_keep : 0.f;
            x[2] = hv.z > 0.f ? x[2] * P.inv_keep : 0.f, x[3] = hv.w > 0.f ? x[3] * P.inv_keep : 0.f;
        } else {  // aux0 = the pre-activation; keep bytes (injected or written by the forward)
            const float z[4] = {hv.x, hv.y, hv.z, hv.w};
            uint32_t km = 0xFFFFFFFFu;
            if (P.keep_prob < 1.0f) km = *reinterpret_cast<const uint32_t*>(P.keep_mask + (int64_t)row * N + col);
#pragma unroll
            for (int e = 0; e < 4; ++e)
                x[e] = ((km >> (8 * e)) & 0xFFu) ? x[e] * P.inv_keep * act_grad(P.act, z[e]) : 0.f;
        }
    }
    if (E == EPI_GATE_OUT && P.C == nullptr) return;  // sharded item owner: aug is formed by the requester
    st4(P.C + (int64_t)split * P.slab_stride + (int64_t)row * P.ldc + col, make_float4(x[0], x[1], x[2], x[3]));
}

// EPI_HIDDEN: bias, ReLU, dropout.  Dropout stream: the keep decision of column c of row r is
// 16-bit uniform (c & 1 ? high : low half) of word (c & 7) >> 1 of ONE Philox4x32-10 draw keyed
// by (row key, c / 8); keep iff u < round_down(keep_prob * 2^16) (resolution 2^-16).  Eight
// decisions per draw instead of four halve the tail's integer-multiply work (v_mul_hi is quarter
// rate), which bounded the first layer's epilogue.  A thread stores 4 columns of two rows
// (ra, rb = ra + row step), so a wave's stores stay contiguous; the lane pair (l, l ^ 1) holds the
// two halves of one 8-column group, each lane draws one of the two rows' words and they swap the
// halves the other needs.  An injected mask (uint8 per element, the parity tests) replaces the
// draw.  Both lanes of a pair must reach this call (a lane past N still draws; it stores nothing).
__device__ __forceinline__ uint32_t keep_threshold16(float keep_prob) {
    const float t = keep_prob * 65536.0f;  // exact (power-of-two scale)
    return t >= 65536.0f ? 65536u : (uint32_t)t;
}
__device__ __forceinline__ int64_t dropout_key(const KArg(GemmProblem) & P, int row) {
    return P.row_key ? P.row_key[row] : (row < P.key_split ? P.key_base0 + row : P.key_base1 + (row - P.key_split));
}
__device__ __forceinline__ void epilogue_hidden_pair(const KArg(GemmProblem) & P, float4 va, float4 vb, float4 bias4,
                                                     int split, int ra, int rb, bool oka, bool okb, int col) {
    const bool drop = P.keep_prob < 1.0f;
    uint32_t wa[2] = {0u, 0u}, wb[2] = {0u, 0u};
    if (drop && P.keep_mask == nullptr) {
        const int half = (col >> 2) & 1;
        const int M = P.M;
        const int my = min(half ? rb : ra, M - 1);  // half 0 draws row ra's group, half 1 row rb's
        const u32x4 d = philox4x32(u32x4{(uint32_t)dropout_key(P, my), (uint32_t)(col >> 3), P.rng_c2, P.rng_c3},
                                   P.rng_k0, P.rng_k1);
        // half 0 needs words 0, 1 of both rows; half 1 words 2, 3: send the partner its pair
        const uint32_t s0 = half ? d.x : d.z, s1 = half ? d.y : d.w;
        const uint32_t r0 = (uint32_t)__shfl_xor((int)s0, 1), r1 = (uint32_t)__shfl_xor((int)s1, 1);
        wa[0] = half ? r0 : d.x, wa[1] = half ? r1 : d.y;
        wb[0] = half ? d.z : r0, wb[1] = half ? d.w : r1;
    }
    const uint32_t thresh = keep_threshold16(P.keep_prob);
    auto tail = [&](float4 v, const uint32_t w[2], int row) {
        float x[4] = {v.x + bias4.x, v.y + bias4.y, v.z + bias4.z, v.w + bias4.w};
        if (P.pre) st4(P.pre + (int64_t)row * P.ldc + col, make_float4(x[0], x[1], x[2], x[3]));
        uint32_t km = 0xFFFFFFFFu, kept = 0u;
        if (drop && P.keep_mask) km = *reinterpret_cast<const uint32_t*>(P.keep_mask + (int64_t)row * P.N + col);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float hv = P.act == TTAMM_ACT_RELU ? (x[e] > 0.f ? x[e] : 0.f) : act_fwd(P.act, x[e]);
            if (drop) {
                const bool keep = P.keep_mask ? ((km >> (8 * e)) & 0xFFu) != 0
                                              : ((w[e >> 1] >> (16 * (e & 1))) & 0xFFFFu) < thresh;
                hv = hv * (keep ? P.inv_keep : 0.f);
                kept |= keep ? (1u << (8 * e)) : 0u;
            }
            x[e] = hv;
        }
        if (P.mask_out && drop) *reinterpret_cast<uint32_t*>(P.mask_out + (int64_t)row * P.N + col) = kept;
        st4(P.C + (int64_t)split * P.slab_stride + (int64_t)row * P.ldc + col, make_float4(x[0], x[1], x[2], x[3]));
    };
    if (oka) tail(va, wa, ra);
    if (okb) tail(vb, wb, rb);
}

// The same stream, one thread per 8 consecutive columns of a row (one draw each): the split
// kernel's epilogue measured faster this way (its stores are 32-B strided per instruction but its
// loop half as long); the bf16-operand kernel's faster with the lane pairs above.
__device__ __forceinline__ void epilogue8_hidden(const KArg(GemmProblem) & P, float4 v0, float4 v1, float4 b0,
                                                 float4 b1, int split, int row, int col) {
    const int N = P.N;
    float x[8] = {v0.x + b0.x, v0.y + b0.y, v0.z + b0.z, v0.w + b0.w,
                  v1.x + b1.x, v1.y + b1.y, v1.z + b1.z, v1.w + b1.w};
    const bool hi_ok = col + 4 < N;
    const bool drop = P.keep_prob < 1.0f;
    u32x4 rnd = {0u, 0u, 0u, 0u};
    if (drop && P.keep_mask == nullptr)
        rnd = philox4x32(u32x4{(uint32_t)dropout_key(P, row), (uint32_t)(col >> 3), P.rng_c2, P.rng_c3}, P.rng_k0,
                         P.rng_k1);
    uint32_t km[2] = {0xFFFFFFFFu, 0xFFFFFFFFu};
    if (drop && P.keep_mask) {
        const uint8_t* mrow = P.keep_mask + (int64_t)row * N + col;
        km[0] = *reinterpret_cast<const uint32_t*>(mrow);
        if (hi_ok) km[1] = *reinterpret_cast<const uint32_t*>(mrow + 4);
    }
    const uint32_t thresh = keep_threshold16(P.keep_prob);
    const uint32_t w[4] = {rnd.x, rnd.y, rnd.z, rnd.w};
    if (P.pre) {  // non-ReLU layers: the pre-activation for the backward
        float* pr = P.pre + (int64_t)row * P.ldc + col;
        *reinterpret_cast<float4*>(pr) = make_float4(x[0], x[1], x[2], x[3]);
        if (hi_ok) *reinterpret_cast<float4*>(pr + 4) = make_float4(x[4], x[5], x[6], x[7]);
    }
    uint32_t kept[2] = {0u, 0u};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        float hv = P.act == TTAMM_ACT_RELU ? (x[e] > 0.f ? x[e] : 0.f) : act_fwd(P.act, x[e]);
        if (drop) {
            const bool keep = P.keep_mask ? ((km[e >> 2] >> (8 * (e & 3))) & 0xFFu) != 0
                                          : ((w[e >> 1] >> (16 * (e & 1))) & 0xFFFFu) < thresh;
            hv = hv * (keep ? P.inv_keep : 0.f);
            kept[e >> 2] |= keep ? (1u << (8 * (e & 3))) : 0u;
        }
        x[e] = hv;
    }
    if (P.mask_out && drop) {  // the drawn keep decisions, for a non-ReLU layer's backward
        uint8_t* mo = P.mask_out + (int64_t)row * N + col;
        *reinterpret_cast<uint32_t*>(mo) = kept[0];
        if (hi_ok) *reinterpret_cast<uint32_t*>(mo + 4) = kept[1];
    }
    // plain (write-back) stores: a wave's two store instructions each cover every other 16 B of
    // its rows' span, and L2 merges the halves into whole lines; non-temporal stores of the halves
    // doubled the HBM write bytes (PMC WRITE_SIZE 82 MB vs 44 MB of hidden rows at C2)
    float* out = P.C + (int64_t)split * P.slab_stride + (int64_t)row * P.ldc + col;
    *reinterpret_cast<float4*>(out) = make_float4(x[0], x[1], x[2], x[3]);
    if (hi_ok) *reinterpret_cast<float4*>(out + 4) = make_float4(x[4], x[5], x[6], x[7]);
}

template <class CF, int E, bool BF>
__global__ __launch_bounds__(kThreads) void gemm_kernel(GemmBatch batch) {
    constexpr int BM = CF::BM, BN = CF::BN, TM = CF::TM, TN = CF::TN, I = CF::I, J = CF::J;
    constexpr bool AK = CF::A_KMAJ, BKM = CF::B_KMAJ;
    __shared__ __attribute__((aligned(16))) float lds[CF::LDS];

    // ---- problem / tile --------------------------------------------------------------------
    const KArg(GemmBatch)* kb = (const KArg(GemmBatch)*)(__builtin_amdgcn_kernarg_segment_ptr());
    int tile = blockIdx.x;
    int pi = 0;
#pragma unroll 1
    for (int q = 1; q < kb->count; ++q)
        if (tile >= kb->p[q].tile_begin) pi = q;
    const KArg(GemmProblem)& P = kb->p[pi];
    tile -= P.tile_begin;
    const int tiles_mn = P.tiles_m * P.tiles_n;
    const int split = tile / tiles_mn;
    tile -= split * tiles_mn;
    const int tm = tile / P.tiles_n, tn = tile - tm * P.tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const int M = P.M, N = P.N;
    const int k_begin = split * P.k_split;
    const int k_end = min(P.K, k_begin + P.k_split);

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / CF::WAVES_N, wn = wave % CF::WAVES_N;
    constexpr int MF = CF::MF;
    // lane -> (row/column in an MFMA block, k slot): 32x32x2 has 2 k slots of 32 lanes,
    // 16x16x4 has 4 k slots of 16 lanes
    const int li = lane & (MF - 1), h = lane / MF;
    float* As = lds;
    float* Bs = lds + 2 * CF::A_STAGE;

    // ---- global -> register staging ---------------------------------------------------------
    // MN-major A: thread -> (m row, 4 k), row pointers resolved once (gather on m).
    // K-major A:  thread -> (k row, 4 m), gather indices of the whole k range staged in LDS.
    const float* a_rp[CF::A_LOADS];
    bool a_ok[CF::A_LOADS];
    int a_r[CF::A_LOADS], a_c[CF::A_LOADS];
#pragma unroll
    for (int it = 0; it < CF::A_LOADS; ++it) {
        const int lin = tid + it * kThreads;
        if (!AK) {
            a_r[it] = lin / (BK / 4);
            a_c[it] = (lin % (BK / 4)) * 4;
            const int gm = m0 + a_r[it];
            a_ok[it] = lin < CF::A_F4 && gm < M;
            const int gmc = min(gm, M - 1);
            a_rp[it] = P.A + (P.a_idx ? P.a_idx[gmc] : (int64_t)gmc) * P.lda;
        } else {
            a_r[it] = lin / (BM / 4);
            a_c[it] = (lin % (BM / 4)) * 4;
            a_ok[it] = lin < CF::A_F4;
            a_rp[it] = P.A;
        }
    }
    int64_t* kidx = reinterpret_cast<int64_t*>(lds + CF::STAGE);  // K-major gather rows
    if (AK) {
        for (int k = tid; k < k_end - k_begin; k += kThreads)
            kidx[k] = P.a_idx ? P.a_idx[k_begin + k] : (int64_t)(k_begin + k);
        __syncthreads();
    }
    // two register sets: the k-tile two ahead is in flight while the next one is written to LDS
    float4 ra[2][CF::A_LOADS], rb[2][CF::B_LOADS];

    // Interior blocks with whole k-tiles take the FAST variant of the main loop: pointers
    // resolved once, plain float4 loads, no masking.  Edge blocks take the masked variant.
    // The choice is block-uniform and made once, outside the loop.
    const bool fast = ((k_end - k_begin) % BK == 0) && (n0 + BN <= N) &&
                      (AK ? (m0 + BM <= P.a_cols) : (m0 + BM <= M));
    const float* b_rp[CF::B_LOADS];
#pragma unroll
    for (int it = 0; it < CF::B_LOADS; ++it) {
        const int lin = tid + it * kThreads;
        if (!BKM) b_rp[it] = P.B + (int64_t)min(n0 + (lin >> 2), N - 1) * P.ldb + (lin & 3) * 4;
        else b_rp[it] = P.B + (int64_t)(lin / (BN / 4)) * P.ldb + n0 + (lin % (BN / 4)) * 4;
    }

    using Acc = std::conditional_t<MF == 32, f32x16, f32x4_t>;
    Acc acc[I][J];
#pragma unroll
    for (int i = 0; i < I; ++i)
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
            for (int r = 0; r < CF::NR; ++r) acc[i][j][r] = 0.f;

    auto mainloop = [&](auto fast_tag) {
        constexpr bool FAST = decltype(fast_tag)::value;
        auto load_tile = [&](auto S, int k0) {
            constexpr int R = decltype(S)::value;
#pragma unroll
            for (int it = 0; it < CF::A_LOADS; ++it) {
                if (!AK) {
                    ra[R][it] = FAST ? *reinterpret_cast<const float4*>(a_rp[it] + k0 + a_c[it])
                                  : raw4(a_rp[it], k0 + a_c[it], P.lda);
                } else {
                    const int k = FAST ? k0 + a_r[it] : min(k0 + a_r[it], k_end - 1);
                    const float* rp = P.A + kidx[k - k_begin] * P.lda;
                    ra[R][it] = FAST ? *reinterpret_cast<const float4*>(rp + m0 + a_c[it]) : raw4(rp, m0 + a_c[it], P.lda);
                }
            }
#pragma unroll
            for (int it = 0; it < CF::B_LOADS; ++it) {
                const int lin = tid + it * kThreads;
                if (!BKM) {
                    rb[R][it] = FAST ? *reinterpret_cast<const float4*>(b_rp[it] + k0)
                                     : raw4(b_rp[it] - (lin % (BK / 4)) * 4, k0 + (lin % (BK / 4)) * 4, P.ldb);
                } else if (FAST) {
                    rb[R][it] = *reinterpret_cast<const float4*>(b_rp[it] + (int64_t)k0 * P.ldb);
                } else {
                    const int k = min(k0 + lin / (BN / 4), k_end - 1);
                    rb[R][it] = raw4(P.B + (int64_t)k * P.ldb, n0 + (lin % (BN / 4)) * 4, P.ldb);
                }
            }
        };
        auto store_tile = [&](auto S, auto Buf, int k0) {
            constexpr int R = decltype(S)::value;  // register set
            constexpr int buf = decltype(Buf)::value;
            float* as = As + buf * CF::A_STAGE;
            float* bs = Bs + buf * CF::B_STAGE;
#pragma unroll
            for (int it = 0; it < CF::A_LOADS; ++it) {
                const int lin = tid + it * kThreads;
                if (lin >= CF::A_F4) continue;
                if (!AK) {
                    const float4 v = FAST ? ra[R][it] : mask4(ra[R][it], k0 + a_c[it], k_end, P.lda, -1, a_ok[it]);
                    *reinterpret_cast<float4*>(as + a_r[it] * SK + a_c[it]) = v;
                } else {
                    const float4 v = FAST ? ra[R][it]
                                          : mask4(ra[R][it], m0 + a_c[it], P.a_cols, P.lda, P.a_ones_col,
                                                  k0 + a_r[it] < k_end);
                    *reinterpret_cast<float4*>(as + a_r[it] * BM + a_c[it]) = v;
                }
            }
#pragma unroll
            for (int it = 0; it < CF::B_LOADS; ++it) {
                const int lin = tid + it * kThreads;
                if (lin >= CF::B_F4) continue;
                if (!BKM) {
                    const int n = n0 + (lin >> 2), c = k0 + (lin & 3) * 4;
                    *reinterpret_cast<float4*>(bs + (lin >> 2) * SK + (lin & 3) * 4) =
                        FAST ? rb[R][it] : mask4(rb[R][it], c, k_end, P.ldb, -1, n < N);
                } else {
                    const int kr = lin / (BN / 4), nc = (lin % (BN / 4)) * 4;
                    *reinterpret_cast<float4*>(bs + kr * BN + nc) =
                        FAST ? rb[R][it] : mask4(rb[R][it], n0 + nc, N, P.ldb, -1, k0 + kr < k_end);
                }
            }
        };

        const int nk = k_end > k_begin ? (k_end - k_begin + BK - 1) / BK : 0;
        auto kof = [&](int kt) { return k_begin + kt * BK; };
        // k-tile kt lives in LDS buffer kt & 1 and passes through register set kt & 1
        auto compute = [&](auto S) {
            constexpr int buf = decltype(S)::value;
            const float* as = As + buf * CF::A_STAGE;
            const float* bs = Bs + buf * CF::B_STAGE;
            // the lane's 4 k values kb .. kb+3 of A row m / B column n, kb = 8h + 4*s4 (32x32:
            // lane half h walks k = 8h..8h+7) or 4h (16x16: k slot h walks k = 4h..4h+3)
            auto kbase = [&](int s4) { return MF == 32 ? 8 * h + 4 * s4 : 4 * h; };
            auto frag_a = [&](int i, int s4) -> float4 {
                const int m = wm * TM + i * MF + li;
                if (!AK) return *reinterpret_cast<const float4*>(as + m * SK + kbase(s4));
                const float* c = as + kbase(s4) * BM + m;
                return make_float4(c[0], c[BM], c[2 * BM], c[3 * BM]);
            };
            auto frag_b = [&](int j, int s4) -> float4 {
                const int n = wn * TN + j * MF + li;
                if (!BKM) return *reinterpret_cast<const float4*>(bs + n * SK + kbase(s4));
                const float* c = bs + kbase(s4) * BN + n;
                return make_float4(c[0], c[BN], c[2 * BN], c[3 * BN]);
            };
            if constexpr (MF == 16) {
                static_assert(!BF, "16x16 blocks are fp32 only");
                float4 af[I], bf[J];
#pragma unroll
                for (int i = 0; i < I; ++i) af[i] = frag_a(i, 0);
#pragma unroll
                for (int j = 0; j < J; ++j) bf[j] = frag_b(j, 0);
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int i = 0; i < I; ++i)
#pragma unroll
                        for (int j = 0; j < J; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4get(af[i], q), f4get(bf[j], q),
                                                                             acc[i][j], 0, 0, 0);
            } else if constexpr (BF) {
                bf16x8 a8[I], b8[J];
#pragma unroll
                for (int i = 0; i < I; ++i) a8[i] = pack_bf16(frag_a(i, 0), frag_a(i, 1));
#pragma unroll
                for (int j = 0; j < J; ++j) b8[j] = pack_bf16(frag_b(j, 0), frag_b(j, 1));
#pragma unroll
                for (int i = 0; i < I; ++i)
#pragma unroll
                    for (int j = 0; j < J; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a8[i], b8[j], acc[i][j], 0, 0, 0);
            } else {
#pragma unroll
                for (int s4 = 0; s4 < 2; ++s4) {
                    float4 af[I], bf[J];
#pragma unroll
                    for (int i = 0; i < I; ++i) af[i] = frag_a(i, s4);
#pragma unroll
                    for (int j = 0; j < J; ++j) bf[j] = frag_b(j, s4);
#pragma unroll
                    for (int q = 0; q < 4; ++q)
#pragma unroll
                        for (int i = 0; i < I; ++i)
#pragma unroll
                            for (int j = 0; j < J; ++j)
                                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4get(af[i], q), f4get(bf[j], q),
                                                                                 acc[i][j], 0, 0, 0);
                }
            }
        };
        using S0 = std::integral_constant<int, 0>;
        using S1 = std::integral_constant<int, 1>;
        // Prefetch depth: MN-major A (forward / dgrad) keeps two k-tiles in flight through two
        // register sets; the K-major gathered A of the weight gradients keeps one (measured
        // faster: the second set costs occupancy there).
        constexpr bool DEEP = !AK;
        if (nk > 0) {
            load_tile(S0{}, kof(0));
            store_tile(S0{}, S0{}, kof(0));
        }
        if (DEEP && nk > 1) load_tile(S1{}, kof(1));
        __syncthreads();
        // one step on LDS buffer B: DEEP — prefetch k-tile kt+2 into register set B (its LDS
        // buffer is free after the barrier), compute kt, write kt+1 (set NB) to buffer NB;
        // shallow — prefetch kt+1 into set 0, compute kt, write set 0 to buffer NB
        auto step = [&](auto Bf, auto NB, int kt) {
            if constexpr (DEEP) {
#if TTAMM_GEMM_ABLATE != 1  // developer ablation 1: no k-loop traffic (measures the MFMA/LDS loop)
                if (kt + 2 < nk) load_tile(Bf, kof(kt + 2));
#endif
                compute(Bf);
#if TTAMM_GEMM_ABLATE != 1
                if (kt + 1 < nk) store_tile(NB, NB, kof(kt + 1));
#endif
            } else {
#if TTAMM_GEMM_ABLATE != 1
                if (kt + 1 < nk) load_tile(S0{}, kof(kt + 1));
#endif
                compute(Bf);
#if TTAMM_GEMM_ABLATE != 1
                if (kt + 1 < nk) store_tile(S0{}, NB, kof(kt + 1));
#endif
            }
            __syncthreads();
        };
        int kt = 0;
        for (; kt + 1 < nk; kt += 2) {
            step(S0{}, S1{}, kt);
            step(S1{}, S0{}, kt + 1);
        }
        if (kt < nk) step(S0{}, S1{}, kt);
    };
    if (fast) mainloop(std::true_type{});
    else mainloop(std::false_type{});

    // ---- epilogue through LDS, in row slices ----------------------------------------------------
    float* Cs = lds;
    for (int ph = 0; ph < CF::EPI_PHASES; ++ph) {
        const int row_lo = ph * CF::EPI_ROWS;
        const int rows_here = min(CF::EPI_ROWS, BM - row_lo);
#pragma unroll
        for (int i = 0; i < I; ++i) {
            const int br = wm * TM + i * MF;  // first tile row of MFMA row block i
            if (br < row_lo || br >= row_lo + CF::EPI_ROWS) continue;
#pragma unroll
            for (int j = 0; j < J; ++j)
#pragma unroll
                for (int r = 0; r < CF::NR; ++r) {
                    const int rr = br - row_lo + (MF == 32 ? (r & 3) + 8 * (r >> 2) + 4 * h : 4 * h + r);
                    Cs[rr * CF::CLD + wn * TN + j * MF + li] = acc[i][j][r];
                }
        }
        __syncthreads();
        // each thread owns one 4-column group (bias loaded once) and walks rows
        if constexpr (E == EPI_HIDDEN) {
            // two rows per pass; lane pairs share the dropout draws (epilogue_hidden_pair)
            constexpr int C4 = BN / 4;
            constexpr int RSTEP = kThreads / C4;
            static_assert(C4 % 2 == 0, "lane pairs hold 8-column groups");
            const int c4 = tid % C4, r0 = tid / C4;
            const int col = n0 + c4 * 4;
            if (r0 < RSTEP && col < ((N + 7) & ~7)) {
                const float4 bias4 = (P.bias && col < N) ? ld4(P.bias + col) : make_float4(0.f, 0.f, 0.f, 0.f);
                const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 2
                for (int rr = r0; rr < rows_here; rr += 2 * RSTEP) {
                    const int rb_ = rr + RSTEP;
                    const int ra = m0 + row_lo + rr, rb = m0 + row_lo + rb_;
                    const bool in_b = rb_ < rows_here;
                    epilogue_hidden_pair(P, ld4(Cs + rr * CF::CLD + c4 * 4), in_b ? ld4(Cs + rb_ * CF::CLD + c4 * 4) : z4, bias4,
                                         split, ra, rb, ra < M && col < N, in_b && rb < M && col < N, col);
                }
            }
        } else {
            constexpr int C4 = BN / 4;
            constexpr int RSTEP = kThreads / C4;
            const int c4 = tid % C4, r0 = tid / C4;
            const int col = n0 + c4 * 4;
            if (r0 < RSTEP && col < N) {
                const bool has_bias = (E == EPI_STORE || E == EPI_HIDDEN || E == EPI_GATE_HIDDEN || E == EPI_GATE_OUT) &&
                                      P.bias != nullptr;
                const float4 bias4 = has_bias ? ld4(P.bias + col) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 4
                for (int rr = r0; rr < rows_here; rr += RSTEP) {
                    const int row = m0 + row_lo + rr;
                    if (row < M) epilogue4<E>(P, ld4(Cs + rr * CF::CLD + c4 * 4), bias4, split, row, col);
                }
            }
        }
        __syncthreads();
    }
}

// ---- split-bf16 MFMA GEMM (fp32 products from three bf16 planes) ------------------------------
// Same problems, staging and epilogues as gemm_kernel; the matrix core is
// v_mfma_f32_32x32x16_bf16 (16x the rate of v_mfma_f32_32x32x2_f32).  Each staged fp32 value x
// is split, once, when its k-tile is written to LDS:
//     hi = bf16(x),  mid = bf16(x - hi),  lo = bf16(x - hi - mid)      (RNE; all differences exact)
// hi + mid + lo == x exactly for normal x (8 + 8 + 8 significand bits), so with PL = 3 planes
//     a.b = ah.bh + ah.bm + am.bh + ah.bl + al.bh + am.bm   (+ terms below 2^-24 relative)
// six bf16 MFMAs reproduce each fp32 product to within fp32 rounding, accumulated in fp32:
// 6/16 of the fp32 MFMA's cycles.  PL = 1 keeps only hi: the bf16 towers of config C5 (the
// operands rounded RNE once, as before).
// Pipeline: KT = 16 k per tile (one 32x32x16 step), LDS double buffered, two register sets —
// the k-tile two ahead is loaded while the current one is multiplied and the next one split
// into the other buffer; one barrier per k-tile; two workgroups per CU.
// LDS image per plane:
//   MN-major operand: [mn][16 k] bf16, 32-B rows, the two 16-B halves swapped on rows with
//                     bit 3 set — a lane's 8 k values are one ds_read_b128, conflict-free over
//                     the b128 lane groups;
//   K-major operand:  [16 k][mn] bf16, row stride = 64 or 192 (mod 256) bytes — fragments are
//                     two ds_read_b64_tr_b16 (hardware transpose: lane i of a 16-lane group gets
//                     column i of a 4 x 16 block), conflict-free per 32-lane half.
template <int BM_, int BN_, int WAVES_M_, int WAVES_N_, bool A_KMAJ_, bool B_KMAJ_, int KT_ = 16, int AD_ = 2,
          bool APL_ = false, bool A16_ = false>
struct XCfg {
    static constexpr int BM = BM_, BN = BN_, WAVES_M = WAVES_M_, WAVES_N = WAVES_N_;
    static constexpr bool A_KMAJ = A_KMAJ_, B_KMAJ = B_KMAJ_;
    static constexpr int KT = KT_;     // k per tile: 16 (three planes) or 32 (bf16, one plane)
    static constexpr int AD = AD_;     // 16-k tiles: A register sets (3: A loads two k-tiles ahead)
    // A pre-split in memory (GemmProblem::A3p: [row][k / 16][hi, mid, lo][16] bf16, the feature rows
    // split once): staged as 16-B pieces of the three planes, no split arithmetic in the loop
    static constexpr bool APL = APL_;
    // A16: K-major A already bf16 in memory (GemmProblem::A16 / lda16, rows gathered by a_idx; the bf16
    // towers' feature copy): 16-B pieces of 8 columns straight into the plane, no conversion
    static constexpr bool A16 = A16_;
    static_assert(!A16 || (A_KMAJ_ && KT_ == 32 && !APL_), "bf16 A: K-major, one plane (32-k tiles)");
    static constexpr int RB = KT * 2;  // MN-major row bytes
    static constexpr int TM = BM / WAVES_M, TN = BN / WAVES_N, I = TM / 32, J = TN / 32;
    // blocks per CU the register budget is planned for: wave tiles of 8 or more accumulator tiles
    // (128 registers and up) run one wave per SIMD with the whole register file
    static constexpr int MINB = I * J >= 8 ? 1 : 2;
    static constexpr int A_F4 = APL ? BM * KT * 6 / 16 : (A16 ? BM * KT / 8 : BM * KT / 4), B_F4 = BN * KT / 4;
    static_assert(!APL || KT == 16, "A planes: 16-k tiles (one 96-byte chunk per row and k-tile)");
    static constexpr int A_LOADS = (A_F4 + kThreads - 1) / kThreads;
    static constexpr int B_LOADS = (B_F4 + kThreads - 1) / kThreads;
    static constexpr int kmaj_stride(int mn) {
        int s = mn * 2;
        while (s % 256 != 64 && s % 256 != 192) s += 16;
        return s;
    }
    static constexpr int SA = A_KMAJ ? kmaj_stride(BM) : RB;  // row stride, bytes
    static constexpr int SB = B_KMAJ ? kmaj_stride(BN) : RB;
    static constexpr int A_PLANE = A_KMAJ ? KT * SA : BM * RB;  // bytes
    static constexpr int B_PLANE = B_KMAJ ? KT * SB : BN * RB;
    static_assert(KT == 16 || KT == 32, "k tile of 16 or 32");
    static constexpr int CLD = BN + 4;
    static constexpr int EPI_ROWS = WAVES_M >= 2 ? BM / 2 : (I > 1 ? (I + 1) / 2 * 32 : BM);
    static constexpr int EPI_PHASES = (BM + EPI_ROWS - 1) / EPI_ROWS;
    // K-major A: the split's (gathered) row ids as int32 (tables < 2^31 rows): 4 KB, so the
    // 128 x 96 weight-gradient tile fits three blocks per CU (53,248 B of LDS each)
    static constexpr int KIDX_BYTES = A_KMAJ ? 4 * kWgradMaxRowsPerSplit : 0;
    static constexpr int buf_bytes(int pl) { return pl * (A_PLANE + B_PLANE); }
    static constexpr int lds_bytes(int pl) {
        const int st = 2 * buf_bytes(pl) + KIDX_BYTES, ep = EPI_ROWS * CLD * 4;
        return st > ep ? st : ep;
    }
    static_assert(WAVES_M * WAVES_N == 4, "4 waves per block");
    static_assert(TM % 32 == 0 && TN % 32 == 0, "wave tile must be a multiple of 32");
    static_assert(A_F4 % kThreads == 0, "whole A staging rounds");
    static_assert(WAVES_M == 1 || WAVES_M % EPI_PHASES == 0, "epilogue slices must hold whole wave rows");
};

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4e __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

#ifndef TTAMM_X_ABLATE
#define TTAMM_X_ABLATE 0
#endif
#ifndef TTAMM_SPLIT8
#define TTAMM_SPLIT8 0
#endif
// The mid x mid partial product (|mid| <= 2^-9 |x|, so <= 2^-18 of |ab|): kept (six products).
// Without it (-DTTAMM_SPLIT_MM=0, five) the GEMMs ran 1.2-1.5 % faster at C2 but their error
// against fp64 tripled (max |err| / max |C| 9.4e-7 -> 2.7e-6 on layer 1, fp32 MFMA 9.5e-7) and the
// C1-large epoch-1 mean moved to 5.5e-5 of float64 (profiles/r06_s14_*); the in-batch
// kernel, whose errors did not move, takes five (inbatch.hip TTAMM_IB_PRODUCTS)
#ifndef TTAMM_SPLIT_MM
#define TTAMM_SPLIT_MM 1
#endif
#ifndef TTAMM_BF16_DEEP
#define TTAMM_BF16_DEEP 1
#endif
// x -> (hi, mid, lo) bf16 quadruples, 8 bytes each
template <int PL>
__device__ __forceinline__ void split_bf16(float4 v, uint2 out[PL]) {
#if TTAMM_X_ABLATE == 4  // developer ablation 4: no split arithmetic (the raw bits as planes)
    out[0] = uint2{__float_as_uint(v.x), __float_as_uint(v.y)};
    if constexpr (PL == 3) {
        out[1] = uint2{__float_as_uint(v.z), __float_as_uint(v.w)};
        out[2] = out[0];
    }
    return;
#endif
    const f32x4e x = {v.x, v.y, v.z, v.w};
    const bf16x4 h = __builtin_convertvector(x, bf16x4);
    out[0] = __builtin_bit_cast(uint2, h);
    if constexpr (PL == 3) {
        const f32x4e r = x - __builtin_convertvector(h, f32x4e);
        const bf16x4 m = __builtin_convertvector(r, bf16x4);
        const f32x4e r2 = r - __builtin_convertvector(m, f32x4e);
        out[1] = __builtin_bit_cast(uint2, m);
        out[2] = __builtin_bit_cast(uint2, __builtin_convertvector(r2, bf16x4));
    }
}

// byte offset of k values [c, c + 4) of row `row` in an MN-major plane of RB-byte rows: the
// row's 16-B chunks are XOR-permuted by the row's index among the rows that share a 256-B bank
// window (32-B rows: halves swapped on rows with bit 3 set; 64-B rows: chunk ^ (row >> 2) & 3),
// so the 16 rows of every ds_read_b128 lane group hit 16 distinct bank quads
template <int RB>
__device__ __forceinline__ int mn_off(int row, int c) {
    constexpr int CH = RB / 16, PER = 256 / RB;  // chunks per row, rows per bank window
    return row * RB + (((c >> 3) ^ ((row / PER) & (CH - 1))) << 4) + (c & 4) * 2;
}

// 32x32x16 operand fragment of MFMA block rows [r0, r0 + 32) (lane l: row r0 + (l & 31),
// k = 8 (l >> 5) + j)
template <bool KMAJ, int S>
__device__ __forceinline__ bf16x8 frag16(const unsigned char* plane, int r0, int kk, int lane) {
    if constexpr (!KMAJ) {
        return *reinterpret_cast<const bf16x8*>(plane + mn_off<S>(r0 + (lane & 31), kk + 8 * (lane >> 5)));
    } else {
        // lane 4q+p of 16-lane group g: block row k = kk + 8(g>>1) + q, columns r0 + 16(g&1) + 4p
        const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
        const unsigned char* a = plane + (kk + 8 * (g >> 1) + q) * S + (r0 + 16 * (g & 1) + 4 * p) * 2;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a + 4 * S));
        const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        return __builtin_bit_cast(bf16x8, v);
    }
}

__device__ __forceinline__ int xcd_remap(int b, int n) {  // bijective: consecutive tiles on one XCD
    const int q = n / 8, r = n % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

template <class CX, int E, int PL>
__global__ __launch_bounds__(kThreads, CX::MINB) void gemm_x_kernel(GemmBatch batch) {
    constexpr int BM = CX::BM, BN = CX::BN, TM = CX::TM, TN = CX::TN, I = CX::I, J = CX::J, KT = CX::KT;
    constexpr bool AK = CX::A_KMAJ, BKM = CX::B_KMAJ;
    __shared__ __attribute__((aligned(16))) unsigned char lds[CX::lds_bytes(PL)];

    const KArg(GemmBatch)* kb = (const KArg(GemmBatch)*)(__builtin_amdgcn_kernarg_segment_ptr());
    // weight gradients (K-major A): the M-tiles of one row split are consecutive tiles; remapped
    // onto one XCD (round-robin dispatch: blocks b and b + 8 share one) they read the split's dY
    // chunk from that XCD's L2 once instead of once per M-tile from the fabric
    int tile = AK ? xcd_remap(blockIdx.x, kb->total_tiles) : (int)blockIdx.x;
    int pi = 0;
#pragma unroll 1
    for (int q = 1; q < kb->count; ++q)
        if (tile >= kb->p[q].tile_begin) pi = q;
    const KArg(GemmProblem)& P = kb->p[pi];
    tile -= P.tile_begin;
    const int tiles_mn = P.tiles_m * P.tiles_n;
    const int split = tile / tiles_mn;
    tile -= split * tiles_mn;
    const int tm = tile / P.tiles_n, tn = tile - tm * P.tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const int M = P.M, N = P.N;
    const int k_begin = split * P.k_split;
    const int k_end = min(P.K, k_begin + P.k_split);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / CX::WAVES_N, wn = wave % CX::WAVES_N;
    const int li = lane & 31, h = lane >> 5;

    // staging maps: MN-major thread -> (row lin / 4, k 4 * (lin % 4)); K-major -> (k row, 4 mn)
    const float* a_rp[CX::A_LOADS];
    bool a_ok[CX::A_LOADS];
    int a_r[CX::A_LOADS], a_c[CX::A_LOADS];
    // A planes: piece lin of a k-tile = (row, plane, 8-k half) — MN-major: row lin / 6, then
    // (plane, half) = lin % 6; K-major: k row lin / 48, 16-column chunk (lin % 48) / 6, then
    // (plane, half).  a_c holds the piece's element offset inside the row's planes, relative to the
    // k-tile's (MN-major) or the M-tile's (K-major) first chunk; a_rp the row (MN-major)
    const uint16_t* ap_rp[CX::APL ? CX::A_LOADS : 1];
    int ap_lds[CX::APL ? CX::A_LOADS : 1];  // byte offset in the buffer's A planes
#pragma unroll
    for (int it = 0; it < CX::A_LOADS; ++it) {
        const int lin = tid + it * kThreads;
        if constexpr (CX::APL) {
            const int ph = AK ? (lin % 48) % 6 : lin % 6, pl = ph >> 1, hf = ph & 1;
            if (!AK) {
                a_r[it] = lin / 6;
                a_c[it] = pl * 16 + hf * 8;
                const int gm = m0 + a_r[it];
                a_ok[it] = gm < M;
                const int gmc = min(gm, M - 1);
                ap_rp[it] = P.A3p + (P.a_idx ? P.a_idx[gmc] : (int64_t)gmc) * P.lda3;
                ap_lds[it] = pl * CX::A_PLANE + mn_off<CX::RB>(a_r[it], hf * 8);
            } else {
                const int ch = (lin % 48) / 6, last = (P.a_cols + 15) / 16 - 1 - (m0 >> 4);
                a_r[it] = lin / 48;
                a_c[it] = min(ch, last) * 48 + pl * 16 + hf * 8;  // loads stay inside the row's planes
                a_ok[it] = ch <= last;  // chunks past the row's planes: zero
                ap_rp[it] = P.A3p;
                ap_lds[it] = pl * CX::A_PLANE + a_r[it] * CX::SA + (ch * 16 + hf * 8) * 2;
            }
            a_rp[it] = nullptr;
        } else if constexpr (CX::A16) {  // k row lin / (BM / 8), columns 8 (lin % (BM / 8)) .. + 7
            a_r[it] = lin / (BM / 8);
            a_c[it] = (lin % (BM / 8)) * 8;
            a_ok[it] = m0 + a_c[it] < P.a_cols;  // the copy is zero from a_cols to its row end
            a_rp[it] = nullptr;
        } else if (!AK) {
            a_r[it] = lin / (KT / 4);
            a_c[it] = (lin % (KT / 4)) * 4;
            const int gm = m0 + a_r[it];
            a_ok[it] = gm < M;
            const int gmc = min(gm, M - 1);
            a_rp[it] = P.A + (P.a_idx ? P.a_idx[gmc] : (int64_t)gmc) * P.lda;
        } else {
            a_r[it] = lin / (BM / 4);
            a_c[it] = (lin % (BM / 4)) * 4;
            a_ok[it] = true;
            a_rp[it] = P.A;
        }
    }
    int32_t* kidx = reinterpret_cast<int32_t*>(lds + 2 * CX::buf_bytes(PL));
    if (AK) {
        for (int k = tid; k < k_end - k_begin; k += kThreads)
            kidx[k] = (int32_t)(P.a_idx ? P.a_idx[k_begin + k] : (int64_t)(k_begin + k));
        __syncthreads();
    }
    const float* b_rp[CX::B_LOADS];
#pragma unroll
    for (int it = 0; it < CX::B_LOADS; ++it) {
        const int lin = tid + it * kThreads;
        if (!BKM) b_rp[it] = P.B + (int64_t)min(n0 + lin / (KT / 4), N - 1) * P.ldb + (lin % (KT / 4)) * 4;
        else b_rp[it] = P.B + (int64_t)(lin / (BN / 4)) * P.ldb + n0 + (lin % (BN / 4)) * 4;
    }
    const bool fast = ((k_end - k_begin) % KT == 0) && (n0 + BN <= N) &&
                      (AK ? (m0 + BM <= P.a_cols) : (m0 + BM <= M));

    f32x16 acc[I][J];
#pragma unroll
    for (int i = 0; i < I; ++i)
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    // weight gradients with b_colsum: the blocks of M-tile 0 sum the dY values they stage (the
    // bias gradient, written to C row M after the main loop)
    // (bf16 towers and pre-split X planes only: the fp32 split kernels take the bias gradient as an
    // implicit ones column of X — the column-sum registers pushed the 128 x 192 fp32 weight gradient
    // to 256 VGPRs with scratch spills, C2 +6 us per step, profiles/r06_s2_bisect.txt)
    constexpr bool CSUM = AK && BKM && (PL == 1 || CX::APL);
    const bool colsum = CSUM && P.b_colsum && tm == 0;
    float4 bsum[CSUM ? CX::B_LOADS : 1];
#pragma unroll
    for (int it = 0; it < (CSUM ? CX::B_LOADS : 1); ++it) bsum[it] = make_float4(0.f, 0.f, 0.f, 0.f);
    // 16-k tiles, and 32-k tiles (bf16) with at most four 32 x 32 accumulators per wave (128 x 128,
    // 128 x 96 tiles): two register sets, the k-tile two ahead in flight while the next one is
    // written to LDS between the current tile's MFMAs.  32-k tiles with more accumulators (128 x 192)
    // keep one set (the register budget), loaded at a step's start and written after its MFMAs —
    // one k-tile of MFMAs (8-12 per wave) cannot hide an HBM load, which left C5's bf16 GEMMs
    // latency-bound (build with -DTTAMM_BF16_DEEP=0 for one set everywhere)
    constexpr bool XDEEP = KT == 16 || (I * J <= 4 && TTAMM_BF16_DEEP);
    // A3: A in three register sets, loaded two k-tiles ahead (B, L2-resident weights or dY, one)
    constexpr bool A3 = XDEEP && CX::AD == 3;
    float4 ra[XDEEP ? (A3 ? 3 : 2) : 1][CX::A_LOADS], rb[XDEEP ? 2 : 1][CX::B_LOADS];

    auto mainloop = [&](auto fast_tag) {
        constexpr bool FAST = decltype(fast_tag)::value;
        auto load_a = [&](auto S, int k0) {
            constexpr int R = decltype(S)::value;
#pragma unroll
            for (int it = 0; it < CX::A_LOADS; ++it) {
                if constexpr (CX::APL) {
                    // one 16-B piece: MN-major, k-tile k0 / 16 of the row; K-major, k row k0 + a_r
                    // (clamped), chunks from the M-tile's first; masked when the tile is written
                    if (!AK) {
                        ra[R][it] = *reinterpret_cast<const float4*>(ap_rp[it] + (k0 >> 4) * 48 + a_c[it]);
                    } else {
                        const int k = FAST ? k0 + a_r[it] : min(k0 + a_r[it], k_end - 1);
                        const uint16_t* rp = P.A3p + (int64_t)kidx[k - k_begin] * P.lda3 + (m0 >> 4) * 48;
                        ra[R][it] = *reinterpret_cast<const float4*>(rp + a_c[it]);
                    }
                    continue;
                }
                if constexpr (CX::A16) {
                    const int k = FAST ? k0 + a_r[it] : min(k0 + a_r[it], k_end - 1);
                    const uint16_t* rp = P.A16 + (int64_t)kidx[k - k_begin] * P.lda16 + m0 + a_c[it];
                    ra[R][it] = (FAST || a_ok[it]) ? *reinterpret_cast<const float4*>(rp) : make_float4(0.f, 0.f, 0.f, 0.f);
                    continue;
                }
                if (!AK) {
                    ra[R][it] = FAST ? *reinterpret_cast<const float4*>(a_rp[it] + k0 + a_c[it])
                                     : raw4(a_rp[it], k0 + a_c[it], P.lda);
                } else {
                    const int k = FAST ? k0 + a_r[it] : min(k0 + a_r[it], k_end - 1);
                    const float* rp = P.A + (int64_t)kidx[k - k_begin] * P.lda;
                    ra[R][it] = FAST ? *reinterpret_cast<const float4*>(rp + m0 + a_c[it]) : raw4(rp, m0 + a_c[it], P.lda);
                }
            }
        };
        auto load_b = [&](auto S, int k0) {
            constexpr int R = decltype(S)::value;
#pragma unroll
            for (int it = 0; it < CX::B_LOADS; ++it) {
                const int lin = tid + it * kThreads;
                if (CX::B_F4 % kThreads && lin >= CX::B_F4) continue;  // partial last round (BN = 96)
                if (!BKM) {
                    rb[R][it] = FAST ? *reinterpret_cast<const float4*>(b_rp[it] + k0)
                                     : raw4(b_rp[it] - (lin % (KT / 4)) * 4, k0 + (lin % (KT / 4)) * 4, P.ldb);
                } else if (FAST) {
                    rb[R][it] = *reinterpret_cast<const float4*>(b_rp[it] + (int64_t)k0 * P.ldb);
                } else {
                    const int k = min(k0 + lin / (BN / 4), k_end - 1);
                    rb[R][it] = raw4(P.B + (int64_t)k * P.ldb, n0 + (lin % (BN / 4)) * 4, P.ldb);
                }
            }
        };
        auto load_tile = [&](auto S, int k0) {
            load_a(S, k0);
            load_b(S, k0);
        };
        // staged item q (A loads first, then B loads) of register sets SA (A) / SB (B) -> its
        // planes in buffer Buf
        // fresh: the k-tile is not a clamped repeat of the last one (kof) — its B values are summed once
        auto store_item2 = [&](auto SA, auto SB, auto Buf, int q, int k0, bool fresh) {
            constexpr int RA = decltype(SA)::value, RB = decltype(SB)::value;
            unsigned char* Ap = lds + decltype(Buf)::value * CX::buf_bytes(PL);
            unsigned char* Bp = Ap + PL * CX::A_PLANE;
            float4 v;
            int off;
            unsigned char* base;
            int plane;
            if (q < CX::A_LOADS) {
                const int it = q;
                if constexpr (CX::APL) {
                    // a pre-split piece: straight into its plane (rows past M / k rows past the split
                    // and chunks past the row's planes are zero)
                    unsigned char* Ap2 = lds + decltype(Buf)::value * CX::buf_bytes(PL);
                    const bool ok = AK ? (a_ok[it] && (FAST || k0 + a_r[it] < k_end)) : (FAST || a_ok[it]);
                    // a value select per component (a select of the two float4 objects compiled to a
                    // select of their addresses: both spilled to scratch)
                    const float4 r = ra[RA][it];
                    const float4 v = make_float4(ok ? r.x : 0.f, ok ? r.y : 0.f, ok ? r.z : 0.f, ok ? r.w : 0.f);
                    *reinterpret_cast<float4*>(Ap2 + ap_lds[it]) = v;
                    return;
                }
                if constexpr (CX::A16) {  // eight bf16 columns of k row a_r (zero past the split's rows)
                    const bool ok = FAST || k0 + a_r[it] < k_end;
                    const float4 r = ra[RA][it];
                    const float4 v = make_float4(ok ? r.x : 0.f, ok ? r.y : 0.f, ok ? r.z : 0.f, ok ? r.w : 0.f);
                    *reinterpret_cast<float4*>(Ap + a_r[it] * CX::SA + a_c[it] * 2) = v;
                    return;
                }
                if (!AK) {
                    v = FAST ? ra[RA][it] : mask4(ra[RA][it], k0 + a_c[it], k_end, P.lda, -1, a_ok[it]);
                    off = mn_off<CX::RB>(a_r[it], a_c[it]);
                } else {
                    v = FAST ? ra[RA][it]
                             : mask4(ra[RA][it], m0 + a_c[it], P.a_cols, P.lda, P.a_ones_col, k0 + a_r[it] < k_end);
                    off = a_r[it] * CX::SA + a_c[it] * 2;
                }
                base = Ap;
                plane = CX::A_PLANE;
            } else {
                const int it = q - CX::A_LOADS;
                const int lin = tid + it * kThreads;
                if (CX::B_F4 % kThreads && lin >= CX::B_F4) return;  // partial last round (BN = 96)
                if (!BKM) {
                    const int n = n0 + lin / (KT / 4), c = k0 + (lin % (KT / 4)) * 4;
                    v = FAST ? rb[RB][it] : mask4(rb[RB][it], c, k_end, P.ldb, -1, n < N);
                    off = mn_off<CX::RB>(lin / (KT / 4), (lin % (KT / 4)) * 4);
                } else {
                    const int kr = lin / (BN / 4), nc = (lin % (BN / 4)) * 4;
                    v = FAST ? rb[RB][it] : mask4(rb[RB][it], n0 + nc, N, P.ldb, -1, k0 + kr < k_end);
                    off = kr * CX::SB + nc * 2;
                    if constexpr (CSUM) {
                        if (colsum && fresh) {
                            float4 u = v;
                            if constexpr (PL == 1) {  // bf16 towers: the bias gradient sums bf16(dY)
                                const f32x4e x = {v.x, v.y, v.z, v.w};
                                const f32x4e r = __builtin_convertvector(__builtin_convertvector(x, bf16x4), f32x4e);
                                u = make_float4(r[0], r[1], r[2], r[3]);
                            }
                            bsum[it].x += u.x, bsum[it].y += u.y, bsum[it].z += u.z, bsum[it].w += u.w;
                        }
                    }
                }
                base = Bp;
                plane = CX::B_PLANE;
            }
            uint2 w[PL];
            split_bf16<PL>(v, w);
#pragma unroll
            for (int pl = 0; pl < PL; ++pl) *reinterpret_cast<uint2*>(base + pl * plane + off) = w[pl];
        };
        auto store_item = [&](auto S, auto Buf, int q, int k0, bool fresh) { store_item2(S, S, Buf, q, k0, fresh); };
        constexpr int NITEMS = CX::A_LOADS + CX::B_LOADS;
        auto store_tile = [&](auto S, auto Buf, int k0, bool fresh) {
#pragma unroll
            for (int q = 0; q < NITEMS; ++q) store_item(S, Buf, q, k0, fresh);
        };
        // multiply the k-tile in buffer Buf; the split + LDS writes of the next k-tile (register
        // set S -> buffer NB) are spread between the MFMA groups so the vector work issues in the
        // matrix pipe's shadow
        auto compute2 = [&](auto Buf, auto SA, auto SB, auto NB, int k0n, bool fresh) {
            const unsigned char* Ap = lds + decltype(Buf)::value * CX::buf_bytes(PL);
            const unsigned char* Bp = Ap + PL * CX::A_PLANE;
            constexpr int NP = I * J, KS = KT / 16, NSLOT = KS * NP;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                bf16x8 af[PL][I], bf[PL][J];
#pragma unroll
                for (int pl = 0; pl < PL; ++pl) {
#pragma unroll
                    for (int i = 0; i < I; ++i)
                        af[pl][i] = frag16<AK, CX::SA>(Ap + pl * CX::A_PLANE, wm * TM + i * 32, ks * 16, lane);
#pragma unroll
                    for (int j = 0; j < J; ++j)
                        bf[pl][j] = frag16<BKM, CX::SB>(Bp + pl * CX::B_PLANE, wn * TN + j * 32, ks * 16, lane);
                }
#pragma unroll
                for (int pq = 0; pq < NP; ++pq) {
                    const int i = pq / J, j = pq % J;
                    if constexpr (PL == 3 && TTAMM_SPLIT8) {  // developer: the 2^-24 terms ml, lm too
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1][i], bf[2][j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[2][i], bf[1][j], acc[i][j], 0, 0, 0);
                    }
                    if constexpr (PL == 3 && TTAMM_X_ABLATE != 2) {  // small terms first (ablation 2: hh only)
                        if constexpr (TTAMM_SPLIT_MM)  // mid x mid (<= 2^-18 relative; not kept by default)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1][i], bf[1][j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[2][i], bf[0][j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0][i], bf[2][j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1][i], bf[0][j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0][i], bf[1][j], acc[i][j], 0, 0, 0);
                    }
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0][i], bf[0][j], acc[i][j], 0, 0, 0);
#if TTAMM_X_ABLATE != 3
                    if constexpr (XDEEP) {
                        const int slot = ks * NP + pq;
#pragma unroll
                        for (int q = (slot * NITEMS) / NSLOT; q < ((slot + 1) * NITEMS) / NSLOT; ++q)
                            store_item2(SA, SB, NB, q, k0n, fresh);
                    }
#endif
                }
            }
        };
        auto compute = [&](auto Buf, auto S, auto NB, int k0n, bool fresh) { compute2(Buf, S, S, NB, k0n, fresh); };
        using S0 = std::integral_constant<int, 0>;
        using S1 = std::integral_constant<int, 1>;
        const int nk = k_end > k_begin ? (k_end - k_begin + KT - 1) / KT : 0;
        if (nk == 0) return;
        // tile index clamped to the last one: the loop body has no branches (the surplus loads and
        // writes at the end go to the free buffer and are never read)
        auto kof = [&](int kt) { return k_begin + min(kt, nk - 1) * KT; };
        if constexpr (!XDEEP) {
            load_tile(S0{}, kof(0));
            store_tile(S0{}, S0{}, kof(0), true);
            __syncthreads();
            auto sstep = [&](auto Buf, auto NB, int kt) {
#if TTAMM_X_ABLATE != 3
                load_tile(S0{}, kof(kt + 1));
#endif
                compute(Buf, S0{}, NB, kof(kt + 1), kt + 1 < nk);
#if TTAMM_X_ABLATE != 3
                store_tile(S0{}, NB, kof(kt + 1), kt + 1 < nk);
#endif
                __syncthreads();
            };
            int kt = 0;
            for (; kt + 1 < nk; kt += 2) {
                sstep(S0{}, S1{}, kt);
                sstep(S1{}, S0{}, kt + 1);
            }
            if (kt < nk) sstep(S0{}, S1{}, kt);
        } else if constexpr (A3) {
            // k-tile kt (i = kt mod 6): LDS buffer i & 1; A register set i mod 3, B set i & 1.  Step
            // kt loads A of kt + 3 into the A set tile kt left and B of kt + 2 into the B set tile kt
            // left (both already in LDS), multiplies kt while splitting kt + 1 (A set (i + 1) mod 3,
            // B set (i + 1) & 1) into the other buffer: A two k-tiles ahead, B one.
            using S2 = std::integral_constant<int, 2>;
            load_tile(S0{}, kof(0));
            store_tile(S0{}, S0{}, kof(0), true);
            load_tile(S1{}, kof(1));
            load_a(S2{}, kof(2));
            __syncthreads();
            auto step3 = [&](auto I6, int kt) {
                constexpr int i = decltype(I6)::value;
                using Buf = std::integral_constant<int, i & 1>;
                using NB = std::integral_constant<int, (i + 1) & 1>;
                using LA = std::integral_constant<int, i % 3>;
                using SA = std::integral_constant<int, (i + 1) % 3>;
#if TTAMM_X_ABLATE != 3
                load_a(LA{}, kof(kt + 3));
                load_b(Buf{}, kof(kt + 2));
#endif
                compute2(Buf{}, SA{}, NB{}, NB{}, kof(kt + 1), kt + 1 < nk);
                __syncthreads();
            };
            int kt = 0;
            for (; kt + 5 < nk; kt += 6) {
                step3(std::integral_constant<int, 0>{}, kt);
                step3(std::integral_constant<int, 1>{}, kt + 1);
                step3(std::integral_constant<int, 2>{}, kt + 2);
                step3(std::integral_constant<int, 3>{}, kt + 3);
                step3(std::integral_constant<int, 4>{}, kt + 4);
                step3(std::integral_constant<int, 5>{}, kt + 5);
            }
            if (kt < nk) step3(std::integral_constant<int, 0>{}, kt);
            if (kt + 1 < nk) step3(std::integral_constant<int, 1>{}, kt + 1);
            if (kt + 2 < nk) step3(std::integral_constant<int, 2>{}, kt + 2);
            if (kt + 3 < nk) step3(std::integral_constant<int, 3>{}, kt + 3);
            if (kt + 4 < nk) step3(std::integral_constant<int, 4>{}, kt + 4);
        } else {
            load_tile(S0{}, kof(0));
            store_tile(S0{}, S0{}, kof(0), true);
            load_tile(S1{}, kof(1));
            __syncthreads();
            // k-tile kt: register set kt & 1, LDS buffer kt & 1.  Prefetch kt + 2 into the set tile
            // kt left (already in LDS), multiply kt while splitting kt + 1 into the other buffer
            // (last read in k-tile kt - 1, before that tile's barrier).
            auto step = [&](auto Bf, auto NB, int kt) {
#if TTAMM_X_ABLATE != 3  // developer ablation 3: no k-loop traffic (MFMA + LDS reads only)
                load_tile(Bf, kof(kt + 2));
#endif
                compute(Bf, NB, NB, kof(kt + 1), kt + 1 < nk);
                __syncthreads();
            };
            int kt = 0;
            for (; kt + 1 < nk; kt += 2) {
                step(S0{}, S1{}, kt);
                step(S1{}, S0{}, kt + 1);
            }
            if (kt < nk) step(S0{}, S1{}, kt);
        }
    };
    if (fast) mainloop(std::true_type{});
    else mainloop(std::false_type{});

    if constexpr (CSUM) {
        // bias gradient of this split: the column sums of dY, reduced over the k rows of a tile in a
        // fixed order (every (k row, column) slot of the staging map belongs to one thread) and
        // written to row M of the split's slab
        static_assert(KT * BN * 4 <= CX::lds_bytes(PL), "column-sum scratch fits the staging LDS");
        if (colsum) {
            float* red = reinterpret_cast<float*>(lds);
            __syncthreads();
#pragma unroll
            for (int it = 0; it < CX::B_LOADS; ++it) {
                const int lin = tid + it * kThreads;
                if (CX::B_F4 % kThreads && lin >= CX::B_F4) continue;
                const int kr = lin / (BN / 4), nc = (lin % (BN / 4)) * 4;
                *reinterpret_cast<float4*>(red + kr * BN + nc) = bsum[it];
            }
            __syncthreads();
            for (int c = tid; c < BN; c += kThreads) {
                float acc_s = 0.f;
                for (int kr = 0; kr < KT; ++kr) acc_s += red[kr * BN + c];
                if (n0 + c < N) P.C[(int64_t)split * P.slab_stride + (int64_t)M * P.ldc + n0 + c] = acc_s;
            }
            __syncthreads();
        }
    }

    // ---- epilogue through LDS, in row slices (as gemm_kernel) ---------------------------------
    float* Cs = reinterpret_cast<float*>(lds);
    for (int ph = 0; ph < CX::EPI_PHASES; ++ph) {
        const int row_lo = ph * CX::EPI_ROWS;
        const int rows_here = min(CX::EPI_ROWS, BM - row_lo);
#pragma unroll
        for (int i = 0; i < I; ++i) {
            const int br = wm * TM + i * 32;
            if (br < row_lo || br >= row_lo + CX::EPI_ROWS) continue;
#pragma unroll
            for (int j = 0; j < J; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int rr = br - row_lo + (r & 3) + 8 * (r >> 2) + 4 * h;
                    Cs[rr * CX::CLD + wn * TN + j * 32 + li] = acc[i][j][r];
                }
        }
        __syncthreads();
        if constexpr (E == EPI_HIDDEN) {
            // 8 columns per thread: one dropout draw each (epilogue8_hidden)
            constexpr int C8 = BN / 8;
            constexpr int RSTEP8 = kThreads / C8;
            const int c8 = tid % C8, r8 = tid / C8;
            const int col = n0 + c8 * 8;
            if (r8 < RSTEP8 && col < N) {
                const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
                const float4 b0 = P.bias ? ld4(P.bias + col) : z4;
                const float4 b1 = (P.bias && col + 4 < N) ? ld4(P.bias + col + 4) : z4;
#pragma unroll 2
                for (int rr = r8; rr < rows_here; rr += RSTEP8) {
                    const int row = m0 + row_lo + rr;
                    if (row < M)
                        epilogue8_hidden(P, ld4(Cs + rr * CX::CLD + c8 * 8), ld4(Cs + rr * CX::CLD + c8 * 8 + 4), b0, b1,
                                         split, row, col);
                }
            }
        } else {
            constexpr int C4 = BN / 4;
            constexpr int RSTEP = kThreads / C4;
            const int c4 = tid % C4, r0 = tid / C4;
            const int col = n0 + c4 * 4;
            if (r0 < RSTEP && col < N) {
                const bool has_bias = (E == EPI_STORE || E == EPI_HIDDEN || E == EPI_GATE_HIDDEN || E == EPI_GATE_OUT) &&
                                      P.bias != nullptr;
                const float4 bias4 = has_bias ? ld4(P.bias + col) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 4
                for (int rr = r0; rr < rows_here; rr += RSTEP) {
                    const int row = m0 + row_lo + rr;
                    if (row < M) epilogue4<E>(P, ld4(Cs + rr * CX::CLD + c4 * 4), bias4, split, row, col);
                }
            }
        }
        __syncthreads();
    }
}

// ---- bf16-operand forward GEMM (C5 layer 1) --------------------------------------------------
// C[M, N] = epilogue(A16[M, K] . B16[N, K]^T) with both operands bf16 in HBM (the feature matrix
// converted once, the weight once per step; the same RNE-rounded values the fp32-staged
// variant forms in registers), v_mfma_f32_32x32x16_bf16, fp32 accumulation.
// 256 x 256 tiles, BK = 64, 512 threads = 8 waves as 2 (M) x 4 (N), each wave 128 x 64
// (4 x 2 MFMA blocks).  Operands are register-staged into double-buffered LDS images with
// 144-B rows (64 bf16 + 16 B pad: ds_read_b128 fragment reads hit distinct bank quads), one
// barrier per k-tile, the next k-tile's loads in flight during the current MFMAs.  Tiles are
// remapped so the N-tiles of one M-tile run on one XCD (shared A rows in its L2).
constexpr int kB16M = 256, kB16N = 256, kB16K = 64, kB16Threads = 512;
constexpr int kB16Ld = kB16K + 8;                               // LDS row stride, bf16 elements
constexpr int kB16Stage = (kB16M + kB16N) * kB16Ld;             // bf16 per buffer
constexpr int kB16EpiRows = 64;                                 // epilogue slice
constexpr int kB16Cld = kB16N + 4;
constexpr int kB16Lds = 2 * kB16Stage * 2 > kB16EpiRows * kB16Cld * 4 ? 2 * kB16Stage * 2 : kB16EpiRows * kB16Cld * 4;
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));


template <int E>
__global__ __launch_bounds__(kB16Threads) void gemm_bf16_kernel(GemmBatch batch) {
    __shared__ __attribute__((aligned(16))) unsigned char lds_raw[kB16Lds];
    uint16_t* lds = reinterpret_cast<uint16_t*>(lds_raw);
    const KArg(GemmBatch)* kb = (const KArg(GemmBatch)*)(__builtin_amdgcn_kernarg_segment_ptr());
    int tile = xcd_remap(blockIdx.x, kb->total_tiles);
    int pi = 0;
#pragma unroll 1
    for (int q = 1; q < kb->count; ++q)
        if (tile >= kb->p[q].tile_begin) pi = q;
    const KArg(GemmProblem)& P = kb->p[pi];
    tile -= P.tile_begin;
    const int tm = tile / P.tiles_n, tn = tile - tm * P.tiles_n;
    const int m0 = tm * kB16M, n0 = tn * kB16N;
    const int M = P.M, N = P.N, K = P.K;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 2, wn = wave & 3, li = lane & 31, h = lane >> 5;

    // staging: thread -> 4 A chunks and 4 B chunks of 16 B (row = c / 8, k chunk = c % 8)
    const uint16_t* a_rp[4];
    const uint16_t* b_rp[4];
    bool a_ok[4], b_ok[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int c = tid + i * kB16Threads, row = c >> 3;
        const int gm = m0 + row, gn = n0 + row;
        a_ok[i] = gm < M;
        b_ok[i] = gn < N;
        const int gmc = min(gm, M - 1), gnc = min(gn, N - 1);
        a_rp[i] = P.A16 + (P.a_idx ? P.a_idx[gmc] : (int64_t)gmc) * P.lda + (c & 7) * 8;
        b_rp[i] = P.B16 + (int64_t)gnc * P.ldb + (c & 7) * 8;
    }
    u32x4v ra[4], rb[4];
    const u32x4v zero4 = {0u, 0u, 0u, 0u};
    // unconditional loads from clamped in-bounds addresses, masked afterwards: a load under a
    // runtime condition makes hipcc branch around it and wait for it on the spot
    auto load = [&](int k0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int ch = ((tid + i * kB16Threads) & 7) * 8;
            const int kc = min(k0, K - 8 - ch);  // k0 + ch <= K - 8
            ra[i] = *reinterpret_cast<const u32x4v*>(a_rp[i] + kc);
            rb[i] = *reinterpret_cast<const u32x4v*>(b_rp[i] + kc);
        }
    };
    auto mask = [&](int k0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const bool in_k = k0 + ((tid + i * kB16Threads) & 7) * 8 < K;
            ra[i] = (a_ok[i] && in_k) ? ra[i] : zero4;
            rb[i] = (b_ok[i] && in_k) ? rb[i] : zero4;
        }
    };
    auto store = [&](int buf) {
        uint16_t* as = lds + buf * kB16Stage;
        uint16_t* bs = as + kB16M * kB16Ld;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int c = tid + i * kB16Threads, row = c >> 3, ch = (c & 7) * 8;
            *reinterpret_cast<u32x4v*>(as + row * kB16Ld + ch) = ra[i];
            *reinterpret_cast<u32x4v*>(bs + row * kB16Ld + ch) = rb[i];
        }
    };
    f32x16 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int nk = (K + kB16K - 1) / kB16K;
    load(0);
    mask(0);
    store(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
#if TTAMM_B16_ABLATE != 2  // developer ablation 2: no k-loop loads (MFMA + LDS only)
        if (kt + 1 < nk) load((kt + 1) * kB16K);  // in flight during this k-tile's MFMAs
#endif
        const uint16_t* as = lds + buf * kB16Stage;
        const uint16_t* bs = as + kB16M * kB16Ld;
#pragma unroll
        for (int ks = 0; ks < kB16K / 16; ++ks) {
            bf16x8 af[4], bfr[2];
#pragma unroll
            for (int i = 0; i < 4; ++i)
                af[i] = *reinterpret_cast<const bf16x8*>(as + (wm * 128 + i * 32 + li) * kB16Ld + ks * 16 + 8 * h);
#pragma unroll
            for (int j = 0; j < 2; ++j)
                bfr[j] = *reinterpret_cast<const bf16x8*>(bs + (wn * 64 + j * 32 + li) * kB16Ld + ks * 16 + 8 * h);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
        // the other buffer was last read in k-tile kt - 1, before that tile's barrier
        if (kt + 1 < nk) {
            mask((kt + 1) * kB16K);
            store(buf ^ 1);
        }
        __syncthreads();
    }

    // ---- epilogue: 64-row slices through LDS (the fp32 kernel's fused tails) ------------------
    float* Cs = reinterpret_cast<float*>(lds_raw);
    for (int ph = 0; ph < kB16M / kB16EpiRows; ++ph) {
        const int row_lo = ph * kB16EpiRows;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int br = wm * 128 + i * 32;
            if (br < row_lo || br >= row_lo + kB16EpiRows) continue;
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int rr = br - row_lo + (r & 3) + 8 * (r >> 2) + 4 * h;
                    Cs[rr * kB16Cld + wn * 64 + j * 32 + li] = acc[i][j][r];
                }
        }
        __syncthreads();
        if constexpr (E == EPI_HIDDEN) {
            // two rows per pass; lane pairs share the dropout draws (epilogue_hidden_pair)
            constexpr int C4 = kB16N / 4;
            constexpr int RSTEP = kB16Threads / C4;
            static_assert(C4 % 2 == 0, "lane pairs hold 8-column groups");
            const int c4 = tid % C4, r0 = tid / C4;
            const int col = n0 + c4 * 4;
            if (r0 < RSTEP && col < ((N + 7) & ~7)) {
                const float4 bias4 = (P.bias && col < N) ? ld4(P.bias + col) : make_float4(0.f, 0.f, 0.f, 0.f);
                const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 2
                for (int rr = r0; rr < kB16EpiRows; rr += 2 * RSTEP) {
                    const int rb_ = rr + RSTEP;
                    const int ra = m0 + row_lo + rr, rb = m0 + row_lo + rb_;
                    const bool in_b = rb_ < kB16EpiRows;
                    epilogue_hidden_pair(P, ld4(Cs + rr * kB16Cld + c4 * 4), in_b ? ld4(Cs + rb_ * kB16Cld + c4 * 4) : z4, bias4,
                                         0, ra, rb, ra < M && col < N, in_b && rb < M && col < N, col);
                }
            }
        } else {
            constexpr int C4 = kB16N / 4;              // 64 column groups
            constexpr int RSTEP = kB16Threads / C4;    // 8 rows per pass
            const int c4 = tid % C4, r0 = tid / C4;
            const int col = n0 + c4 * 4;
            if (col < N) {
                const bool has_bias = (E == EPI_STORE || E == EPI_HIDDEN || E == EPI_GATE_HIDDEN || E == EPI_GATE_OUT) &&
                                      P.bias != nullptr;
                const float4 bias4 = has_bias ? ld4(P.bias + col) : make_float4(0.f, 0.f, 0.f, 0.f);
    #pragma unroll 2
                for (int rr = r0; rr < kB16EpiRows; rr += RSTEP) {
                    const int row = m0 + row_lo + rr;
    #if TTAMM_B16_ABLATE == 1  // developer ablation 1: plain store instead of the fused tail
                    if (row < M) st4(P.C + (int64_t)row * P.ldc + col, ld4(Cs + rr * kB16Cld + c4 * 4));
    #else
                    if (row < M) epilogue4<E>(P, ld4(Cs + rr * kB16Cld + c4 * 4), bias4, 0, row, col);
    #endif
                }
            }
        }
        __syncthreads();
    }
}

__global__ void to_bf16_kernel(const float* __restrict__ src, int64_t rows, int cols, int64_t ld_src,
                               uint16_t* __restrict__ dst, int64_t ld_dst) {
    const int64_t total = rows * ld_dst;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / ld_dst;
        const int c = (int)(i - r * ld_dst);
        const __bf16 v = (__bf16)(c < cols ? src[r * ld_src + c] : 0.f);  // RNE
        dst[i] = __builtin_bit_cast(uint16_t, v);
    }
}

// fp32 rows -> bf16 planes: thread = 4 consecutive columns of a row; hi / mid / lo exactly as
// split_bf16 forms them in the GEMM's staging (so a pre-split operand multiplies bit-identically)
__global__ void to_planes_kernel(const float* __restrict__ src, int64_t rows, int cols, int64_t ld_src,
                                 uint16_t* __restrict__ dst, int64_t ld_dst, int kc) {
    const int64_t per_row = (int64_t)kc * 4;  // 4-column groups
    const int64_t total = rows * per_row;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / per_row;
        const int g = (int)(i - r * per_row), c0 = 4 * g;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = c0 + e < cols ? src[r * ld_src + c0 + e] : 0.f;
        uint2 w[3];
        split_bf16<3>(make_float4(v[0], v[1], v[2], v[3]), w);
        uint16_t* o = dst + r * ld_dst + (c0 >> 4) * 48 + (c0 & 15);
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) *reinterpret_cast<uint2*>(o + 16 * pl) = w[pl];
    }
}

// grad_w[m_out][n_in] = sum_s slab[s][n_in][m_out] ; grad_b[m_out] = sum_s slab[s][N_in][m_out]
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
    const int Mo = P.M;
    const int64_t plane = (int64_t)(P.N + 1) * Mo;
    const int n = (int)(off / Mo), m = (int)(off - (int64_t)n * Mo);
    // fixed summation order (split 0, 1, ...); the loads of 8 splits are issued before their adds
    float s = 0.f;
    const float* src = P.slab + off;
    int sp = 0;
    for (; sp + 8 <= P.splits; sp += 8) {
        float v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = src[(int64_t)(sp + i) * plane];
#pragma unroll
        for (int i = 0; i < 8; ++i) s += v[i];
    }
    for (; sp < P.splits; ++sp) s += src[(int64_t)sp * plane];
    if (n < P.N) P.grad_w[(int64_t)m * P.N + n] = s;
    else if (P.grad_b) P.grad_b[m] = s;
}

template <class CF, int E, bool BF>
int launch_one(GemmBatch& b, hipStream_t s) {
    int tiles = 0;
    for (int i = 0; i < b.count; ++i) {
        GemmProblem& p = b.p[i];
        p.tiles_m = (int)ceil_div(p.M, CF::BM);
        p.tiles_n = (int)ceil_div(p.N, CF::BN);
        if (p.k_split <= 0) p.k_split = p.K;
        p.tile_begin = tiles;
        tiles += p.tiles_m * p.tiles_n * (int)ceil_div(p.K, p.k_split);
    }
    b.total_tiles = tiles;
    if (tiles == 0) return TTAMM_OK;
    hipLaunchKernelGGL((gemm_kernel<CF, E, BF>), dim3(tiles), dim3(kThreads), 0, s, b);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

template <class CX, int E, int PL>
int launch_one_x(GemmBatch& b, hipStream_t s) {
    int tiles = 0;
    for (int i = 0; i < b.count; ++i) {
        GemmProblem& p = b.p[i];
        p.tiles_m = (int)ceil_div(p.M, CX::BM);
        p.tiles_n = (int)ceil_div(p.N, CX::BN);
        if (p.k_split <= 0) p.k_split = p.K;
        p.tile_begin = tiles;
        tiles += p.tiles_m * p.tiles_n * (int)ceil_div(p.K, p.k_split);
    }
    b.total_tiles = tiles;
    if (tiles == 0) return TTAMM_OK;
    hipLaunchKernelGGL((gemm_x_kernel<CX, E, PL>), dim3(tiles), dim3(kThreads), 0, s, b);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}
template <class CX, int PL>
int dispatch_epi_x(GemmBatch& b, hipStream_t s) {
    switch (b.p[0].epi) {
        case EPI_STORE: return launch_one_x<CX, EPI_STORE, PL>(b, s);
        case EPI_HIDDEN: return launch_one_x<CX, EPI_HIDDEN, PL>(b, s);
        case EPI_GATE_HIDDEN: return launch_one_x<CX, EPI_GATE_HIDDEN, PL>(b, s);
        case EPI_GATE_OUT: return launch_one_x<CX, EPI_GATE_OUT, PL>(b, s);
        case EPI_DGRAD_RELU: return launch_one_x<CX, EPI_DGRAD_RELU, PL>(b, s);
        case EPI_DGRAD_GATE_EF: return launch_one_x<CX, EPI_DGRAD_GATE_EF, PL>(b, s);
        case EPI_DGRAD_HIDDEN: return launch_one_x<CX, EPI_DGRAD_HIDDEN, PL>(b, s);
        default: return fail(TTAMM_E_INVALID, "gemm: unknown epilogue");
    }
}
// three planes on 16-k tiles (fp32 towers), or one plane on 32-k tiles (bf16 towers: twice the
// MFMAs per barrier, the same LDS footprint)
// fp32 towers, forward (weights MN-major): the A operand two k-tiles ahead (three register sets)
// unless TTAMM_GEMM_ADEEP=2.  Alone the layer-1 forward runs 3 % slower that way (105 -> 108 us,
// one spilled register), in the step beside the aux stream's gather and catch-up 6 % faster
// (129 -> 122 us; C2 0.650 -> 0.641-0.644 ms, profiles/r04_gemm_adeep_s29.txt).  dgrad (K-major
// weights, six k-tiles at C2) keeps two sets.
template <int BM, int BN, int WM, int WN, bool AK, bool BK>
int dispatch_x(GemmBatch& b, hipStream_t s) {
    static const bool adeep2 = [] {
        const char* e = dev_env("TTAMM_GEMM_ADEEP");
        return e && e[0] == '2';
    }();
    if (b.p[0].bf16) return dispatch_epi_x<XCfg<BM, BN, WM, WN, AK, BK, 32>, 1>(b, s);
    if (adeep2 || AK || BK) return dispatch_epi_x<XCfg<BM, BN, WM, WN, AK, BK, 16>, 3>(b, s);
    return dispatch_epi_x<XCfg<BM, BN, WM, WN, AK, BK, 16, 3>, 3>(b, s);
}
// Output tile width of a forward / dgrad launch: the width with the least padded output columns
// over the batch (ties: the first listed).  Layer widths that are multiples of 128 but not of 192
// (C4's 128 / 256, C5's 256 / 512) lost a third of the MFMA work to 128 x 192 tiles.  Latency-
// bound launches (dgrad, or few 128-row tiles) take the narrow set, which keeps more blocks.
int pick_tile_n(const GemmBatch& b, bool narrow, bool bf16) {
    static const bool legacy = [] {
        const char* e = dev_env("TTAMM_GEMM_TILES");
        return e && std::strcmp(e, "legacy") == 0;
    }();
    int maxN = 0;
    for (int i = 0; i < b.count; ++i) maxN = b.p[i].N > maxN ? b.p[i].N : maxN;
    if (maxN <= 96) return 96;
    if (legacy) return narrow ? 96 : 192;
    // (128 x 256 tiles were built and measured: the bf16 kernel spills 200-350 B of scratch per
    // thread at two waves per SIMD; two 128-wide tiles cover 256 with no padding)
    (void)bf16;
    static const int kNarrow[] = {96, 128};
    static const int kWide[] = {192, 128, 96};
    const int* c = narrow ? kNarrow : kWide;
    const int nc = narrow ? 2 : 3;
    int best = c[0];
    int64_t best_cols = -1;
    for (int j = 0; j < nc; ++j) {
        int64_t cols = 0;
        for (int i = 0; i < b.count; ++i) cols += ceil_div(b.p[i].M, 128) * ceil_div(b.p[i].N, c[j]) * c[j];
        if (best_cols < 0 || cols < best_cols) best_cols = cols, best = c[j];
    }
    return best;
}

// Matrix-core path of the fp32 / bf16 GEMMs: the split-bf16 kernel (default), or with
// TTAMM_FP32_MFMA=exact the v_mfma_f32_32x32x2_f32 kernel (exact fp32 products; bf16 towers
// round in registers) — a developer switch, read per launch so tests can compare the two.
bool exact_mfma() {
    const char* e = product_env("TTAMM_FP32_MFMA");
    return e && std::strcmp(e, "exact") == 0;
}

template <class CF, bool BF>
int dispatch_epi_t(GemmBatch& b, hipStream_t s) {
    switch (b.p[0].epi) {
        case EPI_STORE: return launch_one<CF, EPI_STORE, BF>(b, s);
        case EPI_HIDDEN: return launch_one<CF, EPI_HIDDEN, BF>(b, s);
        case EPI_GATE_HIDDEN: return launch_one<CF, EPI_GATE_HIDDEN, BF>(b, s);
        case EPI_GATE_OUT: return launch_one<CF, EPI_GATE_OUT, BF>(b, s);
        case EPI_DGRAD_RELU: return launch_one<CF, EPI_DGRAD_RELU, BF>(b, s);
        case EPI_DGRAD_GATE_EF: return launch_one<CF, EPI_DGRAD_GATE_EF, BF>(b, s);
        case EPI_DGRAD_HIDDEN: return launch_one<CF, EPI_DGRAD_HIDDEN, BF>(b, s);
        default: return fail(TTAMM_E_INVALID, "gemm: unknown epilogue");
    }
}
template <class CF>
int dispatch_epi(GemmBatch& b, hipStream_t s) {
    if constexpr (CF::MF == 16) return dispatch_epi_t<CF, false>(b, s);
    else return b.p[0].bf16 ? dispatch_epi_t<CF, true>(b, s) : dispatch_epi_t<CF, false>(b, s);
}

}  // namespace

int launch_gemm_bf16(GemmBatch& b, hipStream_t s) {
    int tiles = 0;
    for (int i = 0; i < b.count; ++i) {
        GemmProblem& p = b.p[i];
        TTAMM_REQUIRE(p.A16 && p.B16 && !p.b_kn && p.M >= 0 && p.N > 0 && p.K > 0 && p.epi == b.p[0].epi,
                      "gemm bf16: grouped NT problems with bf16 operands required");
        TTAMM_REQUIRE(p.lda % 8 == 0 && p.ldb % 8 == 0 && p.K % 8 == 0 && ((uintptr_t)p.A16 | (uintptr_t)p.B16) % 16 == 0,
                      "gemm bf16: 16-byte aligned rows with leading dims and K % 8 == 0");
        TTAMM_REQUIRE(p.N % 4 == 0 && p.ldc % 4 == 0 && (uintptr_t)p.C % 16 == 0, "gemm: output must be float4-aligned");
        p.tiles_m = (int)ceil_div(p.M, kB16M);
        p.tiles_n = (int)ceil_div(p.N, kB16N);
        p.k_split = p.K;
        p.slab_stride = 0;
        p.tile_begin = tiles;
        tiles += p.tiles_m * p.tiles_n;
    }
    b.total_tiles = tiles;
    if (tiles == 0) return TTAMM_OK;
    switch (b.p[0].epi) {
        case EPI_STORE: hipLaunchKernelGGL(gemm_bf16_kernel<EPI_STORE>, dim3(tiles), dim3(kB16Threads), 0, s, b); break;
        case EPI_HIDDEN: hipLaunchKernelGGL(gemm_bf16_kernel<EPI_HIDDEN>, dim3(tiles), dim3(kB16Threads), 0, s, b); break;
        default: return fail(TTAMM_E_INVALID, "gemm bf16: epilogue not supported");
    }
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

int launch_to_bf16(const float* src, int64_t rows, int cols, int64_t ld_src, uint16_t* dst, int64_t ld_dst,
                   hipStream_t s) {
    TTAMM_REQUIRE(rows >= 0 && cols >= 0 && ld_dst >= cols && ld_src >= cols, "to_bf16: bad shape");
    if (rows == 0 || ld_dst == 0) return TTAMM_OK;
    int64_t blocks = ceil_div(rows * ld_dst, 256);
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(to_bf16_kernel, dim3((unsigned)blocks), dim3(256), 0, s, src, rows, cols, ld_src, dst, ld_dst);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

int launch_to_planes(const float* src, int64_t rows, int cols, int64_t ld_src, uint16_t* dst, int64_t ld_dst,
                     hipStream_t s) {
    const int kc = (int)ceil_div(cols, 16);
    TTAMM_REQUIRE(rows >= 0 && cols >= 0 && ld_src >= cols && ld_dst >= 48 * (int64_t)kc && ld_dst % 8 == 0 &&
                      (uintptr_t)dst % 16 == 0,
                  "to_planes: bad shape (ld_dst >= 48 ceil(cols / 16), a multiple of 8, 16-byte aligned)");
    if (rows == 0 || kc == 0) return TTAMM_OK;
    int64_t blocks = ceil_div(rows * kc * 4, 256);
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(to_planes_kernel, dim3((unsigned)blocks), dim3(256), 0, s, src, rows, cols, ld_src, dst, ld_dst, kc);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

// the first feature layer on pre-split feature rows (GemmProblem::A3p): EPI_HIDDEN / EPI_STORE
template <int BN, int WM, int WN>
int dispatch_x_planes(GemmBatch& b, hipStream_t s) {
    using CX = XCfg<128, BN, WM, WN, false, false, 16, 3, true>;
    if (b.p[0].epi == EPI_HIDDEN) return launch_one_x<CX, EPI_HIDDEN, 3>(b, s);
    if (b.p[0].epi == EPI_STORE) return launch_one_x<CX, EPI_STORE, 3>(b, s);
    return fail(TTAMM_E_INVALID, "gemm: pre-split A planes take EPI_HIDDEN / EPI_STORE");
}

int launch_gemm(GemmBatch& b, hipStream_t s) {
    if (b.count == 0) return TTAMM_OK;
    if (b.p[0].A16) return launch_gemm_bf16(b, s);
    int maxN = 0;
    const int bkn = b.p[0].b_kn;
    for (int i = 0; i < b.count; ++i) {
        GemmProblem& p = b.p[i];
        TTAMM_REQUIRE(p.M >= 0 && p.N > 0 && p.K > 0, "gemm: bad shape");
        TTAMM_REQUIRE(p.epi == b.p[0].epi && p.b_kn == bkn && !p.a_kmaj && p.bf16 == b.p[0].bf16,
                      "gemm: grouped problems must share a variant");
        TTAMM_REQUIRE(p.lda % 4 == 0 && p.ldb % 4 == 0 && ((uintptr_t)p.A | (uintptr_t)p.B) % 16 == 0,
                      "gemm: operands must be 16-byte aligned with leading dims % 4 == 0");
        TTAMM_REQUIRE(p.N % 4 == 0 && p.ldc % 4 == 0 && (uintptr_t)p.C % 16 == 0, "gemm: output must be float4-aligned");
        p.k_split = p.K;
        p.slab_stride = 0;
        maxN = p.N > maxN ? p.N : maxN;
    }
    // wide outputs take 128 x 192 tiles unless that leaves most of the chip idle (in-batch steps
    // have R = 2B rows: C2 in-batch layer 1 is 128 such tiles for 256 CUs), or for dgrad; then
    // 128 x 96 tiles, twice the blocks for a second read of the A rows (TTAMM_GEMM_WIDE_TILES=1
    // keeps 128 x 192)
    int64_t wide_tiles = 0;
    for (int i = 0; i < b.count; ++i) wide_tiles += ceil_div(b.p[i].M, 128) * ceil_div(b.p[i].N, 192);
    // dgrad (K-major weights, K = one layer's width: six k-tiles at C2) is latency-bound: twice the
    // blocks on 128 x 96 tiles hide more of it (C2 0.638 -> 0.630-0.635 ms, profiles/r04_dgrad_tiles_s31.txt)
    const bool narrow_tiles = (wide_tiles < 300 || bkn) && dev_env("TTAMM_GEMM_WIDE_TILES") == nullptr;
    bool planes = b.p[0].A3p != nullptr && !exact_mfma() && !b.p[0].bf16 && !bkn;
    for (int i = 0; i < b.count; ++i) {
        const GemmProblem& p = b.p[i];
        planes = planes && p.A3p != nullptr && p.lda3 % 8 == 0 && (uintptr_t)p.A3p % 16 == 0 &&
                 p.lda3 >= 48 * ceil_div(p.K, 16);
    }
    if (planes) {
        switch (pick_tile_n(b, narrow_tiles, false)) {
            case 192: return dispatch_x_planes<192, 2, 2>(b, s);
            case 128: return dispatch_x_planes<128, 2, 2>(b, s);
            default: return dispatch_x_planes<96, 4, 1>(b, s);
        }
    }
    if (!exact_mfma()) {
        switch (pick_tile_n(b, narrow_tiles, b.p[0].bf16 != 0)) {
            case 192:
                if (bkn) return dispatch_x<128, 192, 2, 2, false, true>(b, s);
                return dispatch_x<128, 192, 2, 2, false, false>(b, s);
            case 128:
                if (bkn) return dispatch_x<128, 128, 2, 2, false, true>(b, s);
                return dispatch_x<128, 128, 2, 2, false, false>(b, s);
            default:
                if (bkn) return dispatch_x<128, 96, 4, 1, false, true>(b, s);
                return dispatch_x<128, 96, 4, 1, false, false>(b, s);
        }
    }
    if (maxN > 96) {
        if (bkn) return dispatch_epi<Cfg<128, 192, 2, 2, false, true>>(b, s);
        return dispatch_epi<Cfg<128, 192, 2, 2, false, false>>(b, s);
    }
    if (bkn) return dispatch_epi<Cfg<128, 96, 4, 1, false, true>>(b, s);
    return dispatch_epi<Cfg<128, 96, 4, 1, false, false>>(b, s);
}

namespace {
// Resident blocks of a wgrad launch config on this device (CUs x occupancy), cached.
using WgradWide = Cfg<128, 192, 2, 2, true, true>;
using WgradNarrow = Cfg<128, 96, 4, 1, true, true>;
using WgradWideX = XCfg<128, 192, 2, 2, true, true>;
using WgradNarrowX = XCfg<128, 96, 4, 1, true, true>;
// the narrow launch's X two k-tiles ahead (178 registers; the wide one would spill 38)
using WgradNarrowXA3 = XCfg<128, 96, 4, 1, true, true, 16, 3>;
using WgradWideX32 = XCfg<128, 192, 2, 2, true, true, 32>;
using WgradNarrowX32 = XCfg<128, 96, 4, 1, true, true, 32>;
using Wgrad128X = XCfg<128, 128, 2, 2, true, true>;
using Wgrad128X32 = XCfg<128, 128, 2, 2, true, true, 32>;
// bf16 weight gradients on 256 x 128 tiles (each wave 128 x 64, 8 accumulator tiles): with one
// plane the 128 x 128 tile (4 per wave) issued ~4 LDS instructions per MFMA (two transposed reads
// per fragment + the staging writes), so the LDS, not the MFMA, set its pace (C5,
// profiles/r05_s21_c5_gemm_sq.txt); 256 x 256 (16 per wave) spilled 444 B per thread
using Wgrad256X32 = XCfg<256, 128, 2, 2, true, true, 32>;
// bf16 X read from the towers' bf16 feature copy (WgradProblem::X16)
using Wgrad128X32A16 = XCfg<128, 128, 2, 2, true, true, 32, 2, false, true>;
using WgradWideX32A16 = XCfg<128, 192, 2, 2, true, true, 32, 2, false, true>;
// X pre-split into planes (the first feature layer's weight gradient, fp32 towers)
using WgradNarrowXP = XCfg<128, 96, 4, 1, true, true, 16, 2, true>;
using WgradWideXP = XCfg<128, 192, 2, 2, true, true, 16, 2, true>;
using Wgrad128XP = XCfg<128, 128, 2, 2, true, true, 16, 2, true>;
// resident blocks of a weight-gradient class's launch configuration (fp32 split kernels; the
// exact fp32-MFMA kernels have two classes)
int wgrad_slots(int cls, bool exact) {
    static int cached[2][kWgradClasses] = {};
    if (exact) cls = cls == 0 ? 0 : 1;
    if (cached[exact][cls]) return cached[exact][cls];
    int dev = 0, cus = 256, per_cu = 1;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const void* k = exact ? (cls ? (const void*)gemm_kernel<WgradWide, EPI_STORE, false>
                                 : (const void*)gemm_kernel<WgradNarrow, EPI_STORE, false>)
                          : cls == 0 ? (const void*)gemm_x_kernel<WgradNarrowX, EPI_STORE, 3>
                          : cls == 1 ? (const void*)gemm_x_kernel<WgradWideX, EPI_STORE, 3>
                                     : (const void*)gemm_x_kernel<Wgrad128X, EPI_STORE, 3>;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, kThreads, 0) != hipSuccess || per_cu < 1) per_cu = 1;
    cached[exact][cls] = cus * per_cu;
    return cached[exact][cls];
}
// output tile width of a class: 96, 192, 128, and class 3 (multiples of 256) on 128-wide tiles
constexpr int kWgradTileN[kWgradClasses] = {96, 192, 128, 128};
}  // namespace

// Rows per split-K chunk of a step's weight gradients, chosen per tile class (the wide and the
// narrow launch run one after the other): a multiple of 32 in [128, 1024] minimising the
// launch's makespan, (rounds of resident blocks) x (rows per block) x (measured time per row of
// a block), plus the fixed-order reduce over the slabs (splits x M x (N + 1) floats written and
// read at HBM speed).  Narrow gradients (M <= 96) are latency-bound per k-tile, so they want
// many short splits; wide ones fill the chip with few.
void wgrad_rows_per_split(const WgradShape* shapes, int n, int rps[kWgradClasses]) {
    // developer / test override (tests/test_step_parity_gpu.py covers splits past 512 rows)
    if (const char* e = dev_env("TTAMM_WGRAD_ROWS_PER_SPLIT")) {
        const int v = std::atoi(e);
        if (v >= BK && v <= kWgradMaxRowsPerSplit && v % BK == 0) {
            for (int c = 0; c < kWgradClasses; ++c) rps[c] = v;
            return;
        }
    }
    const bool exact = exact_mfma();
    // block time per split row (MI355X; 96 / 192 measured at C2, 128 / 256 scaled by tile width)
    const double us_per_row[kWgradClasses] = {0.11, 0.14, 0.12, 0.12};
    const double hbm_us_per_byte = 1.0 / 5.0e6;  // ~5 TB/s
    for (int c = 0; c < kWgradClasses; ++c) {
        int best = 512;
        double best_cost = -1.0;
        for (int r = 128; r <= kWgradMaxRowsPerSplit; r += 32) {
            int64_t tiles = 0;
            double slab_bytes = 0.0;
            for (int i = 0; i < n; ++i) {
                if (shapes[i].R <= 0 || wgrad_class(shapes[i].M) != c) continue;
                const int64_t splits = ceil_div(shapes[i].R, r);
                tiles += ceil_div(shapes[i].N + 1, 128) * ceil_div(shapes[i].M, kWgradTileN[c]) * splits;
                slab_bytes += 2.0 * 4.0 * (double)splits * shapes[i].M * (shapes[i].N + 1);
            }
            if (tiles == 0) break;
            const double cost = (double)ceil_div(tiles, wgrad_slots(c, exact)) * r * us_per_row[c] +
                                slab_bytes * hbm_us_per_byte;
            if (best_cost < 0.0 || cost < best_cost) {
                best_cost = cost;
                best = r;
            }
        }
        rps[c] = best;
        // developer: one class's rows per split (TTAMM_WGRAD_RPS0 narrow, 1 wide, 2 / 3 128-wide)
        if constexpr (kDevKnobs) {
            char name[] = "TTAMM_WGRAD_RPS0";
            name[sizeof(name) - 2] = (char)('0' + c);
            if (const char* e = dev_env(name)) {
                const int v = std::atoi(e);
                if (v >= BK && v <= kWgradMaxRowsPerSplit && v % BK == 0) rps[c] = v;
            }
        }
    }
}

size_t wgrad_slab_floats(int R, int M, int N, int rps) {
    const int splits = R > 0 ? (int)ceil_div(R, rps) : 1;
    return (size_t)splits * M * (N + 1);
}

int wgrad_class(int m_out) {
    static const bool all_narrow = dev_env("TTAMM_WGRAD_ALL_NARROW") != nullptr;
    static const bool legacy = [] {
        const char* e = dev_env("TTAMM_GEMM_TILES");
        return e && std::strcmp(e, "legacy") == 0;
    }();
    if (all_narrow || m_out <= 96) return 0;
    if (legacy) return 1;
    auto pad = [&](int bn) { return ceil_div(m_out, bn) * bn; };
    int best = 1;  // 192
    int64_t bp = pad(192);
    if (pad(256) < bp) best = 3, bp = pad(256);
    if (pad(128) < bp) best = 2, bp = pad(128);
    return best;
}

// TTAMM_WGRAD_ADEEP=3: the narrow weight-gradient launch's X operand two k-tiles ahead
static bool wgrad_a3() {
    static const bool on = [] {
        const char* e = dev_env("TTAMM_WGRAD_ADEEP");
        return e && e[0] == '3';
    }();
    return on;
}

// Weight gradients as C = X^T dY (M = n_in + 1 incl. the ones column, N = m_out, K = rows),
// both operands K-major; one launch per tile configuration, then one fixed-order reduce.
int launch_wgrad(WgradBatch& wb, hipStream_t s, void* const* ev) {
    // one launch per tile configuration: class 0 (128 x 96), 1 (128 x 192), 2 and 3 (128 x 128; a
    // 128 x 256 bf16 tile spilled 132 B of scratch per thread)
    GemmBatch g[kWgradClasses], gp[kWgradClasses];  // gp: X pre-split into planes, or (bf16) X in bf16
    std::memset(g, 0, sizeof(g));
    std::memset(gp, 0, sizeof(gp));
    const bool bf = wb.count > 0 && wb.p[0].bf16;
    const bool exact = exact_mfma();
    // TTAMM_BF16_WGRAD256=1: bf16 weight gradients of the 128-wide classes on 256 x 256 tiles (cfg 3)
    const char* e256 = dev_env("TTAMM_BF16_WGRAD256");
    const bool w256 = e256 && e256[0] == '1';
    auto cfg_of = [&](int cls) {
        if (exact) return cls == 0 ? 0 : 1;  // the fp32-MFMA kernels: narrow / wide
        if (bf && w256 && cls >= 2) return 3;
        return cls == 3 ? 2 : cls;
    };
    auto flush = [&](GemmBatch& b, int cfg, bool planes = false) -> int {
        if (b.count == 0) return TTAMM_OK;
        int rc;
        if (planes && bf) {  // X16 (cfg 1 / 2 only)
            rc = cfg == 1 ? launch_one_x<WgradWideX32A16, EPI_STORE, 1>(b, s)
                          : launch_one_x<Wgrad128X32A16, EPI_STORE, 1>(b, s);
        } else if (planes) {
            rc = cfg == 0   ? launch_one_x<WgradNarrowXP, EPI_STORE, 3>(b, s)
                 : cfg == 1 ? launch_one_x<WgradWideXP, EPI_STORE, 3>(b, s)
                            : launch_one_x<Wgrad128XP, EPI_STORE, 3>(b, s);
        } else if (exact) {
            rc = cfg ? (bf ? launch_one<WgradWide, EPI_STORE, true>(b, s) : launch_one<WgradWide, EPI_STORE, false>(b, s))
                     : (bf ? launch_one<WgradNarrow, EPI_STORE, true>(b, s) : launch_one<WgradNarrow, EPI_STORE, false>(b, s));
        } else if (bf) {
            rc = cfg == 0   ? launch_one_x<WgradNarrowX32, EPI_STORE, 1>(b, s)
                 : cfg == 1 ? launch_one_x<WgradWideX32, EPI_STORE, 1>(b, s)
                 : cfg == 3 ? launch_one_x<Wgrad256X32, EPI_STORE, 1>(b, s)
                            : launch_one_x<Wgrad128X32, EPI_STORE, 1>(b, s);
        } else {
            rc = cfg == 0   ? (wgrad_a3() ? launch_one_x<WgradNarrowXA3, EPI_STORE, 3>(b, s)
                                          : launch_one_x<WgradNarrowX, EPI_STORE, 3>(b, s))
                 : cfg == 1 ? launch_one_x<WgradWideX, EPI_STORE, 3>(b, s)
                            : launch_one_x<Wgrad128X, EPI_STORE, 3>(b, s);
        }
        std::memset(&b, 0, sizeof(b));
        return rc;
    };
    int64_t total = 0;
    for (int i = 0; i < wb.count; ++i) {
        WgradProblem& w = wb.p[i];
        TTAMM_REQUIRE(w.rows_per_split > 0 && w.rows_per_split % BK == 0 && w.rows_per_split <= kWgradMaxRowsPerSplit,
                      "wgrad: rows_per_split must be a multiple of 16 and at most 1024");
        TTAMM_REQUIRE(w.bf16 == wb.p[0].bf16, "wgrad: the batch must share one matmul precision");
        w.splits = w.R > 0 ? (int)ceil_div(w.R, w.rows_per_split) : 1;
        total += (int64_t)w.M * (w.N + 1);
        if (w.R <= 0) {  // no rows: the slab (one split) is zero
            TTAMM_HIP(hipMemsetAsync(w.slab, 0, sizeof(float) * w.M * (w.N + 1), s));
            continue;
        }
        TTAMM_REQUIRE(w.ld_x % 4 == 0 && w.ld_dy % 4 == 0 && ((uintptr_t)w.X | (uintptr_t)w.dY) % 16 == 0,
                      "wgrad: operands must be 16-byte aligned with leading dims % 4 == 0");
        GemmProblem p;
        std::memset(&p, 0, sizeof(p));
        p.A = w.X;
        p.a_idx = w.x_idx;
        p.lda = w.ld_x;
        p.a_kmaj = 1;
        p.a_cols = w.N;
        p.B = w.dY;
        p.ldb = w.ld_dy;
        p.b_kn = 1;
        // bf16 / pre-split-plane kernels: the bias gradient as column sums of dY in the M-tile-0
        // blocks (b_colsum), so M = n_in; the fp32 split and fp32-MFMA kernels: the implicit ones
        // column (M = n_in + 1)
        p.b_colsum = 0;
        p.a_ones_col = w.N;
        p.M = w.N + 1;
        p.N = w.M;
        p.K = w.R;
        p.k_split = w.rows_per_split;
        p.epi = EPI_STORE;
        p.C = w.slab;
        p.ldc = w.M;
        p.slab_stride = (int64_t)(w.N + 1) * w.M;
        p.keep_prob = 1.f;
        p.inv_keep = 1.f;
        p.bf16 = w.bf16;
        const int cfg = cfg_of(wgrad_class(w.M));
        bool planes = w.X3p != nullptr && !exact && !bf && w.ld_x3 % 8 == 0 && (uintptr_t)w.X3p % 16 == 0 &&
                      w.ld_x3 >= 48 * ceil_div(w.N, 16);
        if (planes) {
            p.A3p = w.X3p;
            p.lda3 = w.ld_x3;
        }
        if (!exact && (bf || planes)) {  // (the column-sum kernels: see gemm_x_kernel CSUM)
            p.b_colsum = 1;
            p.a_ones_col = -1;
            p.M = w.N;
        }
        if (bf && w.X16 && (cfg == 1 || cfg == 2) && w.ld_x16 % 8 == 0 && w.ld_x16 >= 8 * ceil_div(w.N, 8) &&
            (uintptr_t)w.X16 % 16 == 0) {
            planes = true;  // (the gp group: X from its bf16 copy)
            p.A16 = w.X16;
            p.lda16 = w.ld_x16;
        }
        GemmBatch& gb = planes ? gp[cfg] : g[cfg];
        if (gb.count == kMaxGemmProblems) {
            const int rc = flush(gb, cfg, planes);
            if (rc) return rc;
        }
        gb.p[gb.count++] = p;
    }
    int rc;
    bool any_wide = false;
    for (int c = 1; c < kWgradClasses; ++c) any_wide = any_wide || g[c].count > 0 || gp[c].count > 0;
    const bool timed = ev && ev[0] && ev[1] && any_wide;
    // The narrow launch (latency-bound: many short splits) first, then the wide ones (MFMA-bound),
    // which the aux stream's memory-bound row updates then run beside: C2 0.660 -> 0.652 ms,
    // the emulated 8-rank C2 0.804 -> 0.769 ms (profiles/r04_wgrad_order_s22.txt).
    // TTAMM_WGRAD_WIDE_FIRST=1: the old order.
    static const bool narrow_first = dev_env("TTAMM_WGRAD_WIDE_FIRST") == nullptr;
    if (narrow_first && ((rc = flush(g[0], 0)) || (rc = flush(gp[0], 0, true)))) return rc;
    if (timed) TTAMM_HIP(hipEventRecord((hipEvent_t)ev[0], s));
    for (int c = 1; c < kWgradClasses; ++c)
        if ((rc = flush(gp[c], c, true)) || (rc = flush(g[c], c))) return rc;
    if (timed) TTAMM_HIP(hipEventRecord((hipEvent_t)ev[1], s));
    if (!narrow_first && ((rc = flush(g[0], 0)) || (rc = flush(gp[0], 0, true)))) return rc;
    if (total > 0) {
        hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)ceil_div(total, 256)), dim3(256), 0, s, wb, total);
        TTAMM_LAUNCH_CHECK();
    }
    return TTAMM_OK;
}

}  // namespace ttamm
