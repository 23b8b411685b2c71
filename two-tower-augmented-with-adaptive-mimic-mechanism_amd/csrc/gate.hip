// Fused FeatureFusionGate forward and backward for fp32 towers (encoders.py:149-168, applied
// at :246-253; the adaptive-mimic augment of adaptive_mimic.py:88-95 rides in the forward
// epilogue).  Per row, with ef = [e | f] (ID row | feature-MLP output):
//
//   forward   z = relu(ef G1^T + c1)            [Hg]
//             g = sigmoid(z G2^T + c2)          [D]
//             t = g e + (1 - g) f ; a = A[idx] ; aug = t + a
//   backward  dq  = (dT e - dT f) (1 - g) g     (SigmoidBackward of the mix, as gate_dq_kernel)
//             dz  = (dq G2) * (z > 0)
//             dEF = dz G1 + [dT g | dT (1 - g)]
//
// The generic path runs these as two GEMM launches (forward) / an elementwise kernel and two
// GEMM launches (backward) that round-trip z, dq and dz through HBM and re-read ef; here each
// wave owns 16 rows and chains the two GEMMs in registers.  The gate matrices are small
// (Hg x 2D, D x Hg), so one persistent block per CU stages them in LDS once and its 8 waves
// stream 16-row slabs (the next slab's rows prefetched during the current one).
//
// MFMA orientation: v_mfma_f32_16x16x4_f32 computes OUT^T = W . X^T (the weights as the A
// operand, the slab's 16 rows as the columns).  Lane l (li = l & 15, q = l >> 4) then holds
// OUT[row li][feature 16*ob + 4q + r] in register r of output tile ob — four consecutive
// features of one row, one float4 in memory — and that is exactly the B fragment of the next
// GEMM when its k-steps are permuted so that step (t, r) covers k = 16t + 4q + r (lane group q
// supplies k-slot q).  The A fragment of that step is W[16*ob + li][16t + 4q + r]: four
// consecutive floats of an LDS row, one ds_read_b128 per four MFMAs.  All four r-steps of a
// k-tile are issued across the output tiles, so consecutive MFMAs never share an accumulator.
#include <cstdlib>

#include "kernels.h"

namespace ttamm {

namespace {

typedef float f4v __attribute__((ext_vector_type(4)));
// D <= 96: 512 threads, 2 waves per SIMD with up to 256 VGPRs each — a wave keeps its slab's
// rows, the next slab's prefetched rows and the MFMA operands of both chained GEMMs in registers.
// D = 128: the fp32 G1 (or G1^T) alone fills 133 KB of LDS, so the narrower matrix (G2, D x Hg)
// is read from global memory (L2-resident: 64 KB read by every wave) and a block is 4 waves, one
// per SIMD with the whole register file (VGPRs + AGPRs), one block per CU.
template <int D>
struct GateWaves {
    static constexpr int NW = D >= 128 ? 4 : 8;
    static constexpr int THREADS = 64 * NW;
};

__device__ __forceinline__ f4v ldg4(const float* p) { return *reinterpret_cast<const f4v*>(p); }
__device__ __forceinline__ f4v lds4(const float* p) { return *reinterpret_cast<const f4v*>(p); }
__device__ __forceinline__ void stg4(float* p, f4v v) { store_nt(p, make_float4(v[0], v[1], v[2], v[3])); }
__device__ __forceinline__ float sigmoid_(float x) { return 1.0f / (1.0f + __expf(-x)); }

// acc[ob] += W[16 (ob0 + ob) + li][16 t + 4 q + r] * b[t][r] over k-tiles t < NK
// The A fragments of k-tile t + 1 are read from LDS while k-tile t's MFMAs issue (two register
// sets), so the MFMA chain does not stop for an LDS round trip at every k-tile.
template <int NO, int NK, int LD>
__device__ __forceinline__ void tile_gemm(const float* w_lds, int ob0, const f4v (&b)[NK], f4v (&acc)[NO], int li,
                                          int q) {
    f4v w[2][NO];
    const float* base = w_lds + (16 * ob0 + li) * LD + 4 * q;
#pragma unroll
    for (int ob = 0; ob < NO; ++ob) w[0][ob] = lds4(base + 16 * ob * LD);
#pragma unroll
    for (int t = 0; t < NK; ++t) {
        const int cur = t & 1;
        if (t + 1 < NK) {
#pragma unroll
            for (int ob = 0; ob < NO; ++ob) w[cur ^ 1][ob] = lds4(base + 16 * ob * LD + 16 * (t + 1));
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int ob = 0; ob < NO; ++ob)
                acc[ob] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[cur][ob][r], b[t][r], acc[ob], 0, 0, 0);
        // keep the scheduler from hoisting every k-tile's LDS reads to the top (register spills)
        __builtin_amdgcn_sched_barrier(0);
    }
}

// tile_gemm with W read from global memory (row-major, leading dimension ld; L2-resident), the
// fragments of k-tile t + 1 in flight during k-tile t's MFMAs
template <int NO, int NK, int ld>
__device__ __forceinline__ void tile_gemm_g(const float* W, int ob0, const f4v (&b)[NK], f4v (&acc)[NO], int li,
                                            int q) {
    f4v w[2][NO];
    const float* base = W + (int64_t)(16 * ob0 + li) * ld + 4 * q;
#pragma unroll
    for (int ob = 0; ob < NO; ++ob) w[0][ob] = *reinterpret_cast<const f4v*>(base + 16 * ob * ld);
#pragma unroll
    for (int t = 0; t < NK; ++t) {
        const int cur = t & 1;
        if (t + 1 < NK) {
#pragma unroll
            for (int ob = 0; ob < NO; ++ob)
                w[cur ^ 1][ob] = *reinterpret_cast<const f4v*>(base + 16 * ob * ld + 16 * (t + 1));
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int ob = 0; ob < NO; ++ob)
                acc[ob] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[cur][ob][r], b[t][r], acc[ob], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// ---- split-bf16 form of the wider GEMM of each direction (G1 forward, G1^T backward) ----------
// The fp32 weight is staged once per block as three bf16 planes (hi, mid, lo: hi + mid + lo = w
// exactly, gemm.hip split_bf16) and each product is six v_mfma_f32_16x16x32_bf16 (hh, hm, mh,
// hl, lh, mm), accumulated in fp32: 6 x 16 cycles per 16 x 16 x 32 step against 8 x 32 cycles of
// v_mfma_f32_16x16x4_f32 for the same product.  The 32 k-slots of step t are, for lane group q,
// columns {32 t + 4 q + j, 32 t + 16 + 4 q + j : j < 4} — exactly the two float4s the lane holds
// from load_row (its k-tiles 2t and 2t + 1) — so the B operand is the lane's own registers,
// split in place, and the weight planes are laid out [t][q][row][8 slots] (one ds_read_b128 per
// plane and fragment, 16 lanes reading 256 contiguous bytes).
typedef __bf16 g_bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 g_bf16x4 __attribute__((ext_vector_type(4)));
typedef float g_f32x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void split8(f4v a, f4v b, g_bf16x8& h, g_bf16x8& m, g_bf16x8& l) {
    const g_f32x8 x = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    h = __builtin_convertvector(x, g_bf16x8);
    const g_f32x8 r = x - __builtin_convertvector(h, g_f32x8);
    m = __builtin_convertvector(r, g_bf16x8);
    l = __builtin_convertvector(r - __builtin_convertvector(m, g_f32x8), g_bf16x8);
}

// byte offset of slot (t, q, j) of weight row f in one plane of an [NT][4][NF][8] image
template <int NF>
__device__ __forceinline__ int xw_off(int t, int q, int f, int j) {
    return ((t * 4 + q) * NF + f) * 16 + j * 2;
}
// slot of k index c (k-step t, lane group q, slot j)
__device__ __forceinline__ void xw_slot(int c, int& t, int& q, int& j) {
    t = c >> 5;
    const int r = c & 31;
    q = (r & 15) >> 2;
    j = ((r >> 4) << 2) | (r & 3);
}
// split 4 consecutive weights (the same t, q, consecutive j) into the three planes
template <int NF, int PLANE>
__device__ __forceinline__ void xw_store4(unsigned char* img, int t, int q, int f, int j0, f4v w) {
    const f4v hf = w;
    const g_bf16x4 h = __builtin_convertvector(hf, g_bf16x4);
    const f4v r = hf - __builtin_convertvector(h, f4v);
    const g_bf16x4 m = __builtin_convertvector(r, g_bf16x4);
    const g_bf16x4 l = __builtin_convertvector(r - __builtin_convertvector(m, f4v), g_bf16x4);
    const int off = xw_off<NF>(t, q, f, j0);
    *reinterpret_cast<g_bf16x4*>(img + off) = h;
    *reinterpret_cast<g_bf16x4*>(img + PLANE + off) = m;
    *reinterpret_cast<g_bf16x4*>(img + 2 * PLANE + off) = l;
}

// acc[ob] += W[16 (ob0 + ob) + li][k] * b[k] over the NT k-steps of 32 (b: 2 NT float4s of the
// lane, load_row layout), W from its three-plane image ([NT][4][NF][8] bf16 per plane)
template <int NO, int NT, int NF>
__device__ __forceinline__ void tile_gemm_x(const unsigned char* img, int ob0, const f4v* b, f4v (&acc)[NO], int li,
                                            int q) {
    constexpr int PLANE = NT * 4 * NF * 16;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        g_bf16x8 bh, bm, bl;
        split8(b[2 * t], b[2 * t + 1], bh, bm, bl);
        const unsigned char* base = img + xw_off<NF>(t, q, 16 * ob0 + li, 0);
#pragma unroll
        for (int ob = 0; ob < NO; ++ob) {
            const unsigned char* p = base + ob * 16 * 16;
            const g_bf16x8 ah = *reinterpret_cast<const g_bf16x8*>(p);
            const g_bf16x8 am = *reinterpret_cast<const g_bf16x8*>(p + PLANE);
            const g_bf16x8 al = *reinterpret_cast<const g_bf16x8*>(p + 2 * PLANE);
            acc[ob] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bm, acc[ob], 0, 0, 0);  // small terms first
            acc[ob] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc[ob], 0, 0, 0);
            acc[ob] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc[ob], 0, 0, 0);
            acc[ob] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bh, acc[ob], 0, 0, 0);
            acc[ob] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bm, acc[ob], 0, 0, 0);
            acc[ob] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc[ob], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <int N>
__device__ __forceinline__ void zero(f4v (&a)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) a[i] = f4v{0.f, 0.f, 0.f, 0.f};
}

// lane (li, q)'s part of row `row` of a [*, ld] matrix: columns 16 t + 4 q .. + 3, t < N
template <int N>
__device__ __forceinline__ void load_row(f4v (&v)[N], const float* base, int64_t ld, int64_t row, int q) {
    const float* p = base + row * ld + 4 * q;
#pragma unroll
    for (int t = 0; t < N; ++t) v[t] = ldg4(p + 16 * t);
}

// Row-contiguous stores of a slab's [16 rows x 16 NO] block held in the MFMA output layout
// (lane (li, q): row li, columns 16 ob + 4 q .. + 3, one float4 per ob): through the wave's LDS
// scratch, eight rows at a time, so a store instruction writes whole row segments (1 KB per
// instruction at NO = 6) instead of 16 rows x 64 B.  The direct form of these stores bounded the
// gate kernels (their time without any output store: 64 -> 42 us forward, 65 -> 49 us backward,
// profiles/r03_c2_gate_store_ablation_s22.txt).
// floats per wave: eight rows of up to max(D, Hg) + 4 pad
template <int D>
constexpr int slab_scratch() { return 8 * ((D < 96 ? 96 : D) + 4); }
template <int NO>
__device__ __forceinline__ void store_slab(float* scr, const f4v (&v)[NO], float* out, int64_t ld, int64_t row0,
                                           int64_t R, int lane) {
    constexpr int W = 16 * NO, LDW = W + 4, C4 = W / 4, PER = 8 * C4 / 64;
    static_assert((8 * C4) % 64 == 0, "slab scratch");
    const int li = lane & 15, q = lane >> 4;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        if ((li >> 3) == half) {
#pragma unroll
            for (int ob = 0; ob < NO; ++ob) *reinterpret_cast<f4v*>(scr + (li & 7) * LDW + 16 * ob + 4 * q) = v[ob];
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes are done
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int idx = lane + 64 * k, r = idx / C4, c = idx - r * C4;
            const f4v val = *reinterpret_cast<const f4v*>(scr + r * LDW + 4 * c);
            const int64_t grow = row0 + 8 * half + r;
            if (grow < R) stg4(out + grow * ld + 4 * c, val);
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // the reads are done before the next half's writes
        __builtin_amdgcn_wave_barrier();
    }
}

// store_slab into compact exchange rows (GateTower::xu): slab row grow goes to out + u * 16 NO for
// u = xu[grow] (a positive) or ~xu[grow] (a negative; left out when pos_only).  xu_li: this lane's
// row's xu[row0 + (lane & 15)], loaded ahead by the caller (a store's row takes it by shuffle)
template <int NO>
__device__ __forceinline__ void store_slab_xu(float* scr, const f4v (&v)[NO], float* out, int xu_li,
                                              bool pos_only, int64_t row0, int64_t R, int lane) {
    constexpr int W = 16 * NO, LDW = W + 4, C4 = W / 4, PER = 8 * C4 / 64;
    static_assert((8 * C4) % 64 == 0, "slab scratch");
    const int li = lane & 15, q = lane >> 4;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        if ((li >> 3) == half) {
#pragma unroll
            for (int ob = 0; ob < NO; ++ob) *reinterpret_cast<f4v*>(scr + (li & 7) * LDW + 16 * ob + 4 * q) = v[ob];
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int idx = lane + 64 * k, r = idx / C4, c = idx - r * C4;
            const f4v val = *reinterpret_cast<const f4v*>(scr + r * LDW + 4 * c);
            const int64_t grow = row0 + 8 * half + r;
            const int u = __shfl(xu_li, 8 * half + r, 64);
            if (grow < R && (u >= 0 || !pos_only)) stg4(out + (int64_t)(u >= 0 ? u : ~u) * W + 4 * c, val);
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
    }
}

// lane (li, q)'s part of a dT row: row `row` at ld, or its compact exchange unit (GateTower::xu)
template <int N>
__device__ __forceinline__ void load_dt_row(f4v (&v)[N], const float* base, int64_t ld, const int64_t* xu, int D,
                                            int64_t row, int q) {
    if (xu) {
        const int64_t u = xu[row];
        load_row(v, base, D, u >= 0 ? u : ~u, q);
    } else {
        load_row(v, base, ld, row, q);
    }
}

template <int D, int HG, int NW_ = GateWaves<D>::NW>
struct GateCfg {
    static constexpr int TD = D / 16, TH = HG / 16, TE = 2 * D / 16;  // 16-feature tiles
    static constexpr int NW = NW_;
    // GG: G2 (forward) / G2^T (backward) read from global memory instead of LDS
    static constexpr bool GG = D >= 128;
    static constexpr int SCR = slab_scratch<(D > HG ? D : HG)>();  // floats of slab scratch per wave
    // forward LDS: G1 [HG][2D] and (!GG) G2 [D][HG] as stored, rows padded by 4 floats, then c1, c2
    static constexpr int F_LD1 = 2 * D + 4, F_LD2 = HG + 4;
    static constexpr int F_LDS = HG * F_LD1 + (GG ? 0 : D * F_LD2) + HG + D;
    // backward LDS: G2^T [HG][D], then G1^T [2D][HG] (GG: one at a time, G1^T over G2^T)
    static constexpr int B_LD1 = D + 4, B_LD2 = HG + 4;
    static constexpr int B_G1T = GG ? 0 : HG * B_LD1;  // offset of G1^T
    static constexpr int B_LDS = B_G1T + 2 * D * B_LD2;
    static_assert(D % 16 == 0 && HG % 16 == 0, "16-feature tiles");
    static_assert((F_LDS + NW * SCR) * 4 <= 163840 && (B_LDS + NW * SCR) * 4 <= 163840,
                  "the gate matrices must fit one CU's LDS");
    // split-bf16: G1 (forward, [HG] rows x 2D k) / G1^T (backward, [2D] rows x HG k) as three bf16
    // planes, 2 B x 3 per weight; G2 / G2^T stay fp32 (the 16x16x4 f32 GEMM)
    static constexpr int X1_BYTES = 3 * 2 * (2 * D) * HG;
    static constexpr int XF_BYTES = X1_BYTES + 4 * (D * F_LD2 + HG + D);
    static constexpr int XB_BYTES = X1_BYTES + 4 * (HG * B_LD1);
    static constexpr bool X_OK = !GG && (2 * D) % 32 == 0 && HG % 32 == 0 && XF_BYTES <= 163840 && XB_BYTES <= 163840;
};

// this block's tower and its index among the tower's blocks
__device__ __forceinline__ int gate_tower(const KArg(GateArgs) * ka, int& bidx) {
    bidx = blockIdx.x;
    if (ka->count > 1 && bidx >= ka->tw[0].blocks) {
        bidx -= ka->tw[0].blocks;
        return 1;
    }
    return 0;
}

template <int D, int HG, bool X, int NW>
__global__ __launch_bounds__(64 * NW) void gate_fwd_kernel(GateArgs) {
    using C = GateCfg<D, HG, NW>;
    constexpr int NT = 64 * NW;
    constexpr int NX = (2 * D) / 32;  // split: k-steps of the first GEMM
    // !X: each wave's slab-store scratch after the matrices (store_slab)
    __shared__ __attribute__((aligned(16))) float lds[X ? C::XF_BYTES / 4 : C::F_LDS + NW * C::SCR];
    const KArg(GateArgs)* ka = (const KArg(GateArgs)*)(__builtin_amdgcn_kernarg_segment_ptr());
    int bidx;
    const KArg(GateTower)& T = ka->tw[gate_tower(ka, bidx)];
    float* g1s = lds;  // fp32 G1, or (X) its three bf16 planes
    unsigned char* img = reinterpret_cast<unsigned char*>(lds);
    float* g2s = X ? reinterpret_cast<float*>(img + C::X1_BYTES) : g1s + HG * C::F_LD1;  // (!GG)
    float* c1s = C::GG ? g2s : g2s + D * C::F_LD2;
    float* c2s = c1s + HG;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int li = lane & 15, q = lane >> 4;
    float* scr = lds + C::F_LDS + wave * C::SCR;  // (!X)
    const int64_t R = T.R;
    const int64_t nslab = (R + 15) / 16;
    const int64_t stride = (int64_t)T.blocks * NW;
    int64_t s = (int64_t)bidx * NW + wave;
    // the first slab's rows are in flight while the block stages the gate matrices
    f4v ef[C::TE];
    int64_t arow = 0;  // the slab row's mimic-table row
    if (s < nslab) {
        const int64_t r0 = s * 16 + li < R ? s * 16 + li : R - 1;
        load_row(ef, T.ef, 2 * D, r0, q);
        if (T.table) arow = T.idx[r0];
    }
    constexpr int N1 = HG * (2 * D / 4), N2 = D * (HG / 4);
#pragma unroll
    for (int e0 = 0; e0 < N1; e0 += NT) {
        const int e = e0 + (int)threadIdx.x;
        if (e < N1) {
            const int i = e / (2 * D / 4), c = 4 * (e % (2 * D / 4));
            const f4v w = ldg4(T.G1 + (int64_t)i * 2 * D + c);
            if constexpr (X) {
                int t, q4, j;
                xw_slot(c, t, q4, j);
                xw_store4<HG, C::X1_BYTES / 3>(img, t, q4, i, j, w);
            } else {
                *reinterpret_cast<f4v*>(g1s + i * C::F_LD1 + c) = w;
            }
        }
    }
    if constexpr (!C::GG) {
#pragma unroll
        for (int e0 = 0; e0 < N2; e0 += NT) {
            const int e = e0 + (int)threadIdx.x;
            if (e < N2) {
                const int i = e / (HG / 4), c = 4 * (e % (HG / 4));
                *reinterpret_cast<f4v*>(g2s + i * C::F_LD2 + c) = ldg4(T.G2 + (int64_t)i * HG + c);
            }
        }
    }
    for (int e = threadIdx.x; e < HG + D; e += NT) c1s[e] = e < HG ? T.c1[e] : T.c2[e - HG];
    __syncthreads();
    for (; s < nslab; s += stride) {
        const int64_t row = s * 16 + li;
        const bool ok = row < R;
        f4v a[C::TD];  // mimic rows for the epilogue, requested before the MFMA chain
        if (T.table) load_row(a, T.table, D, arow, q);
        const int xu_li = T.xu && ok ? (int)T.xu[row] : 0;  // compact exchange unit (int: < 2^31 units)
        f4v z[C::TH];
        zero(z);
        if constexpr (X) tile_gemm_x<C::TH, NX, HG>(img, 0, ef, z, li, q);  // z^T = G1 . ef^T
        else tile_gemm<C::TH, C::TE, C::F_LD1>(g1s, 0, ef, z, li, q);
        // the next slab's rows, in flight during the rest of this one (GG: a wave rarely has a
        // second slab, and the registers hold the global G2 fragments instead)
        f4v nx[C::GG ? 1 : C::TE];
        int64_t arow_n = 0;
        const int64_t sn = s + stride;
        if (!C::GG && sn < nslab) {
            const int64_t rn = sn * 16 + li < R ? sn * 16 + li : R - 1;
            load_row(nx, T.ef, 2 * D, rn, q);
            if (T.table) arow_n = T.idx[rn];
        }
#pragma unroll
        for (int ob = 0; ob < C::TH; ++ob) {
            const f4v c1 = lds4(c1s + 16 * ob + 4 * q);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float v = z[ob][r] + c1[r];
                z[ob][r] = v > 0.f ? v : 0.f;
            }
            if ((X || (kDevKnobs && ka->direct)) && ok && !(kDevKnobs && ka->ablate)) stg4(T.z + row * HG + 16 * ob + 4 * q, z[ob]);
        }
        if (!(X || (kDevKnobs && ka->direct)) && !(kDevKnobs && ka->ablate)) store_slab<C::TH>(scr, z, T.z, HG, s * 16, R, lane);
        f4v x[C::TD];
        zero(x);
        if constexpr (C::GG) tile_gemm_g<C::TD, C::TH, HG>(T.G2, 0, z, x, li, q);  // (pre-sigmoid)^T = G2 . z^T
        else tile_gemm<C::TD, C::TH, C::F_LD2>(g2s, 0, z, x, li, q);
        if (!(X || (kDevKnobs && ka->direct)) && !(kDevKnobs && ka->ablate)) {
            // g, then t = g e + (1 - g) f in place, a, then aug = t + a in place: one live array
#pragma unroll
            for (int ob = 0; ob < C::TD; ++ob) {
                const f4v c2 = lds4(c2s + 16 * ob + 4 * q);
#pragma unroll
                for (int r = 0; r < 4; ++r) x[ob][r] = sigmoid_(x[ob][r] + c2[r]);
            }
            store_slab<C::TD>(scr, x, T.g, D, s * 16, R, lane);
#pragma unroll
            for (int ob = 0; ob < C::TD; ++ob) {
                const f4v e = ef[ob], f = ef[C::TD + ob];  // this lane's columns of e and f
#pragma unroll
                for (int r = 0; r < 4; ++r) x[ob][r] = x[ob][r] * e[r] + (1.0f - x[ob][r]) * f[r];
            }
            if (T.xu) {  // compact exchange rows: (t | a) of a positive, t + a of a negative
                store_slab_xu<C::TD>(scr, a, T.a, xu_li, true, s * 16, R, lane);
                const bool neg = xu_li < 0;
#pragma unroll
                for (int ob = 0; ob < C::TD; ++ob)
#pragma unroll
                    for (int r = 0; r < 4; ++r) x[ob][r] = neg ? x[ob][r] + a[ob][r] : x[ob][r];
                store_slab_xu<C::TD>(scr, x, T.t, xu_li, false, s * 16, R, lane);
            } else {
                store_slab<C::TD>(scr, x, T.t, T.ld_t, s * 16, R, lane);
                if (T.table) {
                    store_slab<C::TD>(scr, a, T.a, T.ld_t, s * 16, R, lane);
#pragma unroll
                    for (int ob = 0; ob < C::TD; ++ob)
#pragma unroll
                        for (int r = 0; r < 4; ++r) x[ob][r] = x[ob][r] + a[ob][r];
                }
                if (T.aug) store_slab<C::TD>(scr, x, T.aug, D, s * 16, R, lane);
            }
        }
        if ((X || (kDevKnobs && ka->direct)) && ok && !(kDevKnobs && ka->ablate)) {
            // compact exchange rows (T.xu): a positive's t and a at its unit, a negative's t + a
            const int64_t xu = xu_li;
            float* tdst = T.xu ? T.t + (xu >= 0 ? xu : ~xu) * D : T.t + row * T.ld_t;
            float* adst = T.xu ? (xu >= 0 ? T.a + xu * D : nullptr) : (T.table ? T.a + row * T.ld_t : nullptr);
#pragma unroll
            for (int ob = 0; ob < C::TD; ++ob) {
                const int col = 16 * ob + 4 * q;
                const f4v c2 = lds4(c2s + col);
                const f4v e = ef[ob], f = ef[C::TD + ob];  // this lane's columns of e and f
                f4v g, tt;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    g[r] = sigmoid_(x[ob][r] + c2[r]);
                    tt[r] = g[r] * e[r] + (1.0f - g[r]) * f[r];
                }
                stg4(T.g + row * D + col, g);
                f4v aug = tt;
                if (T.table) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) aug[r] = tt[r] + a[ob][r];
                }
                stg4(tdst + col, T.xu && xu < 0 ? aug : tt);
                if (adst) stg4(adst + col, a[ob]);
                if (T.aug) stg4(T.aug + row * D + col, aug);
            }
        }
        if constexpr (C::GG) {
            if (sn < nslab) {
                const int64_t rn = sn * 16 + li < R ? sn * 16 + li : R - 1;
                load_row(ef, T.ef, 2 * D, rn, q);
                if (T.table) arow = T.idx[rn];
            }
        } else if (sn < nslab) {
#pragma unroll
            for (int t = 0; t < C::TE; ++t) ef[t] = nx[t];
            arow = arow_n;
        }
    }
}

template <int D, int HG, bool X, int NW>
__global__ __launch_bounds__(64 * NW) void gate_bwd_kernel(GateArgs) {
    using C = GateCfg<D, HG, NW>;
    constexpr int NT = 64 * NW;
    constexpr int NX = HG / 32;  // split: k-steps of the dEF GEMM
    __shared__ __attribute__((aligned(16))) float lds[X ? C::XB_BYTES / 4 : C::B_LDS + NW * C::SCR];
    const KArg(GateArgs)* ka = (const KArg(GateArgs)*)(__builtin_amdgcn_kernarg_segment_ptr());
    int bidx;
    const KArg(GateTower)& T = ka->tw[gate_tower(ka, bidx)];
    unsigned char* img = reinterpret_cast<unsigned char*>(lds);  // (X) G1^T as three bf16 planes
    float* g2t = X ? reinterpret_cast<float*>(img + C::X1_BYTES) : lds;  // G2^T [HG][D]
    float* g1t = lds + C::B_G1T;  // G1^T [2D][HG] (GG: over G2^T, staged after it)
    float* scr = lds + C::B_LDS + (threadIdx.x >> 6) * C::SCR;          // (!X)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int li = lane & 15, q = lane >> 4;
    const int64_t R = T.R;
    const int64_t nslab = (R + 15) / 16;
    const int64_t stride = (int64_t)T.blocks * NW;
    // transposed staging: float4 reads along a row, four scalar LDS writes down a column
    constexpr int N2 = D * (HG / 4), N1 = HG * (2 * D / 4);
    auto stage_g2t = [&]() {
#pragma unroll
        for (int e0 = 0; e0 < N2; e0 += NT) {
            const int e = e0 + (int)threadIdx.x;
            if (e < N2) {
                const int d = e / (HG / 4), j = 4 * (e % (HG / 4));  // G2 [D][HG]
                const f4v v = ldg4(T.G2 + (int64_t)d * HG + j);
#pragma unroll
                for (int i = 0; i < 4; ++i) g2t[(j + i) * C::B_LD1 + d] = v[i];
            }
        }
    };
    if constexpr (C::GG) {
        // the two matrices do not fit together: per round of NW slabs the block stages G2^T, every
        // wave forms its slab's dq and dz, then G1^T over it and every wave forms dEF (every wave
        // passes every barrier; one round at C4, where R / 16 <= blocks x NW)
        for (int64_t s0 = (int64_t)bidx * NW; s0 < nslab; s0 += stride) {
            const int64_t s = s0 + wave;
            const bool has = s < nslab;
            const int64_t row = s * 16 + li;
            const bool ok = has && row < R;
            const int64_t rr = ok ? row : R - 1;
            f4v d[C::TD], g[C::TD], dz[C::TH];
            {
                f4v ef[C::TE];
                load_dt_row(d, T.dT, T.ld_dT, T.xu, D, rr, q);
                load_row(ef, T.ef, 2 * D, rr, q);
                load_row(g, T.g, D, rr, q);
                stage_g2t();
                __syncthreads();
                if (has) {
                    f4v dq[C::TD];  // dq = (dT e - dT f) (1 - g) g
#pragma unroll
                    for (int t = 0; t < C::TD; ++t)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const float dg = d[t][r] * ef[t][r] - d[t][r] * ef[C::TD + t][r];
                            dq[t][r] = dg * (1.0f - g[t][r]) * g[t][r];
                        }
                    if (!(kDevKnobs && ka->ablate)) store_slab<C::TD>(scr, dq, T.dq, D, s * 16, R, lane);
                    f4v zr[C::TH];
                    load_row(zr, T.z, HG, rr, q);
                    zero(dz);
                    tile_gemm<C::TH, C::TD, C::B_LD1>(g2t, 0, dq, dz, li, q);  // dz^T = G2^T . dq^T
#pragma unroll
                    for (int ob = 0; ob < C::TH; ++ob)
#pragma unroll
                        for (int r = 0; r < 4; ++r) dz[ob][r] = zr[ob][r] > 0.f ? dz[ob][r] : 0.f;
                    if (!(kDevKnobs && ka->ablate)) store_slab<C::TH>(scr, dz, T.dz, HG, s * 16, R, lane);
                }
            }
            __syncthreads();
#pragma unroll
            for (int e0 = 0; e0 < N1; e0 += NT) {
                const int e = e0 + (int)threadIdx.x;
                if (e < N1) {
                    const int j = e / (2 * D / 4), c = 4 * (e % (2 * D / 4));  // G1 [HG][2D]
                    const f4v v = ldg4(T.G1 + (int64_t)j * 2 * D + c);
#pragma unroll
                    for (int i = 0; i < 4; ++i) g1t[(c + i) * C::B_LD2 + j] = v[i];
                }
            }
            __syncthreads();
            if (has) {
#pragma unroll 1
                for (int half = 0; half < 2; ++half) {  // dEF^T = G1^T . dz^T + [dT g | dT (1 - g)]
                    f4v de[C::TD];
                    zero(de);
                    tile_gemm<C::TD, C::TH, C::B_LD2>(g1t, half * C::TD, dz, de, li, q);
#pragma unroll
                    for (int ob = 0; ob < C::TD; ++ob)
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            de[ob][r] += half == 0 ? d[ob][r] * g[ob][r] : d[ob][r] * (1.0f - g[ob][r]);
                    if (!(kDevKnobs && ka->ablate)) store_slab<C::TD>(scr, de, T.dEF + half * D, 2 * D, s * 16, R, lane);
                }
            }
            __syncthreads();  // the next round's G2^T overwrites G1^T
        }
        return;
    }
    stage_g2t();
#pragma unroll
    for (int e0 = 0; e0 < N1; e0 += NT) {
        const int e = e0 + (int)threadIdx.x;
        if (e < N1) {
            const int j = e / (2 * D / 4), c = 4 * (e % (2 * D / 4));  // G1 [HG][2D]
            const f4v v = ldg4(T.G1 + (int64_t)j * 2 * D + c);
            if constexpr (X) {  // hidden unit j is k slot (t, q4, js) of rows c .. c + 3
                int t, q4, js;
                xw_slot(j, t, q4, js);
                constexpr int PL = C::X1_BYTES / 3;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float w = v[i];
                    const __bf16 h = (__bf16)w;
                    const float r = w - (float)h;
                    const __bf16 m = (__bf16)r;
                    const __bf16 l = (__bf16)(r - (float)m);
                    const int off = xw_off<2 * D>(t, q4, c + i, js);
                    *reinterpret_cast<__bf16*>(img + off) = h;
                    *reinterpret_cast<__bf16*>(img + PL + off) = m;
                    *reinterpret_cast<__bf16*>(img + 2 * PL + off) = l;
                }
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) g1t[(c + i) * C::B_LD2 + j] = v[i];
            }
        }
    }
    __syncthreads();
    for (int64_t s = (int64_t)bidx * NW + wave; s < nslab; s += stride) {
        const int64_t row = s * 16 + li;
        const bool ok = row < R;
        const int64_t rr = ok ? row : R - 1;
        // every operand of the slab requested at once
        f4v d[C::TD], ef[C::TE], g[C::TD], zr[C::TH];
        load_dt_row(d, T.dT, T.ld_dT, T.xu, D, rr, q);
        load_row(ef, T.ef, 2 * D, rr, q);
        load_row(g, T.g, D, rr, q);
        load_row(zr, T.z, HG, rr, q);
        f4v dz[C::TH];
        {
            f4v dq[C::TD];  // dq = (dT e - dT f) (1 - g) g
#pragma unroll
            for (int t = 0; t < C::TD; ++t) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float dg = d[t][r] * ef[t][r] - d[t][r] * ef[C::TD + t][r];
                    dq[t][r] = dg * (1.0f - g[t][r]) * g[t][r];
                }
                if ((X || (kDevKnobs && ka->direct)) && ok && !(kDevKnobs && ka->ablate)) stg4(T.dq + row * D + 16 * t + 4 * q, dq[t]);
            }
            if (!(X || (kDevKnobs && ka->direct)) && !(kDevKnobs && ka->ablate))
                store_slab<C::TD>(scr, dq, T.dq, D, s * 16, R, lane);
            zero(dz);
            tile_gemm<C::TH, C::TD, C::B_LD1>(g2t, 0, dq, dz, li, q);  // dz^T = G2^T . dq^T
        }
#pragma unroll
        for (int ob = 0; ob < C::TH; ++ob) {
#pragma unroll
            for (int r = 0; r < 4; ++r) dz[ob][r] = zr[ob][r] > 0.f ? dz[ob][r] : 0.f;
            if ((X || (kDevKnobs && ka->direct)) && ok && !(kDevKnobs && ka->ablate)) stg4(T.dz + row * HG + 16 * ob + 4 * q, dz[ob]);
        }
        if (!(X || (kDevKnobs && ka->direct)) && !(kDevKnobs && ka->ablate))
            store_slab<C::TH>(scr, dz, T.dz, HG, s * 16, R, lane);
        // dEF^T = G1^T . dz^T + [dT g | dT (1 - g)], in two halves (e part, f part)
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            f4v de[C::TD];
            zero(de);
            if constexpr (X) tile_gemm_x<C::TD, NX, 2 * D>(img, half * C::TD, dz, de, li, q);
            else tile_gemm<C::TD, C::TH, C::B_LD2>(g1t, half * C::TD, dz, de, li, q);
#pragma unroll
            for (int ob = 0; ob < C::TD; ++ob)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    de[ob][r] += half == 0 ? d[ob][r] * g[ob][r] : d[ob][r] * (1.0f - g[ob][r]);
            if ((X || (kDevKnobs && ka->direct)) && ok && !(kDevKnobs && ka->ablate)) {
#pragma unroll
                for (int ob = 0; ob < C::TD; ++ob) stg4(T.dEF + row * 2 * D + half * D + 16 * ob + 4 * q, de[ob]);
            }
            if (!(X || (kDevKnobs && ka->direct)) && !(kDevKnobs && ka->ablate))
                store_slab<C::TD>(scr, de, T.dEF + half * D, 2 * D, s * 16, R, lane);
        }
    }
}

// persistent grid: about one block per CU, split between the towers by row count
int gate_blocks(GateArgs& a, int waves) {
    static int cus = 0;
    if (cus == 0) {
        int dev = 0, n = 0;
        cus = 256;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
            cus = n;
    }
    int64_t total = 0;
    for (int i = 0; i < a.count; ++i) total += a.tw[i].R;
    int sum = 0;
    for (int i = 0; i < a.count; ++i) {
        const int64_t need = ceil_div(ceil_div(a.tw[i].R, 16), waves);  // blocks with a slab per wave
        int64_t share = (cus * a.tw[i].R + total - 1) / total;
        if (share > need) share = need;
        a.tw[i].blocks = (int)(share < 1 ? 1 : share);
        sum += a.tw[i].blocks;
    }
    return sum;
}

template <int D, int HG, int NW>
int launch_gate_nw(GateArgs& a, bool backward, hipStream_t s) {
    const int blocks = gate_blocks(a, NW);
    // TTAMM_GATE_SPLIT=1: the 2D-wide GEMM on split-bf16 MFMA.  Measured at C2 (D = 96): forward
    // 64 -> 62 us, backward 67 -> 79 us, step 0.726 -> 0.758 ms (profiles/r03_c2_gate_split_s17.txt):
    // the kernels are not MFMA-bound (SQ: ~31 % MFMA busy, profiles/r03_c2_pmc_sq_s13.json) and the
    // split variant runs at the 256-VGPR limit, so both GEMMs stay on v_mfma_f32_16x16x4_f32
    static const bool split = dev_env("TTAMM_GATE_SPLIT") != nullptr;
    constexpr bool XOK = GateCfg<D, HG, NW>::X_OK;
    if (XOK && split) {
        if (backward) hipLaunchKernelGGL((gate_bwd_kernel<D, HG, XOK, NW>), dim3(blocks), dim3(64 * NW), 0, s, a);
        else hipLaunchKernelGGL((gate_fwd_kernel<D, HG, XOK, NW>), dim3(blocks), dim3(64 * NW), 0, s, a);
        TTAMM_LAUNCH_CHECK();
        return TTAMM_OK;
    }
    if (backward) hipLaunchKernelGGL((gate_bwd_kernel<D, HG, false, NW>), dim3(blocks), dim3(64 * NW), 0, s, a);
    else hipLaunchKernelGGL((gate_fwd_kernel<D, HG, false, NW>), dim3(blocks), dim3(64 * NW), 0, s, a);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

template <int D, int HG>
int launch_gate_t(GateArgs& a, bool backward, hipStream_t s) {
    // TTAMM_GATE_4W=1 (D = 96): 4-wave blocks, one wave per SIMD with the whole register file (the
    // split variant then has room: TTAMM_GATE_SPLIT=1)
    if constexpr (D == 96) {
        static const bool w4 = [] {
            const char* e = dev_env("TTAMM_GATE_4W");
            return e && e[0] == '1';
        }();
        if (w4) return launch_gate_nw<D, HG, 4>(a, backward, s);
    }
    return launch_gate_nw<D, HG, GateWaves<D>::NW>(a, backward, s);
}

}  // namespace

bool gate_fused_supported(int D, int HG) { return D == HG && (D == 32 || D == 64 || D == 96 || D == 128); }

int launch_gate(GateArgs& a, bool backward, hipStream_t s) {
    if (a.planes) {
        int rc;
        if (!a.images_ready && (rc = launch_gate16_prep(a, s))) return rc;
        return launch_gate16(a, backward, s);
    }
    static const bool ablate = dev_env("TTAMM_GATE_ABLATE") != nullptr;
    static const bool direct = dev_env("TTAMM_GATE_DIRECT_STORES") != nullptr;
    a.ablate = ablate ? 1 : 0;
    a.direct = direct ? 1 : 0;
    TTAMM_REQUIRE(a.count >= 1 && a.count <= 2 && gate_fused_supported(a.D, a.HG), "fused gate: unsupported shape");
    for (int i = 0; i < a.count; ++i) TTAMM_REQUIRE(a.tw[i].R > 0, "fused gate: empty tower");
    switch (a.D) {
        case 32: return launch_gate_t<32, 32>(a, backward, s);
        case 64: return launch_gate_t<64, 64>(a, backward, s);
        case 96: return launch_gate_t<96, 96>(a, backward, s);
        default: return launch_gate_t<128, 128>(a, backward, s);
    }
}

}  // namespace ttamm
