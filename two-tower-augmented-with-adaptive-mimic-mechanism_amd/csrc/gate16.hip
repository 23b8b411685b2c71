// Fused FeatureFusionGate for bf16 towers (BASELINE C5: D = Hg = 256; encoders.py:149-168,
// applied at :246-253, with the adaptive-mimic augment of adaptive_mimic.py:88-95).  The bf16
// semantics of the generic path are kept: every GEMM operand rounded to bf16 (RNE), fp32
// accumulation, the elementwise work in fp32.  Per row, with ef = [e | f]:
//
//   forward   z = relu(ef G1^T + c1) ; g = sigmoid(z G2^T + c2) ; t = g e + (1 - g) f ; aug = t + A[idx]
//   backward  dq = (dT e - dT f)(1 - g) g ; dz = (dq G2) * (z > 0) ; dEF = dz G1 + [dT g | dT (1 - g)]
//
// The generic path runs these as 4 GEMM launches + 2 elementwise kernels that round-trip the
// pre-activation, z, dq and dz through HBM (C5: ~470 us per step, each launch latency-bound).
// Here a wave owns 32 rows and chains both GEMMs of a direction in registers with
// v_mfma_f32_32x32x16_bf16 in the "rows on the lanes" orientation: OUT^T = W . X^T, the weight as
// the A operand, the 32 rows as the B operand's columns.  The first product's accumulators hold
// OUT^T with the row on the lane and 16 output features in registers — exactly the B operand of
// the next product (which sums over those features) after a pairwise bf16 conversion, no LDS and
// no lane movement: registers 8s .. 8s+7 are k-step s, element j of lane half h being feature
// 16s + 8(j>>2) + 4h + (j&3) of the 32-feature tile.  The weight of that next product is therefore
// stored with its k (input-feature) index permuted inside every 16-group (perm16), so lane half
// h's eight elements are contiguous.  The 4 waves of a block share the weights: 64-k chunks of the
// bf16 weight images (formed once per step by gate16_prep_kernel) are double-buffered through LDS
// (rows padded to 144 B: conflict-free ds_read_b128), one barrier per chunk.
#include "kernels.h"

namespace ttamm {

namespace {

typedef float f4v __attribute__((ext_vector_type(4)));
typedef float g16_f32x8 __attribute__((ext_vector_type(8)));
typedef float g16_f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 g16_bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int g16_u32x4 __attribute__((ext_vector_type(4)));

constexpr int kG16Waves = 4;
constexpr int kG16Threads = 64 * kG16Waves;
constexpr int kG16Rows = 32 * kG16Waves;  // rows per block
#ifndef TTAMM_G16_NT
#define TTAMM_G16_NT 0
#endif
constexpr bool kG16NtStores = TTAMM_G16_NT != 0;  // developer A/B (-DTTAMM_G16_NT=1)

// position of input feature u inside its 16-group in a "next product" weight image
__device__ __forceinline__ int perm16(int u) {
    return (u & ~15) | (((u >> 2) & 1) << 3) | (((u >> 3) & 1) << 2) | (u & 3);
}

// NP bf16 planes of an operand: NP = 1 rounds it (bf16 towers), NP = 3 splits an fp32 value exactly
// into hi + mid + lo (fp32 towers, gemm.hip's split-bf16: six MFMAs per product, fp32-accurate)
template <int NP>
struct Frag {
    g16_bf16x8 p[NP];
};
template <int NP>
__device__ __forceinline__ Frag<NP> split(const g16_f32x8& x) {
    Frag<NP> f;
    f.p[0] = __builtin_convertvector(x, g16_bf16x8);
    if constexpr (NP == 3) {
        const g16_f32x8 r = x - __builtin_convertvector(f.p[0], g16_f32x8);
        f.p[1] = __builtin_convertvector(r, g16_bf16x8);
        f.p[2] = __builtin_convertvector(r - __builtin_convertvector(f.p[1], g16_f32x8), g16_bf16x8);
    }
    return f;
}
template <int NP>
__device__ __forceinline__ Frag<NP> split(f4v a, f4v b) {
    const g16_f32x8 x = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    return split<NP>(x);
}
// accumulator registers 8s .. 8s + 7 as the B fragment of k-step s
template <int NP>
__device__ __forceinline__ Frag<NP> acc_frag(const g16_f32x16& a, int s) {
    const g16_f32x8 x = {a[8 * s], a[8 * s + 1], a[8 * s + 2], a[8 * s + 3],
                         a[8 * s + 4], a[8 * s + 5], a[8 * s + 6], a[8 * s + 7]};
    return split<NP>(x);
}
// acc += A . B: one MFMA (NP = 1) or the six of a split product, small terms first
template <int NP>
__device__ __forceinline__ void mma(g16_f32x16& acc, const Frag<NP>& a, const Frag<NP>& b) {
    if constexpr (NP == 3) {
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[1], b.p[1], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[2], b.p[0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[0], b.p[2], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[1], b.p[0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[0], b.p[1], acc, 0, 0, 0);
    }
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[0], b.p[0], acc, 0, 0, 0);
}

__device__ __forceinline__ f4v ld4(const float* p) { return *reinterpret_cast<const f4v*>(p); }
// plain stores: a lane writes 16 B and a store instruction 32 B per row in the accumulator layout,
// so the L2 must merge the pieces of a line before it is written back (a non-temporal store of a
// partial line is not merged: 457 -> 273 us at C5)
__device__ __forceinline__ void st4(float* p, f4v v) {
    if (kG16NtStores) store_nt(p, make_float4(v[0], v[1], v[2], v[3]));
    else *reinterpret_cast<f4v*>(p) = v;
}
__device__ __forceinline__ f4v quad(const g16_f32x16& a, int g) { return f4v{a[4 * g], a[4 * g + 1], a[4 * g + 2], a[4 * g + 3]}; }
__device__ __forceinline__ g16_f32x16 zero16() {
    g16_f32x16 z;
#pragma unroll
    for (int i = 0; i < 16; ++i) z[i] = 0.f;
    return z;
}

__device__ __forceinline__ int g16_tower(const KArg(GateArgs) * ka, int& bidx) {
    bidx = blockIdx.x;
    if (ka->count > 1 && bidx >= ka->tw[0].blocks) {
        bidx -= ka->tw[0].blocks;
        return 1;
    }
    return 0;
}

// Weight images (bf16, per tower, NP planes of gate16_image_elems / NP each): W1 [Hg][2D] as G1;
// W1T [2D][Hg] = G1^T with the Hg index perm16'd; W2 [D][Hg] = G2 with the Hg index perm16'd;
// W2T [Hg][D] = G2^T.  Chunks of KC k-columns of D rows (every image's A-operand rows number D
// here, Hg = D) are staged per plane into LDS rows of KC + 8 bf16 (conflict-free ds_read_b128).
template <int D, int NP>
struct G16 {
    static constexpr int HG = D, K1 = 2 * D, NT = D / 32;
    static constexpr int KC = D % 64 == 0 ? 64 : 32;  // k per staged chunk
    static constexpr int TPC = KC / 32;               // 32-wide tiles of the next product per chunk
    static constexpr int LROW = KC + 8;               // bf16 per LDS row
    static constexpr int PLANE = D * LROW;            // bf16 per plane of one buffer
    static constexpr int BUF = NP * PLANE;            // bf16 per buffer
    static constexpr int64_t IMG = 2 * (int64_t)HG * K1 + 2 * (int64_t)D * HG;  // bf16 per plane image
    static constexpr int64_t W1 = 0, W1T = (int64_t)HG * K1, W2 = 2 * (int64_t)HG * K1, W2T = W2 + (int64_t)D * HG;
    static constexpr int PIECES = NP * D * KC / 8;    // 16-B pieces per chunk
    static constexpr int PPT = (PIECES + kG16Threads - 1) / kG16Threads;
    static_assert(D % 32 == 0 && K1 % (2 * KC) == 0 && HG % KC == 0, "gate16 shape");
};

template <int D, int NP>
struct Chunk {
    g16_u32x4 v[G16<D, NP>::PPT];
};
// columns [k0, k0 + KC) of D rows of every plane of an image (leading dimension ld)
template <int D, int NP>
__device__ __forceinline__ void chunk_load(Chunk<D, NP>& c, const uint16_t* img, int ld, int k0) {
    using C = G16<D, NP>;
#pragma unroll
    for (int i = 0; i < C::PPT; ++i) {
        const int q = (int)threadIdx.x + kG16Threads * i;
        if (C::PIECES % kG16Threads == 0 || q < C::PIECES) {
            const int plane = q / (D * C::KC / 8), rem = q - plane * (D * C::KC / 8);
            const int row = rem / (C::KC / 8), col = (rem - row * (C::KC / 8)) * 8;
            c.v[i] = *reinterpret_cast<const g16_u32x4*>(img + plane * C::IMG + (int64_t)row * ld + k0 + col);
        }
    }
}
template <int D, int NP>
__device__ __forceinline__ void chunk_store(const Chunk<D, NP>& c, uint16_t* buf) {
    using C = G16<D, NP>;
#pragma unroll
    for (int i = 0; i < C::PPT; ++i) {
        const int q = (int)threadIdx.x + kG16Threads * i;
        if (C::PIECES % kG16Threads == 0 || q < C::PIECES) {
            const int plane = q / (D * C::KC / 8), rem = q - plane * (D * C::KC / 8);
            const int row = rem / (C::KC / 8), col = (rem - row * (C::KC / 8)) * 8;
            *reinterpret_cast<g16_u32x4*>(buf + plane * C::PLANE + row * C::LROW + col) = c.v[i];
        }
    }
}
template <int D, int NP>
__device__ __forceinline__ Frag<NP> lds_frag(const uint16_t* buf, int row, int col) {
    using C = G16<D, NP>;
    Frag<NP> f;
#pragma unroll
    for (int p = 0; p < NP; ++p)
        f.p[p] = *reinterpret_cast<const g16_bf16x8*>(buf + p * C::PLANE + row * C::LROW + col);
    return f;
}

__global__ __launch_bounds__(256) void gate16_prep_kernel(GateArgs) {
    const KArg(GateArgs)* ka = (const KArg(GateArgs)*)(__builtin_amdgcn_kernarg_segment_ptr());
    const KArg(GateTower)& T = ka->tw[blockIdx.y];
    const int D = ka->D, HG = ka->HG, K1 = 2 * D, NP = ka->planes;
    const int64_t n1 = (int64_t)HG * K1, n2 = (int64_t)D * HG, img = 2 * n1 + 2 * n2;
    uint16_t* w = T.w16;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n1 + n2; e += (int64_t)gridDim.x * blockDim.x) {
        const float x = e < n1 ? T.G1[e] : T.G2[e - n1];
        int64_t o0, o1;  // the element's positions in the two images it belongs to
        if (e < n1) {
            const int u = (int)(e / K1), k = (int)(e - (int64_t)u * K1);
            o0 = e;
            o1 = n1 + (int64_t)k * HG + perm16(u);
        } else {
            const int64_t e2 = e - n1;
            const int f = (int)(e2 / HG), u = (int)(e2 - (int64_t)f * HG);
            o0 = 2 * n1 + (int64_t)f * HG + perm16(u);
            o1 = 2 * n1 + n2 + (int64_t)u * D + f;
        }
        float r = x;
        for (int p = 0; p < NP; ++p) {  // hi, mid, lo (RNE, exact differences)
            const __bf16 v = (__bf16)r;
            r = r - (float)v;
            w[p * img + o0] = __builtin_bit_cast(uint16_t, v);
            w[p * img + o1] = __builtin_bit_cast(uint16_t, v);
        }
    }
}

// LDS plan (floats): the two weight-chunk buffers, then (backward) each wave's dq rows (bf16 for
// NP = 1, fp32 for NP = 3: split when read); the row epilogues reuse the whole array for each
// wave's 32 output rows in fp32 (stride D + 4)
template <int D, int NP>
struct G16Lds {
    static constexpr int CHUNKS = G16<D, NP>::BUF;           // 2 buffers of BUF bf16 = BUF floats
    static constexpr int QROW = NP == 1 ? D + 8 : D + 4;     // dq row: bf16 (528 B at D = 256) or fp32
    static constexpr int QS = CHUNKS;                        // offset (floats) of the dq rows
    static constexpr int QWAVE = NP == 1 ? 32 * QROW / 2 : 32 * QROW;  // floats per wave
    static constexpr int XROW = D + 4;                       // floats per epilogue row
    static constexpr int XWAVE = 32 * XROW;
    static constexpr int FWD = CHUNKS > kG16Waves * XWAVE ? CHUNKS : kG16Waves * XWAVE;
    static constexpr int BWD_A = QS + kG16Waves * QWAVE;
    static constexpr int BWD = BWD_A > kG16Waves * XWAVE ? BWD_A : kG16Waves * XWAVE;
    static_assert((FWD + 2 * D) * 4 <= 163840 && BWD * 4 <= 163840, "gate16 LDS");
};

// the wave's accumulator tiles (OUT^T: row r on the lane, output 32 n + 8 g + 4 h + i in register
// 4 g + i of tile n) as row-major fp32 rows in its LDS rows
template <int D>
__device__ __forceinline__ void acc_to_rows(float* xs, const g16_f32x16 (&acc)[D / 32], int r, int h) {
#pragma unroll
    for (int n = 0; n < D / 32; ++n)
#pragma unroll
        for (int g = 0; g < 4; ++g)
            *reinterpret_cast<f4v*>(xs + r * (D + 4) + 32 * n + 8 * g + 4 * h) = quad(acc[n], g);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes are done
    __builtin_amdgcn_wave_barrier();
}

// the row epilogues: float4 q = it * 64 + lane of the wave's 32 rows x D / 4 float4s
template <int D>
struct RowIt {
    static constexpr int F4 = D / 4, ITS = 32 * F4 / 64;
    static_assert((32 * F4) % 64 == 0, "row iterations");
};

template <int D, int NP>
__global__ __launch_bounds__(kG16Threads) void gate16_fwd_kernel(GateArgs) {
    using C = G16<D, NP>;
    using L = G16Lds<D, NP>;
    using RI = RowIt<D>;
    constexpr int HG = C::HG, K1 = C::K1, NT = C::NT, KC = C::KC, NC1 = K1 / KC, NC2 = HG / KC;
    __shared__ __attribute__((aligned(16))) float ldsf[L::FWD];
    __shared__ float cb[HG + D];
    uint16_t* lds = reinterpret_cast<uint16_t*>(ldsf);
    const KArg(GateArgs)* ka = (const KArg(GateArgs)*)(__builtin_amdgcn_kernarg_segment_ptr());
    int bidx;
    const KArg(GateTower)& T = ka->tw[g16_tower(ka, bidx)];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
    const int64_t R = T.R;
    const int64_t wrow0 = (int64_t)bidx * kG16Rows + wave * 32;
    const int64_t row = wrow0 + r;
    const bool ok = row < R;
    const int64_t rr = ok ? row : R - 1;
    const uint16_t* W1 = T.w16 + C::W1;
    const uint16_t* W2 = T.w16 + C::W2;
    const float* efr = T.ef + rr * K1;
    for (int e = threadIdx.x; e < HG + D; e += kG16Threads) cb[e] = e < HG ? T.c1[e] : T.c2[e - HG];

    // z^T = G1 . ef^T: NT tiles of 32 hidden units, k over the 2D inputs in KC-wide chunks
    Chunk<D, NP> ch;
    chunk_load(ch, W1, K1, 0);
    chunk_store(ch, lds);
    // ef values of chunks c and c + 1 in flight (bx[c & 1]): k-step s of a chunk covers its
    // k = 16 s + 8 h .. + 7
    constexpr int KS = KC / 16;
    f4v bx[2][2 * KS];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            bx[c][2 * s] = ld4(efr + c * KC + 16 * s + 8 * h);
            bx[c][2 * s + 1] = ld4(efr + c * KC + 16 * s + 8 * h + 4);
        }
    __syncthreads();
    g16_f32x16 acc[NT];
#pragma unroll
    for (int m = 0; m < NT; ++m) acc[m] = zero16();
    int buf = 0;
    // chunk c with its ef values in bx[b] (b = c & 1, a constant at each call: two calls per loop trip)
    auto gemm1_step = [&](int c, int b) {
        if (c + 1 < NC1) chunk_load(ch, W1, K1, (c + 1) * KC);
        else chunk_load(ch, W2, HG, 0);
        Frag<NP> bf[KS];
#pragma unroll
        for (int s = 0; s < KS; ++s) bf[s] = split<NP>(bx[b][2 * s], bx[b][2 * s + 1]);
        if (c + 2 < NC1) {
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                bx[b][2 * s] = ld4(efr + (c + 2) * KC + 16 * s + 8 * h);
                bx[b][2 * s + 1] = ld4(efr + (c + 2) * KC + 16 * s + 8 * h + 4);
            }
        }
        const uint16_t* Lb = lds + buf * C::BUF;
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int m = 0; m < NT; ++m) mma<NP>(acc[m], lds_frag<D, NP>(Lb, 32 * m + r, 16 * s + 8 * h), bf[s]);
        chunk_store(ch, lds + (buf ^ 1) * C::BUF);
        __syncthreads();
        buf ^= 1;
    };
    static_assert(NC1 % 2 == 0, "chunk pairs");
    for (int c = 0; c < NC1; c += 2) {
        gemm1_step(c, 0);
        gemm1_step(c + 1, 1);
    }
    // z = relu(. + c1): stored (the backward's ReLU mask), and kept as the next product's B operand
    Frag<NP> zb[NT][2];
#pragma unroll
    for (int m = 0; m < NT; ++m) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int u0 = 32 * m + 8 * g + 4 * h;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float v = acc[m][4 * g + i] + cb[u0 + i];
                acc[m][4 * g + i] = v > 0.f ? v : 0.f;
            }
            if (ok) st4(T.z + row * HG + u0, quad(acc[m], g));
        }
        zb[m][0] = acc_frag<NP>(acc[m], 0);
        zb[m][1] = acc_frag<NP>(acc[m], 1);
    }
    // (pre-sigmoid)^T = G2 . z^T: NT tiles of 32 outputs, k over the Hg units (chunk c = z tiles
    // TPC c .. TPC c + TPC - 1, two k-steps each)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[n] = zero16();
#pragma unroll
    for (int c = 0; c < NC2; ++c) {
        if (c + 1 < NC2) chunk_load(ch, W2, HG, (c + 1) * KC);
        const uint16_t* Lb = lds + buf * C::BUF;
#pragma unroll
        for (int mm = 0; mm < C::TPC; ++mm)
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int n = 0; n < NT; ++n)
                    mma<NP>(acc[n], lds_frag<D, NP>(Lb, 32 * n + r, 32 * mm + 16 * s + 8 * h), zb[C::TPC * c + mm][s]);
        if (c + 1 < NC2) chunk_store(ch, lds + (buf ^ 1) * C::BUF);
        __syncthreads();
        buf ^= 1;
    }
    // the wave's pre-sigmoid rows through LDS (every wave is past the last chunk: the loop's
    // barrier), then whole row segments: g, t = g e + (1 - g) f, a = A[idx], aug = t + a (fp32, as
    // gate_mix_kernel / gate.hip); a batch's loads are issued before its stores (the stores may
    // alias the loads as far as the compiler knows, so it would not hoist them itself)
    float* xs = ldsf + wave * L::XWAVE;
    acc_to_rows<D>(xs, acc, r, h);
    constexpr int RB = RI::ITS % 8 == 0 ? 8 : (RI::ITS % 6 == 0 ? 6 : 4);
    static_assert(RI::ITS % RB == 0, "row batches");
    for (int it0 = 0; it0 < RI::ITS; it0 += RB) {
        f4v e4[RB], fv[RB], a4[RB];
#pragma unroll
        for (int j = 0; j < RB; ++j) {
            const int q = (it0 + j) * 64 + lane, rl = q / RI::F4, f0 = 4 * (q - rl * RI::F4);
            const int64_t g0 = wrow0 + rl;
            const int64_t gr = g0 < R ? g0 : R - 1;
            e4[j] = ld4(T.ef + gr * K1 + f0);
            fv[j] = ld4(T.ef + gr * K1 + D + f0);
            if (T.table) a4[j] = ld4(T.table + T.idx[gr] * (int64_t)D + f0);
        }
#pragma unroll
        for (int j = 0; j < RB; ++j) {
            const int q = (it0 + j) * 64 + lane, rl = q / RI::F4, f0 = 4 * (q - rl * RI::F4);
            const int64_t grow_ = wrow0 + rl;
            if (grow_ >= R) continue;
            const f4v x = *reinterpret_cast<const f4v*>(xs + rl * L::XROW + f0);
            f4v gg, tt;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float v = x[i] + cb[HG + f0 + i];
                gg[i] = NP == 1 ? __builtin_amdgcn_rcpf(1.0f + __expf(-v)) : 1.0f / (1.0f + __expf(-v));
                tt[i] = gg[i] * e4[j][i] + (1.0f - gg[i]) * fv[j][i];
            }
            st4(T.g + grow_ * D + f0, gg);
            f4v aug = tt;
            if (T.table) {
#pragma unroll
                for (int i = 0; i < 4; ++i) aug[i] = tt[i] + a4[j][i];
            }
            if (T.xu) {  // compact exchange rows: (t | a) of a positive, t + a of a negative
                const int64_t u = T.xu[grow_];
                if (u >= 0) {
                    st4(T.t + u * D + f0, tt);
                    st4(T.a + u * D + f0, a4[j]);
                } else {
                    st4(T.t + (~u) * D + f0, aug);
                }
            } else {
                st4(T.t + grow_ * T.ld_t + f0, tt);
                if (T.table) st4(T.a + grow_ * T.ld_t + f0, a4[j]);
            }
            if (T.aug) st4(T.aug + grow_ * D + f0, aug);
        }
    }
}

// row gr's dT: at gr * ld_dT, or its compact exchange unit (GateTower::xu)
__device__ __forceinline__ const float* dt_row(const KArg(GateTower) & T, int64_t gr, int D) {
    if (!T.xu) return T.dT + gr * T.ld_dT;
    const int64_t u = T.xu[gr];
    return T.dT + (u >= 0 ? u : ~u) * D;
}

template <int D, int NP>
__global__ __launch_bounds__(kG16Threads) void gate16_bwd_kernel(GateArgs) {
    using C = G16<D, NP>;
    using L = G16Lds<D, NP>;
    using RI = RowIt<D>;
    constexpr int HG = C::HG, K1 = C::K1, NT = C::NT, KC = C::KC, NC3 = D / KC, NC4 = HG / KC;
    __shared__ __attribute__((aligned(16))) float ldsf[L::BWD];
    uint16_t* lds = reinterpret_cast<uint16_t*>(ldsf);
    const KArg(GateArgs)* ka = (const KArg(GateArgs)*)(__builtin_amdgcn_kernarg_segment_ptr());
    int bidx;
    const KArg(GateTower)& T = ka->tw[g16_tower(ka, bidx)];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
    const int64_t R = T.R;
    const int64_t wrow0 = (int64_t)bidx * kG16Rows + wave * 32;
    const int64_t row = wrow0 + r;
    const bool ok = row < R;
    const int64_t rr = ok ? row : R - 1;
    const uint16_t* W1T = T.w16 + C::W1T;
    const uint16_t* W2T = T.w16 + C::W2T;

    Chunk<D, NP> ch;
    chunk_load(ch, W2T, D, 0);
    chunk_store(ch, lds);
    // dq = (dT e - dT f)(1 - g) g over whole row segments (stored; into the wave's dq rows, the B
    // operand of the dz product: k = feature)
    uint16_t* qs16 = lds + 2 * L::QS + wave * 32 * L::QROW;  // NP = 1
    float* qs32 = ldsf + L::QS + wave * 32 * L::QROW;        // NP = 3
    constexpr int RQ = 4;
    for (int it0 = 0; it0 < RI::ITS; it0 += RQ) {
        f4v d4[RQ], e4[RQ], fv[RQ], g4[RQ];
#pragma unroll
        for (int j = 0; j < RQ; ++j) {
            const int q = (it0 + j) * 64 + lane, rl = q / RI::F4, f0 = 4 * (q - rl * RI::F4);
            const int64_t g0 = wrow0 + rl;
            const int64_t gr = g0 < R ? g0 : R - 1;
            d4[j] = ld4(dt_row(T, gr, D) + f0);
            e4[j] = ld4(T.ef + gr * K1 + f0);
            fv[j] = ld4(T.ef + gr * K1 + D + f0);
            g4[j] = ld4(T.g + gr * D + f0);
        }
#pragma unroll
        for (int j = 0; j < RQ; ++j) {
            const int q = (it0 + j) * 64 + lane, rl = q / RI::F4, f0 = 4 * (q - rl * RI::F4);
            const int64_t grow_ = wrow0 + rl;
            f4v dq;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float dg = d4[j][i] * e4[j][i] - d4[j][i] * fv[j][i];
                dq[i] = dg * (1.0f - g4[j][i]) * g4[j][i];
            }
            if (grow_ < R) st4(T.dq + grow_ * D + f0, dq);
            if constexpr (NP == 1) {
                typedef __bf16 g16_bf16x4 __attribute__((ext_vector_type(4)));
                *reinterpret_cast<g16_bf16x4*>(qs16 + rl * L::QROW + f0) = __builtin_convertvector(dq, g16_bf16x4);
            } else {
                *reinterpret_cast<f4v*>(qs32 + rl * L::QROW + f0) = dq;
            }
        }
    }
    // z (the ReLU mask) of the first half of the unit tiles in flight during the dz product
    constexpr int NZ = NT / 2;
    f4v zp[NZ > 0 ? NZ : 1][4];
#pragma unroll
    for (int m = 0; m < NZ; ++m)
#pragma unroll
        for (int g = 0; g < 4; ++g) zp[m][g] = ld4(T.z + rr * HG + 32 * m + 8 * g + 4 * h);
    __syncthreads();
    // dz^T = G2^T . dq^T: NT tiles of 32 units, k over the D outputs in KC-wide chunks
    g16_f32x16 acc[NT];
#pragma unroll
    for (int m = 0; m < NT; ++m) acc[m] = zero16();
    int buf = 0;
    for (int c = 0; c < NC3; ++c) {
        if (c + 1 < NC3) chunk_load(ch, W2T, D, (c + 1) * KC);
        else chunk_load(ch, W1T, HG, 0);  // the dEF product's first chunk (pass 0)
        const uint16_t* Lb = lds + buf * C::BUF;
#pragma unroll
        for (int s = 0; s < KC / 16; ++s) {
            Frag<NP> qb;
            if constexpr (NP == 1) {
                qb.p[0] = *reinterpret_cast<const g16_bf16x8*>(qs16 + r * L::QROW + c * KC + 16 * s + 8 * h);
            } else {
                const float* qp = qs32 + r * L::QROW + c * KC + 16 * s + 8 * h;
                qb = split<NP>(ld4(qp), ld4(qp + 4));
            }
#pragma unroll
            for (int m = 0; m < NT; ++m) mma<NP>(acc[m], lds_frag<D, NP>(Lb, 32 * m + r, 16 * s + 8 * h), qb);
        }
        chunk_store(ch, lds + (buf ^ 1) * C::BUF);
        __syncthreads();
        buf ^= 1;
    }
    // dz = dz * (z > 0): stored (the gate weight gradient's input) and kept as B fragments
    Frag<NP> zb[NT][2];
    f4v zq[NT - NZ][4];
#pragma unroll
    for (int m = NZ; m < NT; ++m)
#pragma unroll
        for (int g = 0; g < 4; ++g) zq[m - NZ][g] = ld4(T.z + rr * HG + 32 * m + 8 * g + 4 * h);
#pragma unroll
    for (int m = 0; m < NT; ++m) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int u0 = 32 * m + 8 * g + 4 * h;
            const f4v z4 = m < NZ ? zp[m < NZ ? m : 0][g] : zq[m - NZ][g];
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[m][4 * g + i] = z4[i] > 0.f ? acc[m][4 * g + i] : 0.f;
            if (ok) st4(T.dz + row * HG + u0, quad(acc[m], g));
        }
        zb[m][0] = acc_frag<NP>(acc[m], 0);
        zb[m][1] = acc_frag<NP>(acc[m], 1);
    }
    // dEF^T = G1^T . dz^T + [dT g | dT (1 - g)], in two passes of D outputs (e part, f part); each
    // pass's rows leave through LDS as whole row segments (the pass-1 chunks are staged after pass
    // 0's rows)
    float* xs = ldsf + wave * L::XWAVE;
    constexpr int RB = RI::ITS % 8 == 0 ? 8 : (RI::ITS % 6 == 0 ? 6 : 4);
    static_assert(RI::ITS % RB == 0 && RI::ITS % RQ == 0, "row batches");
    for (int pass = 0; pass < 2; ++pass) {
        const uint16_t* Wp = W1T + (int64_t)pass * D * HG;
        if (pass == 1) {  // pass 0's first chunk came with the dz product's last one
            chunk_load(ch, Wp, HG, 0);
            chunk_store(ch, lds + buf * C::BUF);
            __syncthreads();
        }
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[n] = zero16();
#pragma unroll
        for (int c = 0; c < NC4; ++c) {
            if (c + 1 < NC4) chunk_load(ch, Wp, HG, (c + 1) * KC);
            const uint16_t* Lb = lds + buf * C::BUF;
#pragma unroll
            for (int mm = 0; mm < C::TPC; ++mm)
#pragma unroll
                for (int s = 0; s < 2; ++s)
#pragma unroll
                    for (int n = 0; n < NT; ++n)
                        mma<NP>(acc[n], lds_frag<D, NP>(Lb, 32 * n + r, 32 * mm + 16 * s + 8 * h),
                                zb[C::TPC * c + mm][s]);
            if (c + 1 < NC4) chunk_store(ch, lds + (buf ^ 1) * C::BUF);
            __syncthreads();
            buf ^= 1;
        }
        acc_to_rows<D>(xs, acc, r, h);
        for (int it0 = 0; it0 < RI::ITS; it0 += RB) {
            f4v d4[RB], g4[RB];
#pragma unroll
            for (int j = 0; j < RB; ++j) {
                const int q = (it0 + j) * 64 + lane, rl = q / RI::F4, f0 = 4 * (q - rl * RI::F4);
                const int64_t g0 = wrow0 + rl;
                const int64_t gr = g0 < R ? g0 : R - 1;
                d4[j] = ld4(dt_row(T, gr, D) + f0);
                g4[j] = ld4(T.g + gr * D + f0);
            }
#pragma unroll
            for (int j = 0; j < RB; ++j) {
                const int q = (it0 + j) * 64 + lane, rl = q / RI::F4, f0 = 4 * (q - rl * RI::F4);
                const int64_t grow_ = wrow0 + rl;
                if (grow_ >= R) continue;
                const f4v x = *reinterpret_cast<const f4v*>(xs + rl * L::XROW + f0);
                f4v de;
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    de[i] = x[i] + (pass == 0 ? d4[j][i] * g4[j][i] : d4[j][i] * (1.0f - g4[j][i]));
                st4(T.dEF + grow_ * K1 + pass * D + f0, de);
            }
        }
        __syncthreads();  // every wave is done with its rows before the next pass stages over them
    }
}

template <int D, int NP>
int launch_g16(GateArgs& a, bool backward, hipStream_t s) {
    int total = 0;
    for (int i = 0; i < a.count; ++i) {
        a.tw[i].blocks = (int)ceil_div(a.tw[i].R, kG16Rows);
        total += a.tw[i].blocks;
    }
    if (backward) hipLaunchKernelGGL((gate16_bwd_kernel<D, NP>), dim3(total), dim3(kG16Threads), 0, s, a);
    else hipLaunchKernelGGL((gate16_fwd_kernel<D, NP>), dim3(total), dim3(kG16Threads), 0, s, a);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

}  // namespace

bool gate16_supported(int D, int HG, int planes) {
    return D == HG && (planes == 1 ? (D == 128 || D == 256) : planes == 3 && D == 96);
}

int64_t gate16_image_elems(int D, int HG, int planes) {
    return (int64_t)planes * (2 * (int64_t)HG * 2 * D + 2 * (int64_t)D * HG);
}

int launch_gate16_prep(GateArgs& a, hipStream_t s) {
    TTAMM_REQUIRE(a.count >= 1 && a.count <= 2 && gate16_supported(a.D, a.HG, a.planes), "gate16: unsupported shape");
    for (int i = 0; i < a.count; ++i) TTAMM_REQUIRE(a.tw[i].w16 != nullptr, "gate16: no weight image");
    const int64_t n = (int64_t)a.HG * 2 * a.D + (int64_t)a.D * a.HG;  // source elements
    const int blocks = (int)(ceil_div(n, 256) < 512 ? ceil_div(n, 256) : 512);
    hipLaunchKernelGGL(gate16_prep_kernel, dim3(blocks, a.count), dim3(256), 0, s, a);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

int launch_gate16(GateArgs& a, bool backward, hipStream_t s) {
    TTAMM_REQUIRE(a.count >= 1 && a.count <= 2 && gate16_supported(a.D, a.HG, a.planes), "gate16: unsupported shape");
    for (int i = 0; i < a.count; ++i)
        TTAMM_REQUIRE(a.tw[i].R > 0 && a.tw[i].w16 != nullptr, "gate16: empty tower or no weight image");
    if (a.planes == 3) return launch_g16<96, 3>(a, backward, s);
    return a.D == 128 ? launch_g16<128, 1>(a, backward, s) : launch_g16<256, 1>(a, backward, s);
}

}  // namespace ttamm
