// Row-wise kernels of the training step: embedding row gather, non-gated fusion,
// the gate's sigmoid backward, and the fused score + BCE + mimic-MSE forward/backward.
#include "kernels.h"

namespace ttamm {

namespace {

// Row id r of a table with `rows` rows, or -1 when it is outside the table (the gathers then
// write a zero row instead of reading outside it; the step reports such ids via its status).
__device__ __forceinline__ int64_t checked_row(int64_t r, int64_t rows) { return (r >= 0 && r < rows) ? r : -1; }

// out[r, :] = table[idx[r], :]   (nn.Embedding forward, encoders.py:222-223).
// One float4 per thread, flat over n * dim/4; bit-exact copy.
__global__ void gather_rows_vec4(const float* __restrict__ table, int64_t rows, int d4,
                                 const int64_t* __restrict__ idx, int64_t n, float* __restrict__ out, int64_t out_ld) {
    const int64_t total = n * d4;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / d4;
        const int c = (int)(i - r * d4);
        const int64_t src = checked_row(idx[r], rows);
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (src >= 0) v = reinterpret_cast<const float4*>(table + src * (int64_t)d4 * 4)[c];
        reinterpret_cast<float4*>(out + r * out_ld)[c] = v;
    }
}

// Whole-row gather, rows of D4 float4: a wave takes RPW rows per iteration, their
// RPW x D4 float4 flattened over I = RPW*D4/64 wave instructions (no idle lanes for any D4,
// e.g. 96-wide rows: 8 rows in 3 instructions; 128-wide: 8 rows in 4).  Each lane issues its
// I row indices, then its I row loads, so a CU keeps I x 16 B x 2048 lanes of HBM reads in
// flight — what random rows of a table far larger than the caches need to approach the HBM
// rate (MI355X_MICROARCH.md, "Indexed rows").  Rows are written with streaming stores (the
// consumer is a later kernel).  Bit-exact copy.
constexpr int cgcd(int a, int b) { return b == 0 ? a : cgcd(b, a % b); }
template <int D4>
struct WideGather {
    static constexpr int RPW0 = 64 / cgcd(64, D4);  // fewest rows filling whole instructions
    static constexpr int I0 = RPW0 * D4 / 64;
    static constexpr int MUL = I0 >= 4 ? 1 : (4 + I0 - 1) / I0;
    static constexpr int RPW = RPW0 * MUL, I = I0 * MUL;
};

template <int D4>
__global__ __launch_bounds__(256) void gather_rows_wide(const float4* __restrict__ table, int64_t rows,
                                                         const int64_t* __restrict__ idx, int64_t n,
                                                         float4* __restrict__ out, int64_t out_ld4) {
    constexpr int RPW = WideGather<D4>::RPW, I = WideGather<D4>::I;
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t r0 = ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * RPW; r0 < n;
         r0 += nwaves * RPW) {
        int64_t src[I];
#pragma unroll
        for (int u = 0; u < I; ++u) {
            const int64_t r = r0 + (u * 64 + lane) / D4;
            src[u] = r < n ? checked_row(idx[r], rows) : -1;
        }
        float4 v[I];
#pragma unroll
        for (int u = 0; u < I; ++u) {
            v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (src[u] >= 0) v[u] = table[src[u] * D4 + (u * 64 + lane) % D4];
        }
#pragma unroll
        for (int u = 0; u < I; ++u) {
            const int e = u * 64 + lane;
            const int64_t r = r0 + e / D4;
            if (r < n) store_nt(out + r * out_ld4 + e % D4, v[u]);
        }
    }
}

// gather_rows_wide over up to two (table, idx, out) segments of one row width, blockIdx.y =
// segment: the user and item towers' ID rows in one launch
template <int D4>
__global__ __launch_bounds__(256) void gather_rows_wide_seg(GatherSegs) {
    const KArg(GatherSegs)* ka = (const KArg(GatherSegs)*)(__builtin_amdgcn_kernarg_segment_ptr());
    const KArg(GatherSeg)& S = ka->seg[blockIdx.y];
    constexpr int RPW = WideGather<D4>::RPW, I = WideGather<D4>::I;
    const float4* table = reinterpret_cast<const float4*>(S.table);
    float4* out = reinterpret_cast<float4*>(S.out);
    const int64_t n = S.n, rows = S.rows, out_ld4 = S.out_ld / 4;
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t r0 = ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * RPW; r0 < n;
         r0 += nwaves * RPW) {
        int64_t src[I];
#pragma unroll
        for (int u = 0; u < I; ++u) {
            const int64_t r = r0 + (u * 64 + lane) / D4;
            src[u] = r < n ? checked_row(S.idx[r], rows) : -1;
        }
        float4 v[I];
#pragma unroll
        for (int u = 0; u < I; ++u) {
            v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (src[u] >= 0) v[u] = table[src[u] * D4 + (u * 64 + lane) % D4];
        }
#pragma unroll
        for (int u = 0; u < I; ++u) {
            const int e = u * 64 + lane;
            const int64_t r = r0 + e / D4;
            if (r < n) store_nt(out + r * out_ld4 + e % D4, v[u]);
        }
    }
}

__global__ void gather_rows_scalar(const float* __restrict__ table, int64_t rows, int dim,
                                   const int64_t* __restrict__ idx, int64_t n, float* __restrict__ out, int64_t out_ld) {
    const int64_t total = n * dim;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / dim;
        const int c = (int)(i - r * dim);
        const int64_t src = checked_row(idx[r], rows);
        out[r * out_ld + c] = src >= 0 ? table[src * (int64_t)dim + c] : 0.f;
    }
}

// Index staging of a training step (kernels.h StageArgs); blockIdx.y = segment, y == count: the
// owner's compact exchange units (StageArgs::unit_out)
__global__ void stage_rows_kernel(StageArgs) {
    const KArg(StageArgs)* ka = (const KArg(StageArgs)*)(__builtin_amdgcn_kernarg_segment_ptr());
    if ((int)blockIdx.y == ka->count) {
        extern __shared__ int64_t tab[];  // per group: first row, positive rows before, positive rows
        const int G = ka->unit_groups;
        if (threadIdx.x == 0) {
            int64_t r = 0, p = 0;
            for (int g = 0; g < G; ++g) {
                const int64_t c = ka->unit_counts[g * ka->unit_ld], q = ka->unit_counts[g * ka->unit_ld + 2];
                tab[3 * g] = r;
                tab[3 * g + 1] = p;
                tab[3 * g + 2] = q;
                r += c;
                p += q;
            }
        }
        __syncthreads();
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ka->unit_n;
             i += (int64_t)gridDim.x * blockDim.x) {
            int lo = 0, hi = G - 1;  // the last group starting at or before row i (empty groups share starts)
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (tab[3 * mid] <= i) lo = mid;
                else hi = mid - 1;
            }
            const int64_t r = i - tab[3 * lo], p = tab[3 * lo + 2];
            const int64_t unit = i + tab[3 * lo + 1] + (r < p ? r : p);
            ka->unit_out[i] = r < p ? unit : ~unit;
        }
        return;
    }
    const KArg(StageSeg)& S = ka->seg[blockIdx.y];
    const int64_t n = S.n, rows = S.rows;
    bool bad = false;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t v = S.in[i * (S.ld ? S.ld : 1)];
        const bool ok = v >= 0 && v < rows;
        bad |= !ok;
        if (S.out) S.out[i] = ok ? v : 0;
    }
    if (ka->status && __ballot(bad) != 0ull && (threadIdx.x & 63) == 0)
        atomicOr(ka->status, TTAMM_STATUS_INDEX_OUT_OF_RANGE);
}

// t = e (+ f) ; a = table[idx] ; aug = t + a      (encoders.py:225-240, adaptive_mimic.py:88-95)
__global__ void combine_kernel(const float* __restrict__ e, int64_t ld_e, const float* __restrict__ f,
                               int64_t ld_f, const float* __restrict__ table, int64_t table_rows,
                               const int64_t* __restrict__ idx,
                               int64_t n, int dim, float* __restrict__ t, float* __restrict__ a, int64_t ld_ta,
                               float* __restrict__ aug) {
    const int64_t total = n * dim;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / dim;
        const int c = (int)(i - r * dim);
        float tv = e[r * ld_e + c];
        if (f) tv = tv + f[r * ld_f + c];
        if (t) t[r * ld_ta + c] = tv;
        float av = tv;
        if (table) {
            const int64_t src = checked_row(idx[r], table_rows);
            const float am = src >= 0 ? table[src * (int64_t)dim + c] : 0.f;
            if (a) a[r * ld_ta + c] = am;
            av = tv + am;
        }
        if (aug) aug[i] = av;
    }
}

// dst[r, c] = c < cols ? src[r, c] : 0   (16-byte aligned copy of an nn.Linear weight whose
// in_features is not a multiple of 4, e.g. the 605-wide first feature layer)
__global__ void pad_rows_kernel(const float* __restrict__ src, int64_t rows, int cols, int64_t ld_src,
                                float* __restrict__ dst, int ld_dst) {
    const int64_t total = rows * ld_dst;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / ld_dst;
        const int c = (int)(i - r * ld_dst);
        dst[i] = c < cols ? src[r * ld_src + c] : 0.f;
    }
}

// pad_rows_kernel over up to two segments (blockIdx.y): both towers' first-layer weights
__global__ void pad_rows_seg_kernel(PadSegs) {
    const KArg(PadSegs)* ka = (const KArg(PadSegs)*)(__builtin_amdgcn_kernarg_segment_ptr());
    const KArg(PadSeg)& S = ka->seg[blockIdx.y];
    const int64_t total = S.rows * S.ld_dst;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / S.ld_dst;
        const int c = (int)(i - r * S.ld_dst);
        S.dst[i] = c < S.cols ? S.src[r * S.ld_src + c] : 0.f;
    }
}

// dq = (dT*e - dT*f) * (1 - g) * g
// autograd of gate*e + (1-gate)*f then SigmoidBackward (grad*(1-y)*y), encoders.py:164-168.
__global__ void gate_dq_kernel(const float* __restrict__ dT, int64_t ld_dT, const float* __restrict__ ef,
                               const float* __restrict__ g, int64_t n, int dim, float* __restrict__ dq) {
    const int64_t total = n * dim;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / dim;
        const int c = (int)(i - r * dim);
        const float d = dT[r * ld_dT + c];
        const float ev = ef[r * 2 * dim + c], fv = ef[r * 2 * dim + dim + c];
        const float gv = g[i];
        const float dg = d * ev - d * fv;
        dq[i] = dg * (1.0f - gv) * gv;
    }
}

// BCEWithLogits term, ATen form: (1-y)*x + m + log(exp(-m) + exp(-x-m)), m = max(-x, 0)
__device__ __forceinline__ float bce_logit(float x, float y) {
    const float m = fmaxf(-x, 0.f);
    return (1.0f - y) * x + m + logf(expf(-m) + expf(-x - m));
}

// One wave per interaction b (training.py:770-803, Appendix A of SURVEY.md):
//   s+ = <u_b, p_b>, s-_j = <u_b, n_bj>; ds = (sigmoid(s) - y) / (Bg(1+N))
//   dT_user = ds+ p + sum_j ds-_j n_j ; dT_pos = ds+ u ; dT_neg_j = ds-_j u
//   mimic: dA_user = dT_user + lu * 2/(Bg D) * (a_u - t_p) ; dA_pos = dT_pos + li * 2/(Bg D) * (a_p - t_u)
//          (dA_all: negative rows' dA = dT_neg, the requester ships (dT | dA) for every row)
// Bg is the global batch: in a sharded step each rank's terms are its share of the global mean.
constexpr int kScoreWaves = 4;
constexpr int kMaxDChunks = 8;  // D <= 512
constexpr int kMaxNeg = 64;

// r: the row in the item buffers (item_slot already applied)
// (neg: a negative request's row, which holds t + a already under A.neg_aug)
__device__ __forceinline__ float item_aug_at(const ScoreArgs& A, int64_t r, int d, bool neg = false) {
    if (A.item_aug) return A.item_aug[r * A.ld_item + d];
    const float t = A.t_item[r * A.ld_item + d];
    return A.a_item && !(neg && A.neg_aug) ? t + A.a_item[r * A.ld_item + d] : t;
}

// NCH = ceil(D / 64) chunks per lane.  Every row the wave reads is requested before the first
// reduction (the positive, the user's mimic terms, then the negatives in groups of kScoreNG):
// one memory latency per group instead of one per row, and the NG dot-product reductions
// interleave.  Sums keep the chunk order of the scalar loop (lane partials over c, then the
// butterfly), so the results are those of the one-row-at-a-time form.
constexpr int kScoreNG = 8;
template <int NCH>
__global__ __launch_bounds__(64 * kScoreWaves) void score_loss_kernel(ScoreArgs A) {
    __shared__ float red[kScoreWaves][3];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t b = (int64_t)blockIdx.x * kScoreWaves + w;
    const int D = A.D, N = A.N;
    const int64_t B = A.B;
    const int64_t ldi = A.ld_dti;
    const float inv_numel = A.inv_numel;
    const bool ib = A.ib_du != nullptr;
    float bce = 0.f, mse_u = 0.f, mse_i = 0.f;
    if (b < B) {
        const int64_t pb = A.item_slot ? A.item_slot[b] : b;  // the positive's item row
        bool ok[NCH];
        float u[NCH], p[NCH], du[NCH], dpos[NCH];
        float au[NCH], tp[NCH], ap[NCH], tu[NCH], ibp[NCH], ibu[NCH];
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const int d = c * 64 + lane;
            ok[c] = d < D;
            u[c] = p[c] = au[c] = tp[c] = ap[c] = tu[c] = ibp[c] = ibu[c] = 0.f;
            if (ok[c]) {
                u[c] = A.user_aug[b * D + d];
                p[c] = item_aug_at(A, pb, d);
                if (A.mimic) {
                    au[c] = A.a_user[b * D + d];
                    tp[c] = A.t_item[pb * A.ld_item + d];
                    ap[c] = A.a_item[pb * A.ld_item + d];
                    tu[c] = A.t_user[b * D + d];
                }
                if (ib) {
                    ibp[c] = A.ib_dp[b * A.ib_ld + d];
                    ibu[c] = A.ib_du[b * D + d];
                }
            }
        }
        float dot = 0.f;
#pragma unroll
        for (int c = 0; c < NCH; ++c)
            if (ok[c]) dot += u[c] * p[c];
        const float sp = wave_sum(dot);
        float dsp = 0.f;
        if (!ib) {
            dsp = (1.0f / (1.0f + expf(-sp)) - 1.0f) * inv_numel;
            bce += bce_logit(sp, 1.0f);
        }
        // positive item row: dT_pos = ds+ * u ; user: ds+ * p   (in-batch: the S = U P^T terms)
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const int d = c * 64 + lane;
            dpos[c] = 0.f;
            du[c] = 0.f;
            if (ok[c]) {
                dpos[c] = ib ? ibp[c] : dsp * u[c];
                A.dT_item[pb * ldi + d] = dpos[c];
                du[c] = ib ? ibu[c] : dsp * p[c];
            }
        }
        for (int j0 = 0; j0 < N; j0 += kScoreNG) {
            const int ng = N - j0 < kScoreNG ? N - j0 : kScoreNG;
            int64_t nr[kScoreNG];
            float nv[kScoreNG][NCH];
#pragma unroll
            for (int jj = 0; jj < kScoreNG; ++jj) {
                nr[jj] = 0;
                if (jj < ng) {
                    const int64_t q = B + b * N + j0 + jj;
                    nr[jj] = A.item_slot ? A.item_slot[q] : q;
                }
#pragma unroll
                for (int c = 0; c < NCH; ++c) nv[jj][c] = (jj < ng && ok[c]) ? item_aug_at(A, nr[jj], c * 64 + lane, true) : 0.f;
            }
            float sn[kScoreNG];
#pragma unroll
            for (int jj = 0; jj < kScoreNG; ++jj) {
                float dn = 0.f;
#pragma unroll
                for (int c = 0; c < NCH; ++c)
                    if (ok[c]) dn += u[c] * nv[jj][c];
                sn[jj] = jj < ng ? wave_sum(dn) : 0.f;
            }
#pragma unroll
            for (int jj = 0; jj < kScoreNG; ++jj) {
                if (jj >= ng) continue;
                const float dsn = (1.0f / (1.0f + expf(-sn[jj])) - 0.0f) * inv_numel;
                bce += bce_logit(sn[jj], 0.0f);
#pragma unroll
                for (int c = 0; c < NCH; ++c) {
                    const int d = c * 64 + lane;
                    if (ok[c]) {
                        const float g = dsn * u[c];
                        A.dT_item[nr[jj] * ldi + d] = g;
                        if (A.mimic && A.dA_all) A.dA_item[nr[jj] * ldi + d] = g;
                        du[c] += dsn * nv[jj][c];
                    }
                }
            }
        }
        const float norm = 2.0f / (float)(A.Bg * D);
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const int d = c * 64 + lane;
            if (ok[c]) {
                A.dT_user[b * D + d] = du[c];
                if (A.mimic) {
                    const float xu = au[c] - tp[c], xi = ap[c] - tu[c];
                    mse_u += xu * xu;
                    mse_i += xi * xi;
                    A.dA_user[b * D + d] = du[c] + norm * xu * A.lambda_u;
                    A.dA_item[pb * ldi + d] = dpos[c] + norm * xi * A.lambda_i;
                }
            }
        }
        mse_u = wave_sum(mse_u);
        mse_i = wave_sum(mse_i);
    }
    if (lane == 0) {
        red[w][0] = bce;
        red[w][1] = mse_u;
        red[w][2] = mse_i;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        float s = 0.f;
        for (int i = 0; i < kScoreWaves; ++i) s += red[i][threadIdx.x];
        A.partials[blockIdx.x * 3 + threadIdx.x] = s;
    }
}

// The same scores, gradients and loss terms with G lanes per interaction (64 / G interactions
// per wave) and NV float4 columns per lane (D = 4 G NV: lane s of a group holds columns
// 4 (s + G i) .. + 3, so a group's loads of one row are G consecutive 16-B pieces): 16-B loads
// and stores instead of 4-B ones, all lanes busy at D = 96, and each dot product reduced over
// log2 G lanes instead of 64.  Used when D % (4 G) == 0; the lane partials are summed over
// i and then across the group (a different order from score_loss_kernel's chunk sums).
__device__ __forceinline__ float group_sum(float v, int G) {
    for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float dot4(float4 a, float4 b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }
__device__ __forceinline__ float4 scale4(float s, float4 a) { return make_float4(s * a.x, s * a.y, s * a.z, s * a.w); }
__device__ __forceinline__ float4 fma4(float s, float4 a, float4 c) {
    return make_float4(c.x + s * a.x, c.y + s * a.y, c.z + s * a.z, c.w + s * a.w);
}
__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ float4 addf4(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }

template <int G, int NV>
__global__ __launch_bounds__(64 * kScoreWaves) void score_loss_v_kernel(ScoreArgs A) {
    constexpr int NG = NV <= 3 ? 8 : 4;  // negatives in flight per group
    __shared__ float red[kScoreWaves][3];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, s = lane % G;
    const int64_t b = ((int64_t)blockIdx.x * kScoreWaves + w) * (64 / G) + lane / G;
    constexpr int D = 4 * G * NV;
    const int N = A.N;
    const int64_t B = A.B, ldi = A.ld_dti, ldt = A.ld_item;
    const float inv_numel = A.inv_numel;
    const bool ib = A.ib_du != nullptr;
    float bce = 0.f, mse_u = 0.f, mse_i = 0.f;
    if (b < B) {
        const int64_t pb = A.item_slot ? A.item_slot[b] : b;
        auto item_row = [&](int64_t r, int c, bool neg) {
            if (A.item_aug) return ld4(A.item_aug + r * ldt + c);
            const float4 t = ld4(A.t_item + r * ldt + c);
            return A.a_item && !(neg && A.neg_aug) ? addf4(t, ld4(A.a_item + r * ldt + c)) : t;
        };
        const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
        float4 u[NV], p[NV], au[NV], tp[NV], ap[NV], tu[NV], ibp[NV], ibu[NV];
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const int c = 4 * (s + G * i);
            u[i] = ld4(A.user_aug + b * D + c);
            p[i] = item_row(pb, c, false);
            au[i] = tp[i] = ap[i] = tu[i] = ibp[i] = ibu[i] = z4;
            if (A.mimic) {
                au[i] = ld4(A.a_user + b * D + c);
                tp[i] = ld4(A.t_item + pb * ldt + c);
                ap[i] = ld4(A.a_item + pb * ldt + c);
                tu[i] = ld4(A.t_user + b * D + c);
            }
            if (ib) {
                ibp[i] = ld4(A.ib_dp + b * A.ib_ld + c);
                ibu[i] = ld4(A.ib_du + b * D + c);
            }
        }
        float dot = 0.f;
#pragma unroll
        for (int i = 0; i < NV; ++i) dot += dot4(u[i], p[i]);
        const float sp = group_sum(dot, G);
        float dsp = 0.f;
        if (!ib) {
            dsp = (1.0f / (1.0f + expf(-sp)) - 1.0f) * inv_numel;
            bce += bce_logit(sp, 1.0f);
        }
        float4 du[NV], dpos[NV];
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            dpos[i] = ib ? ibp[i] : scale4(dsp, u[i]);
            du[i] = ib ? ibu[i] : scale4(dsp, p[i]);
            st4(A.dT_item + pb * ldi + 4 * (s + G * i), dpos[i]);
        }
        for (int j0 = 0; j0 < N; j0 += NG) {
            const int ng = N - j0 < NG ? N - j0 : NG;
            int64_t nr[NG];
            float4 nv[NG][NV];
#pragma unroll
            for (int jj = 0; jj < NG; ++jj) {
                nr[jj] = 0;
                if (jj < ng) {
                    const int64_t q = B + b * N + j0 + jj;
                    nr[jj] = A.item_slot ? A.item_slot[q] : q;
                }
#pragma unroll
                for (int i = 0; i < NV; ++i) nv[jj][i] = jj < ng ? item_row(nr[jj], 4 * (s + G * i), true) : z4;
            }
            float sn[NG];
#pragma unroll
            for (int jj = 0; jj < NG; ++jj) {
                float dn = 0.f;
#pragma unroll
                for (int i = 0; i < NV; ++i) dn += dot4(u[i], nv[jj][i]);
                sn[jj] = group_sum(dn, G);
            }
#pragma unroll
            for (int jj = 0; jj < NG; ++jj) {
                if (jj >= ng) continue;
                const float dsn = (1.0f / (1.0f + expf(-sn[jj])) - 0.0f) * inv_numel;
                bce += bce_logit(sn[jj], 0.0f);
#pragma unroll
                for (int i = 0; i < NV; ++i) {
                    const int c = 4 * (s + G * i);
                    const float4 g = scale4(dsn, u[i]);
                    st4(A.dT_item + nr[jj] * ldi + c, g);
                    if (A.mimic && A.dA_all) st4(A.dA_item + nr[jj] * ldi + c, g);
                    du[i] = fma4(dsn, nv[jj][i], du[i]);
                }
            }
        }
        const float norm = 2.0f / (float)(A.Bg * D);
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const int c = 4 * (s + G * i);
            st4(A.dT_user + b * D + c, du[i]);
            if (A.mimic) {
                const float4 xu = make_float4(au[i].x - tp[i].x, au[i].y - tp[i].y, au[i].z - tp[i].z, au[i].w - tp[i].w);
                const float4 xi = make_float4(ap[i].x - tu[i].x, ap[i].y - tu[i].y, ap[i].z - tu[i].z, ap[i].w - tu[i].w);
                mse_u += dot4(xu, xu);
                mse_i += dot4(xi, xi);
                st4(A.dA_user + b * D + c, fma4(norm * A.lambda_u, xu, du[i]));
                st4(A.dA_item + pb * ldi + c, fma4(norm * A.lambda_i, xi, dpos[i]));
            }
        }
    }
    // every lane of a group holds the group's BCE terms: count them once
    bce = wave_sum(s == 0 ? bce : 0.f);
    mse_u = wave_sum(mse_u);
    mse_i = wave_sum(mse_i);
    if (lane == 0) {
        red[w][0] = bce;
        red[w][1] = mse_u;
        red[w][2] = mse_i;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        float t = 0.f;
        for (int i = 0; i < kScoreWaves; ++i) t += red[i][threadIdx.x];
        A.partials[blockIdx.x * 3 + threadIdx.x] = t;
    }
}

// Deterministic final reduction of the per-block partials; total loss as in training.py:798-803.
__global__ void loss_finalize_kernel(const float* __restrict__ partials, int blocks, const float* __restrict__ ib_partials,
                                     int ib_blocks, int64_t bce_count, int64_t B, int64_t Bg, int D,
                                     float lu, float li, int mimic, const float* __restrict__ cal, float lcal,
                                     float* __restrict__ loss_out, double* __restrict__ loss_accum,
                                     const uint32_t* __restrict__ status) {
    __shared__ float red[3][256];
    float s[3] = {0.f, 0.f, 0.f};
    for (int i = threadIdx.x; i < blocks; i += blockDim.x)
        for (int k = 0; k < 3; ++k) s[k] += partials[i * 3 + k];
    for (int i = threadIdx.x; i < ib_blocks; i += blockDim.x) s[0] += ib_partials[i];
    for (int k = 0; k < 3; ++k) red[k][threadIdx.x] = s[k];
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if (threadIdx.x < o)
            for (int k = 0; k < 3; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        // sharded step: this rank's share of the global means (the host sums loss_out over ranks)
        const float bce = red[0][0] / (float)bce_count;
        const float mu = red[1][0] / (float)(Bg * D);
        const float mi = red[2][0] / (float)(Bg * D);
        float total = bce;
        if (mimic && lu > 0.f) total = total + lu * mu;
        if (mimic && li > 0.f) total = total + li * mi;
        const float lc = cal ? cal[0] : 0.f;  // category alignment (training.py:805-820)
        if (cal && lcal > 0.f) total = total + lcal * lc;
        loss_out[0] = total;
        loss_out[1] = bce;
        loss_out[2] = mimic ? mu : 0.f;
        loss_out[3] = mimic ? mi : 0.f;
        loss_out[4] = lc;
        if (loss_accum && !step_poisoned(status)) {
            loss_accum[0] += (double)total * (double)Bg;
            loss_accum[1] += (double)B;
        }
    }
}

// mean((x - y)^2), one block, fixed reduction order (F.mse_loss, reduction='mean').
__global__ void mse_kernel(const float* __restrict__ x, const float* __restrict__ y, int64_t n, float* __restrict__ out) {
    __shared__ float red[1024];
    float s = 0.f;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
        const float d = x[i] - y[i];
        s += d * d;
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[0] = red[0] / (float)n;
}

inline unsigned grid_for(int64_t work, int threads = 256) {
    int64_t g = ceil_div(work, threads);
    if (g > 65536) g = 65536;
    if (g < 1) g = 1;
    return (unsigned)g;
}

// torch embedding_renorm_ on the rows a lookup touches (encoders.py:48,58 max_norm)
__global__ void renorm_rows_kernel(float* __restrict__ table, int64_t table_rows, int dim,
                                   const int64_t* __restrict__ idx, int64_t n, double max_norm,
                                   int32_t* __restrict__ mark, int32_t tag, const int64_t* __restrict__ keys,
                                   int64_t key_split, int key_phase) {
    const int64_t p = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (p >= n) return;
    if (keys && (keys[p] >= key_split) != (key_phase != 0)) return;  // the other lookup's positions
    const int64_t row = idx[p];
    if (row < 0 || row >= table_rows) return;  // reported by the staging kernel
    int claimed = 0;
    if (lane == 0) claimed = atomicExch(&mark[row], tag) != tag;
    claimed = __shfl(claimed, 0);
    if (!claimed) return;
    float* r = table + row * (int64_t)dim;
    float ss = 0.f;
    for (int c = lane; c < dim; c += 64) ss += r[c] * r[c];
    ss = wave_sum(ss);
    const float norm = sqrtf(ss);
    if ((double)norm > max_norm) {  // torch: norm > max_norm, scale = max_norm / (norm + 1e-7) in double
        const float scale = (float)(max_norm / ((double)norm + 1e-7));
        for (int c = lane; c < dim; c += 64) r[c] = r[c] * scale;
    }
}

}  // namespace

int launch_renorm_rows(float* table, int64_t table_rows, int dim, const int64_t* idx, int64_t n, double max_norm,
                       int32_t* mark, int32_t tag, hipStream_t s, const int64_t* keys, int64_t key_split,
                       int key_phase) {
    if (n <= 0) return TTAMM_OK;
    TTAMM_REQUIRE(mark != nullptr && max_norm > 0.0 && tag != 0, "renorm: bad arguments");
    hipLaunchKernelGGL(renorm_rows_kernel, dim3((unsigned)ceil_div(n, 4)), dim3(256), 0, s, table, table_rows, dim, idx, n,
                       max_norm, mark, tag, keys, key_split, key_phase);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

int launch_gather_rows(const float* table, int64_t table_rows, int dim, const int64_t* idx, int64_t n, float* out,
                       int64_t out_ld, hipStream_t s) {
    if (n <= 0) return TTAMM_OK;
    const bool vec = (dim % 4 == 0) && (out_ld % 4 == 0) && ((uintptr_t)table % 16 == 0) &&
                     ((uintptr_t)out % 16 == 0);
    const int d4 = dim / 4;
    auto wide = [&](auto K) {
        constexpr int D4 = decltype(K)::value;
        const int64_t rows_per_block = (int64_t)WideGather<D4>::RPW * 4;
        int64_t blocks = ceil_div(n, rows_per_block);
        if (blocks > 8192) blocks = 8192;  // grid-stride beyond ~4 resident rounds
        hipLaunchKernelGGL(gather_rows_wide<D4>, dim3((unsigned)blocks), dim3(256), 0, s,
                           reinterpret_cast<const float4*>(table), table_rows, idx, n, reinterpret_cast<float4*>(out),
                           out_ld / 4);
    };
    auto try_wide = [&]() -> bool {
        switch (d4) {  // the row widths of the supported configurations (D, 2D, H up to 256 floats)
            case 8: wide(std::integral_constant<int, 8>{}); return true;
            case 16: wide(std::integral_constant<int, 16>{}); return true;
            case 24: wide(std::integral_constant<int, 24>{}); return true;
            case 32: wide(std::integral_constant<int, 32>{}); return true;
            case 48: wide(std::integral_constant<int, 48>{}); return true;
            case 64: wide(std::integral_constant<int, 64>{}); return true;
            default: return false;
        }
    };
    if (vec && try_wide()) {
        // launched
    } else if (vec) {
        hipLaunchKernelGGL(gather_rows_vec4, dim3(grid_for(n * (dim / 4))), dim3(256), 0, s, table, table_rows,
                           dim / 4, idx, n, out, out_ld);
    } else {
        hipLaunchKernelGGL(gather_rows_scalar, dim3(grid_for(n * dim)), dim3(256), 0, s, table, table_rows, dim, idx,
                           n, out, out_ld);
    }
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

int launch_gather_rows_segs(const GatherSegs& g, hipStream_t s) {
    TTAMM_REQUIRE(g.count >= 0 && g.count <= 2, "gather: at most two segments");
    bool one = g.count == 2;
    int d4 = 0;
    int64_t most = 0;
    for (int i = 0; i < g.count; ++i) {
        const GatherSeg& q = g.seg[i];
        one = one && q.dim == g.seg[0].dim && q.dim % 4 == 0 && q.out_ld % 4 == 0 &&
              ((uintptr_t)q.table | (uintptr_t)q.out) % 16 == 0;
        d4 = q.dim / 4;
        most = q.n > most ? q.n : most;
    }
    auto seg = [&](auto K) {
        constexpr int D4 = decltype(K)::value;
        const int64_t rows_per_block = (int64_t)WideGather<D4>::RPW * 4;
        int64_t blocks = ceil_div(most, rows_per_block);
        if (blocks > 8192) blocks = 8192;
        hipLaunchKernelGGL(gather_rows_wide_seg<D4>, dim3((unsigned)blocks, 2), dim3(256), 0, s, g);
        return true;
    };
    bool done = false;
    if (one && most > 0) {
        switch (d4) {
            case 8: done = seg(std::integral_constant<int, 8>{}); break;
            case 16: done = seg(std::integral_constant<int, 16>{}); break;
            case 24: done = seg(std::integral_constant<int, 24>{}); break;
            case 32: done = seg(std::integral_constant<int, 32>{}); break;
            case 48: done = seg(std::integral_constant<int, 48>{}); break;
            case 64: done = seg(std::integral_constant<int, 64>{}); break;
            default: break;
        }
    }
    if (done) {
        TTAMM_LAUNCH_CHECK();
        return TTAMM_OK;
    }
    for (int i = 0; i < g.count; ++i) {
        const GatherSeg& q = g.seg[i];
        const int rc = launch_gather_rows(q.table, q.rows, q.dim, q.idx, q.n, q.out, q.out_ld, s);
        if (rc) return rc;
    }
    return TTAMM_OK;
}

int launch_pad_rows_segs(const PadSegs& p, hipStream_t s) {
    TTAMM_REQUIRE(p.count >= 0 && p.count <= 2, "pad rows: at most two segments");
    if (p.count == 0) return TTAMM_OK;
    int64_t most = 0;
    for (int i = 0; i < p.count; ++i) most = p.seg[i].rows * p.seg[i].ld_dst > most ? p.seg[i].rows * p.seg[i].ld_dst : most;
    if (most == 0) return TTAMM_OK;
    hipLaunchKernelGGL(pad_rows_seg_kernel, dim3(grid_for(most), p.count), dim3(256), 0, s, p);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

// The gated fusion's output pass for the generic (two-GEMM) gate: x = the second gate GEMM's
// pre-activation (bias added, stored in g by an EPI_STORE launch), then per element
// g = sigmoid(x) (in place), t = g e + (1 - g) f, a = table[idx], aug = t + a (aug may be null:
// the sharded item owner) — gemm.hip's EPI_GATE_OUT epilogue as a streaming kernel, whose
// per-row operand loads and four output streams left the GEMM waiting on memory (C5: 187 us,
// 75 % of its wave-cycles waiting, profiles/r04_s41_c5_sq_counters.txt).  As a pass of its own:
// C5 1.576 -> 1.566 ms/step, C4 0.958 -> 0.952 (profiles/r04_s42_gate_mix.txt).
__global__ void gate_mix_kernel(float* __restrict__ g, const float* __restrict__ ef, const float* __restrict__ table,
                                const int64_t* __restrict__ idx, int64_t n, int dim, float* __restrict__ t,
                                float* __restrict__ a, int64_t ld_ta, float* __restrict__ aug) {
    const int d4 = dim / 4;
    const int64_t total = n * d4;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t row = i / d4;
        const int c = (int)(i - row * d4) * 4;
        const float4 x = ld4(g + row * dim + c);
        const float* efr = ef + row * 2 * dim;
        const float4 ev = ld4(efr + c), fv = ld4(efr + dim + c);
        const float4 av = table ? ld4(table + idx[row] * (int64_t)dim + c) : make_float4(0.f, 0.f, 0.f, 0.f);
        const float xs[4] = {x.x, x.y, x.z, x.w}, e4[4] = {ev.x, ev.y, ev.z, ev.w}, f4[4] = {fv.x, fv.y, fv.z, fv.w};
        const float a4[4] = {av.x, av.y, av.z, av.w};
        float gg[4], tt[4], uu[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            gg[e] = 1.0f / (1.0f + __expf(-xs[e]));
            tt[e] = gg[e] * e4[e] + (1.0f - gg[e]) * f4[e];
            uu[e] = table ? tt[e] + a4[e] : tt[e];
        }
        st4(g + row * dim + c, make_float4(gg[0], gg[1], gg[2], gg[3]));
        st4(t + row * ld_ta + c, make_float4(tt[0], tt[1], tt[2], tt[3]));
        if (table) st4(a + row * ld_ta + c, av);
        if (aug) st4(aug + row * dim + c, make_float4(uu[0], uu[1], uu[2], uu[3]));
    }
}

int launch_gate_mix(float* g, const float* ef, const float* table, const int64_t* idx, int64_t n, int dim, float* t,
                    float* a, int64_t ld_ta, float* aug, hipStream_t s) {
    TTAMM_REQUIRE(dim % 4 == 0 && ld_ta % 4 == 0, "gate mix: dim and ld must be multiples of 4");
    if (n <= 0) return TTAMM_OK;
    hipLaunchKernelGGL(gate_mix_kernel, dim3(grid_for(n * (dim / 4))), dim3(256), 0, s, g, ef, table, idx, n, dim, t, a,
                       ld_ta, aug);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

int launch_combine(const float* e, int64_t ld_e, const float* f, int64_t ld_f, const float* table,
                   int64_t table_rows, const int64_t* idx, int64_t n, int dim, float* t, float* a, int64_t ld_ta, float* aug,
                   hipStream_t s) {
    if (n <= 0) return TTAMM_OK;
    hipLaunchKernelGGL(combine_kernel, dim3(grid_for(n * dim)), dim3(256), 0, s, e, ld_e, f, ld_f, table, table_rows, idx, n,
                       dim, t, a, ld_ta, aug);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

int launch_mse(const float* x, const float* y, int64_t n, float* out, hipStream_t s) {
    TTAMM_REQUIRE(n > 0, "mse_loss: empty input");
    hipLaunchKernelGGL(mse_kernel, dim3(1), dim3(1024), 0, s, x, y, n, out);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

int launch_pad_rows(const float* src, int64_t rows, int cols, int64_t ld_src, float* dst, int ld_dst,
                    hipStream_t s) {
    if (rows <= 0) return TTAMM_OK;
    hipLaunchKernelGGL(pad_rows_kernel, dim3(grid_for(rows * ld_dst)), dim3(256), 0, s, src, rows, cols, ld_src, dst,
                       ld_dst);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

int launch_gate_dq(const float* dT, int64_t ld_dT, const float* ef, const float* g, int64_t n, int dim, float* dq,
                   hipStream_t s) {
    if (n <= 0) return TTAMM_OK;
    hipLaunchKernelGGL(gate_dq_kernel, dim3(grid_for(n * dim)), dim3(256), 0, s, dT, ld_dT, ef, g, n, dim, dq);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

static int score_group(int D);
int launch_score_loss(const ScoreArgs& a, hipStream_t s) {
    TTAMM_REQUIRE(a.D <= 64 * kMaxDChunks, "score: embedding dim too large (max 512)");
    TTAMM_REQUIRE(a.N >= (a.ib_du ? 0 : 1) && a.N <= kMaxNeg, "score: negatives_per_positive out of range");
    if (a.B <= 0) return TTAMM_OK;
    const dim3 g(a.blocks), t(64 * kScoreWaves);
    TTAMM_REQUIRE(a.blocks == score_blocks(a.B, a.D), "score: partials sized for another batch");
    // 16-B aligned rows: every leading dimension a multiple of 4 floats
    const uintptr_t ptrs = (uintptr_t)a.user_aug | (uintptr_t)a.item_aug | (uintptr_t)a.t_user | (uintptr_t)a.t_item |
                           (uintptr_t)a.a_user | (uintptr_t)a.a_item | (uintptr_t)a.dT_user | (uintptr_t)a.dT_item |
                           (uintptr_t)a.dA_user | (uintptr_t)a.dA_item | (uintptr_t)a.ib_du | (uintptr_t)a.ib_dp;
    const bool al = ptrs % 16 == 0 && a.ld_item % 4 == 0 && a.ld_dti % 4 == 0 && (!a.ib_dp || a.ib_ld % 4 == 0);
    if (al && score_group(a.D)) {
        switch (a.D) {
            case 32: hipLaunchKernelGGL((score_loss_v_kernel<8, 1>), g, t, 0, s, a); break;
            case 64: hipLaunchKernelGGL((score_loss_v_kernel<8, 2>), g, t, 0, s, a); break;
            case 96: hipLaunchKernelGGL((score_loss_v_kernel<8, 3>), g, t, 0, s, a); break;
            case 128: hipLaunchKernelGGL((score_loss_v_kernel<8, 4>), g, t, 0, s, a); break;
            case 192: hipLaunchKernelGGL((score_loss_v_kernel<16, 3>), g, t, 0, s, a); break;
            case 256: hipLaunchKernelGGL((score_loss_v_kernel<16, 4>), g, t, 0, s, a); break;
            case 384: hipLaunchKernelGGL((score_loss_v_kernel<16, 6>), g, t, 0, s, a); break;
            default: hipLaunchKernelGGL((score_loss_v_kernel<16, 8>), g, t, 0, s, a); break;
        }
        TTAMM_LAUNCH_CHECK();
        return TTAMM_OK;
    }
    switch ((a.D + 63) / 64) {
        case 1: hipLaunchKernelGGL(score_loss_kernel<1>, g, t, 0, s, a); break;
        case 2: hipLaunchKernelGGL(score_loss_kernel<2>, g, t, 0, s, a); break;
        case 3: hipLaunchKernelGGL(score_loss_kernel<3>, g, t, 0, s, a); break;
        case 4: hipLaunchKernelGGL(score_loss_kernel<4>, g, t, 0, s, a); break;
        case 5: case 6: hipLaunchKernelGGL(score_loss_kernel<6>, g, t, 0, s, a); break;
        default: hipLaunchKernelGGL(score_loss_kernel<8>, g, t, 0, s, a); break;
    }
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

// lanes per interaction of score_loss_v_kernel for this D, or 0 (score_loss_kernel)
static int score_group(int D) {
    if (D == 32 || D == 64 || D == 96 || D == 128) return 8;
    if (D == 192 || D == 256 || D == 384 || D == 512) return 16;
    return 0;
}
int score_blocks(int64_t B, int D) {
    const int G = score_group(D);
    return (int)ceil_div(B, G ? (int64_t)kScoreWaves * (64 / G) : kScoreWaves);
}

int launch_loss_finalize(const float* partials, int blocks, const float* ib_partials, int ib_blocks, int64_t bce_count,
                         int64_t B, int64_t Bg, int D, float lu, float li, int mimic, const float* cal, float lcal,
                         float* loss_out, double* loss_accum, const uint32_t* status, hipStream_t s) {
    hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(256), 0, s, partials, blocks, ib_partials, ib_blocks,
                       bce_count, B, Bg, D, lu, li, mimic, cal, lcal, loss_out, loss_accum, status);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

}  // namespace ttamm

namespace ttamm {

namespace {
// out = x (+ y), row-wise over [n, dim]
__global__ void add_rows_kernel(const float* __restrict__ x, int64_t ldx, const float* __restrict__ y, int64_t ldy,
                                int64_t n, int dim, float* __restrict__ out, int64_t ldo,
                                const int64_t* __restrict__ xrow) {
    const int64_t total = n * dim;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / dim;
        const int c = (int)(i - r * dim);
        const int64_t q = xrow ? xrow[r] : r;
        const float v = x[q * ldx + c];
        out[r * ldo + c] = y ? v + y[q * ldy + c] : v;
    }
}
}  // namespace

namespace {
// dst[idx[r]] += (x[r] - y[r]) * scale * (*scale_dev) (idx null: row r), rows with idx[r] != skip_row; float
// atomics (the order of duplicate rows' adds is not fixed: torch's CUDA embedding backward and
// index_add_ are not either).  Module-level autograd only: the fused step sums in a fixed order.
__global__ void scatter_add_rows_kernel(float* __restrict__ dst, int dim, const int64_t* __restrict__ idx, int64_t n,
                                        const float* __restrict__ x, int64_t ldx, const float* __restrict__ y,
                                        int64_t ldy, const float* __restrict__ scale_dev, float scale,
                                        int64_t skip_row, int64_t dst_rows) {
    const float sc = scale_dev ? scale * *scale_dev : scale;
    const int64_t total = n * dim;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / dim;
        const int c = (int)(i - r * dim);
        const int64_t row = idx ? idx[r] : r;
        if (row == skip_row || row < 0 || row >= dst_rows) continue;  // never write outside dst
        float v = x[r * ldx + c];
        if (y) v = v - y[r * ldy + c];
        atomicAdd(dst + row * dim + c, v * sc);
    }
}
}  // namespace

int launch_scatter_add_rows(float* dst, int64_t dst_rows, int dim, const int64_t* idx, int64_t n, const float* x,
                            int64_t ldx, const float* y, int64_t ldy, const float* scale_dev, float scale,
                            int64_t skip_row, hipStream_t s) {
    if (n <= 0) return TTAMM_OK;
    hipLaunchKernelGGL(scatter_add_rows_kernel, dim3(grid_for(n * dim)), dim3(256), 0, s, dst, dim, idx, n, x, ldx, y,
                       ldy, scale_dev, scale, skip_row, dst_rows);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

int launch_add_rows(const float* x, int64_t ldx, const float* y, int64_t ldy, int64_t n, int dim, float* out,
                    int64_t ldo, hipStream_t s, const int64_t* xrow) {
    if (n <= 0) return TTAMM_OK;
    hipLaunchKernelGGL(add_rows_kernel, dim3(grid_for(n * dim)), dim3(256), 0, s, x, ldx, y, ldy, n, dim, out, ldo,
                       xrow);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

int launch_stage_rows(const StageArgs& a, hipStream_t s) {
    TTAMM_REQUIRE(a.count >= 0 && a.count <= kMaxStageSegs, "stage_rows: bad arguments");
    int64_t most = 0;
    for (int i = 0; i < a.count; ++i) most = a.seg[i].n > most ? a.seg[i].n : most;
    const bool units = a.unit_out != nullptr && a.unit_n > 0;
    TTAMM_REQUIRE(!units || (a.unit_counts && a.unit_ld >= 3 && a.unit_groups >= 1 && a.unit_groups <= 1024),
                  "stage_rows: bad unit-map arguments");
    if (units) most = a.unit_n > most ? a.unit_n : most;
    if (most == 0) return TTAMM_OK;
    hipLaunchKernelGGL(stage_rows_kernel, dim3(grid_for(most), a.count + (units ? 1 : 0)), dim3(256),
                       units ? 3 * sizeof(int64_t) * a.unit_groups : 0, s, a);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

}  // namespace ttamm
