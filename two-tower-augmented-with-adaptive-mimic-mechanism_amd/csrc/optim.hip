// Optimizer side of the training step: gradient coalescing for the row tables and the
// fused SparseAdam / AdamW updates.
//
// Row tables receive per-row gradient contributions from the batch (duplicates allowed).
// They are grouped by row (launch_coalesce: counts and first occurrences through per-row
// scratch, a one-block scan, a scatter, then each row's positions put back in ascending order),
// so duplicate rows are summed in batch order — the order torch's CPU index_add / coalesce use
// (training.py:822 backward; _functional.py:44 grad.coalesce()).
//
// Tables in the dense group (the adaptive-mimic tables, adaptive_mimic.py:35-36, put in the
// AdamW group by training.py:306-307) are updated over EVERY row every step.  That sweep is
// split into (1) an AdamW update of the touched rows with their gradient into a side buffer,
// (2) a pure streaming AdamW(g = 0) pass over the whole table — the dominant HBM kernel of
// the step, 24 bytes per element — and (3) a scatter of the side rows over the swept table.
// The result equals one dense AdamW step over the full dense gradient.
#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cmath>
#include <cstring>

#include <type_traits>

#include "kernels.h"

#pragma clang fp contract(off)

namespace ttamm {

namespace {

// torch single-tensor Adam/AdamW (adam.py:419-547):
//   p *= 1 - lr*wd ; m.lerp_(g, 1-b1) ; v = v*b2 + (1-b2)*g*g ;
//   p += -step * m / (sqrt(v)/sqrt(bc2) + eps)
// G0: the gradient is the literal 0 (an untouched dense-table row): lerp(m, 0, w) =
// m + w*(0 - m) == fma(w, -m, m) and v*b2 + (1-b2)*0*0 == v*b2 (v >= +0), bit for bit.
// FAST (g = 0 rows only, ttamm.h TTAMM_G0_FAST): sqrt and 1/denom from v_sqrt_f32 / v_rcp_f32
// (<= 1 ulp each) and a multiply by RN(1 / sqrt(bc2)) — a third of the IEEE sequences' VALU work.
template <bool DECOUPLED, bool G0 = false, bool FAST = false>
__device__ __forceinline__ void adam_elem_t(float& p, float& m, float& v, float g, const AdamConsts& c) {
    if (DECOUPLED) {
        p = p * c.decay;
    } else if (c.wd != 0.f) {
        g = g + p * c.wd;
    }
    if (G0 && DECOUPLED) {
        m = fmaf(c.w1, -m, m);
        v = v * c.b2;
    } else {
        m = fmaf(c.w1, g - m, m);  // ATen lerp (|w| < 0.5): self + w * (end - self), vectorised as fmadd
        v = v * c.b2;
        v = v + c.w2 * g * g;
    }
    if constexpr (FAST) {
        static_assert(G0, "fast arithmetic is for the g = 0 updates only");
        // the step folded into the reciprocal: r = neg_step / denom = rcp(sqrt(v) * fast_ibc +
        // fast_eps), p = fma(m, r, p): one multiply fewer per element than m * rcp(denom) scaled
        // by neg_step, and the denominator's fma pairs into v_pk_fma_f32 (replay_kernel).  The
        // replay is VALU-issue-bound.  m and v stay bit-exact (torch's operations); p moves by the
        // same update term within a few ulp.
        const float d = fmaf(__builtin_amdgcn_sqrtf(v), c.fast_ibc, c.fast_eps);
        p = fmaf(m, __builtin_amdgcn_rcpf(d), p);
    } else {
        const float denom = div_by_const(sqrtf(v), c.bc2_sqrt, c.inv_bc2_sqrt) + c.eps;
        p = p + c.neg_step * (m / denom);
    }
}

// torch.optim.SGD single-tensor step (sgd.py _single_tensor_sgd; training.py:1324-1330):
//   grad = grad.add(param, alpha=wd)                  ATen add: fmadd(param, wd, grad)
//   buf  = grad.clone() (first step) | buf.mul_(momentum).add_(grad, alpha=1 - dampening)
//   grad = grad.add(buf, alpha=momentum) (nesterov) | buf ;  param.add_(grad, alpha=-lr)
// m is the momentum buffer; v aliases it (or, momentum == 0, both alias the parameter), so the
// callers' three stores all write the value that belongs at that address.
__device__ __forceinline__ void sgd_elem(float& p, float& m, float& v, float g, const AdamConsts& c) {
    if (c.wd != 0.f) g = fmaf(p, c.wd, g);
    if (c.sgd_mom != 0.f) {
        const float buf = c.sgd_first ? g : fmaf(g, c.sgd_damp1, m * c.sgd_mom);
        g = c.sgd_nesterov ? fmaf(buf, c.sgd_mom, g) : buf;
        p = fmaf(g, c.sgd_neg_lr, p);
        m = v = buf;
    } else {
        p = fmaf(g, c.sgd_neg_lr, p);
        m = v = p;
    }
}

__device__ __forceinline__ void adam_elem(float& p, float& m, float& v, float g, const AdamConsts& c) {
    if (c.sgd)
        sgd_elem(p, m, v, g, c);
    else if (c.decoupled)
        adam_elem_t<true>(p, m, v, g, c);
    else
        adam_elem_t<false>(p, m, v, g, c);
}
__device__ __forceinline__ void adam_elem_g0(float& p, float& m, float& v, const AdamConsts& c) {
    if (c.sgd) {
        sgd_elem(p, m, v, 0.f, c);
    } else if (c.fast_g0) {
        if (c.decoupled)
            adam_elem_t<true, true, true>(p, m, v, 0.f, c);
        else
            adam_elem_t<false, true, true>(p, m, v, 0.f, c);
    } else if (c.decoupled) {
        adam_elem_t<true, true>(p, m, v, 0.f, c);
    } else {
        adam_elem_t<false, true>(p, m, v, 0.f, c);
    }
}

// torch SparseAdam on one coalesced element (_functional.py:61-84).
__device__ __forceinline__ void sparse_adam_elem(float& p, float& m, float& v, float g, const SparseConsts& c) {
    const float om = m, ov = v;
    float um = (g - om) * c.w1;
    float uv = (g * g - ov) * c.w2;
    m = om + um;
    v = ov + uv;
    const float numer = um + om;
    const float denom = sqrtf(uv + ov) + c.eps;
    p = p + c.neg_step * (numer / denom);
}

// ---- grouping of a batch's row ids (launch_coalesce) ----------------------------------------
// first[key] holds INT_MAX - (first position): 0 = untouched, and atomicMax keeps the earliest.
__global__ void co_count_kernel(const int64_t* __restrict__ idx, int64_t n, int32_t* __restrict__ cnt,
                                int32_t* __restrict__ first) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const int64_t key = idx[p];
    atomicAdd(&cnt[key], 1);
    atomicMax(&first[key], (int32_t)(INT_MAX - p));
}

// co_count_kernel over up to two towers (blockIdx.y = tower); each tower's first block also
// zeroes its catch-up list counters (CatchupList cnt + fill), which the next launch reads
__global__ void co_count_seg_kernel(PrepSegs) {
    const KArg(PrepSegs)* ka = (const KArg(PrepSegs)*)(__builtin_amdgcn_kernarg_segment_ptr());
    const KArg(PrepSeg)& S = ka->seg[blockIdx.y];
    if (blockIdx.x == 0 && S.list_cnt)
        for (int i = threadIdx.x; i < 2 * (ka->cap + 1); i += blockDim.x) S.list_cnt[i] = 0;  // cnt, fill
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= S.n) return;
    const int64_t key = S.idx[p];
    atomicAdd(&S.cnt[key], 1);
    atomicMax(&S.first[key], (int32_t)(INT_MAX - p));
}

// Entry i of the segment scan: (flag, count) — a position's leader flag and its row's count,
// or (sorted mode, entries = the key range) whether key i occurs and its count.
__device__ __forceinline__ void co_entry(int by_key, int64_t i, const int64_t* __restrict__ idx,
                                         const int32_t* __restrict__ cnt, const int32_t* __restrict__ first,
                                         int32_t& f, int32_t& c) {
    if (by_key) {
        c = cnt[i];
        f = c > 0;
    } else {
        const int64_t key = idx[i];
        f = first[key] == (int32_t)(INT_MAX - i);
        c = f ? cnt[key] : 0;
    }
}

// block-wide inclusive scan of (f, c) over 256 threads
__device__ __forceinline__ void block_scan2(int32_t& f, int32_t& c, int32_t* sf, int32_t* sc) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t a = __shfl_up(f, o, 64), b = __shfl_up(c, o, 64);
        if (lane >= o) {
            f += a;
            c += b;
        }
    }
    if (lane == 63) {
        sf[w] = f;
        sc[w] = c;
    }
    __syncthreads();
    int32_t pf = 0, pc = 0;
    for (int i = 0; i < w; ++i) {
        pf += sf[i];
        pc += sc[i];
    }
    f += pf;
    c += pc;
}

// pass 1 of the segment scan: each 256-entry tile's totals
__global__ __launch_bounds__(256) void co_tile_sum_kernel(int64_t n, int by_key, const int64_t* __restrict__ idx,
                                                          const int32_t* __restrict__ cnt,
                                                          const int32_t* __restrict__ first,
                                                          int32_t* __restrict__ tile_f, int32_t* __restrict__ tile_c) {
    __shared__ int32_t sf[4], sc[4];
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    int32_t f = 0, c = 0;
    if (i < n) co_entry(by_key, i, idx, cnt, first, f, c);
    block_scan2(f, c, sf, sc);
    if (threadIdx.x == 255) {
        tile_f[blockIdx.x] = f;
        tile_c[blockIdx.x] = c;
    }
}

// pass 2: exclusive scan of the tile totals (one block; tiles are few), n_unique, total
__global__ __launch_bounds__(1024) void co_tile_scan_kernel(int64_t tiles, int32_t* __restrict__ tile_f,
                                                            int32_t* __restrict__ tile_c, int32_t* __restrict__ seg_start,
                                                            int32_t* __restrict__ n_unique) {
    __shared__ int32_t sf[1024], sc[1024];
    const int t = threadIdx.x;
    const int64_t chunk = (tiles + 1023) / 1024;
    const int64_t lo = min(tiles, t * chunk), hi = min(tiles, lo + chunk);
    int32_t f_sum = 0, c_sum = 0;
    for (int64_t i = lo; i < hi; ++i) {
        f_sum += tile_f[i];
        c_sum += tile_c[i];
    }
    sf[t] = f_sum;
    sc[t] = c_sum;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const int32_t a = t >= o ? sf[t - o] : 0, b = t >= o ? sc[t - o] : 0;
        __syncthreads();
        sf[t] += a;
        sc[t] += b;
        __syncthreads();
    }
    int32_t rf = sf[t] - f_sum, rc = sc[t] - c_sum;
    for (int64_t i = lo; i < hi; ++i) {
        const int32_t a = tile_f[i], b = tile_c[i];
        tile_f[i] = rf;
        tile_c[i] = rc;
        rf += a;
        rc += b;
    }
    if (t == 1023) {
        n_unique[0] = sf[t];
        seg_start[sf[t]] = sc[t];
    }
}

// pass 3: every flagged entry's segment index and start; the index goes to lead[position]
// (first-occurrence order) or first[key] (sorted mode)
__global__ __launch_bounds__(256) void co_tile_write_kernel(int64_t n, int by_key, const int64_t* __restrict__ idx,
                                                            const int32_t* __restrict__ cnt, int32_t* __restrict__ first,
                                                            const int32_t* __restrict__ tile_f,
                                                            const int32_t* __restrict__ tile_c,
                                                            int32_t* __restrict__ lead, int32_t* __restrict__ seg_start) {
    __shared__ int32_t sf[4], sc[4];
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    int32_t f = 0, c = 0;
    if (i < n) co_entry(by_key, i, idx, cnt, first, f, c);
    int32_t fi = f, ci = c;
    block_scan2(fi, ci, sf, sc);
    if (f) {
        const int32_t u = tile_f[blockIdx.x] + fi - 1;
        seg_start[u] = tile_c[blockIdx.x] + ci - c;
        if (by_key) first[i] = u;
        else lead[i] = u;
    }
}

// every position into its row's segment (order within a segment: arbitrary, fixed next)
__global__ void co_fill_kernel(const int64_t* __restrict__ idx, int64_t n, int by_key,
                               const int32_t* __restrict__ lead, const int32_t* __restrict__ first,
                               int32_t* __restrict__ fill, const int32_t* __restrict__ seg_start,
                               int32_t* __restrict__ vals_tmp, int32_t* __restrict__ keys_out,
                               int32_t* __restrict__ n_big) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p == 0) n_big[0] = 0;  // the long-segment list of the ordering pass
    if (p >= n) return;
    const int64_t key = idx[p];
    const int32_t u = by_key ? first[key] : lead[INT_MAX - first[key]];  // the leader's segment
    const int32_t slot = seg_start[u] + atomicAdd(&fill[key], 1);
    vals_tmp[slot] = (int32_t)p;
    keys_out[slot] = (int32_t)key;
}

// Segment ordering: every segment's positions in ascending order (so duplicate rows sum in
// batch order), the long-segment flags, and the row's scratch back to zero.  One thread per
// segment sorts up to kOrderSmall positions in registers (nearly every row of a batch occurs
// once or a few times); longer segments (hot rows) are listed in `big` and ranked by whole
// blocks (co_order_big_kernel).
constexpr int kOrderSmall = 16;

__device__ __forceinline__ void co_reset(const CoalesceWs& W, int32_t key) {
    W.cnt[key] = 0;
    W.first[key] = 0;
    W.fill[key] = 0;
}

__global__ __launch_bounds__(256) void co_order_small_kernel(CoalesceWs W, int32_t* __restrict__ big,
                                                             int32_t* __restrict__ n_big) {
    const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= W.n_unique[0]) return;
    const int32_t k0 = W.seg_start[u], L = W.seg_start[u + 1] - k0;
    if (L > kOrderSmall) {
        big[atomicAdd(n_big, 1)] = (int32_t)u;
        return;
    }
    int32_t v[kOrderSmall];
#pragma unroll
    for (int i = 0; i < kOrderSmall; ++i) v[i] = i < L ? W.vals_tmp[k0 + i] : INT_MAX;
#pragma unroll
    for (int i = 1; i < kOrderSmall; ++i)  // insertion sort, fully unrolled (registers only)
#pragma unroll
        for (int j = i; j > 0; --j) {
            const int32_t a = v[j - 1], b = v[j];
            v[j - 1] = min(a, b);
            v[j] = max(a, b);
        }
    const int32_t longseg = L > kCoalescePiece ? 1 : 0;
#pragma unroll
    for (int i = 0; i < kOrderSmall; ++i)
        if (i < L) {
            W.vals_out[k0 + i] = v[i];
            W.seglong[k0 + i] = longseg;
        }
    co_reset(W, W.keys_out[k0]);
}

// Long segments: the positions are distinct integers, so each one's rank within the segment is
// the number of the segment's positions below it — a bitmap over the segment's position range in
// LDS, per-word prefix popcounts, one lookup per position: O(range / 32 + L) per segment (a
// Zipf-hot item of a C2 batch spans ~50K positions: 1.5K words).  A range wider than the bitmap
// falls back to counting ranks (L^2 / threads).
constexpr int kBitWords = 6144;  // position range up to 196,608 (48 KB of LDS with the prefixes)
__global__ __launch_bounds__(256) void co_order_big_kernel(CoalesceWs W, const int32_t* __restrict__ big,
                                                           const int32_t* __restrict__ n_big) {
    __shared__ uint32_t bits[kBitWords];
    __shared__ int32_t pre[kBitWords];
    __shared__ int32_t sf[4], sc[4], smin[4], smax[4];
    const int nb = n_big[0];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int b = blockIdx.x; b < nb; b += gridDim.x) {
        const int32_t u = big[b];
        const int32_t k0 = W.seg_start[u], k1 = W.seg_start[u + 1], L = k1 - k0;
        const int32_t longseg = L > kCoalescePiece ? 1 : 0;
        // the segment's position range
        int32_t lo = INT_MAX, hi = -1;
        for (int32_t j = threadIdx.x; j < L; j += blockDim.x) {
            const int32_t v = W.vals_tmp[k0 + j];
            lo = min(lo, v);
            hi = max(hi, v);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            lo = min(lo, __shfl_xor(lo, o, 64));
            hi = max(hi, __shfl_xor(hi, o, 64));
        }
        __syncthreads();  // the previous segment's LDS reads are done
        if (lane == 0) {
            smin[wv] = lo;
            smax[wv] = hi;
        }
        __syncthreads();
        lo = min(min(smin[0], smin[1]), min(smin[2], smin[3]));
        hi = max(max(smax[0], smax[1]), max(smax[2], smax[3]));
        const int32_t nw = ((hi - lo) >> 5) + 1;
        if (nw <= kBitWords) {
            for (int32_t w = threadIdx.x; w < nw; w += blockDim.x) bits[w] = 0u;
            __syncthreads();
            for (int32_t j = threadIdx.x; j < L; j += blockDim.x) {
                const int32_t d = W.vals_tmp[k0 + j] - lo;
                atomicOr(&bits[d >> 5], 1u << (d & 31));
            }
            __syncthreads();
            // exclusive prefix of the words' popcounts: contiguous chunks per thread, block scan
            const int32_t chunk = (nw + (int32_t)blockDim.x - 1) / (int32_t)blockDim.x;
            const int32_t w0 = min(nw, (int32_t)threadIdx.x * chunk), w1 = min(nw, w0 + chunk);
            int32_t c = 0;
            for (int32_t w = w0; w < w1; ++w) c += __popc(bits[w]);
            int32_t f = 0, ci = c;
            block_scan2(f, ci, sf, sc);
            int32_t run = ci - c;
            for (int32_t w = w0; w < w1; ++w) {
                pre[w] = run;
                run += __popc(bits[w]);
            }
            __syncthreads();
            for (int32_t j = threadIdx.x; j < L; j += blockDim.x) {
                const int32_t v = W.vals_tmp[k0 + j];
                const int32_t d = v - lo;
                const int32_t r = pre[d >> 5] + __popc(bits[d >> 5] & ((1u << (d & 31)) - 1u));
                W.vals_out[k0 + r] = v;
            }
        } else {
            for (int32_t j = threadIdx.x; j < L; j += blockDim.x) {
                const int32_t v = W.vals_tmp[k0 + j];
                int32_t rank = 0;
                for (int32_t i = k0; i < k1; ++i) rank += W.vals_tmp[i] < v ? 1 : 0;
                W.vals_out[k0 + rank] = v;
            }
        }
        for (int32_t j = threadIdx.x; j < L; j += blockDim.x) W.seglong[k0 + j] = longseg;
        if (threadIdx.x == 0) co_reset(W, W.keys_out[k0]);
    }
}

// Segmented sum of the row-gradient contributions, in two fixed-order levels so a hot row
// (a popular item with hundreds of duplicates in the batch) does not serialise one wave:
//   piece_sum: one wave per chunk of kPiece sorted positions sums each run of equal keys
//              inside its chunk ("piece") and stores it at the run's first position;
//   row_update: one wave per unique row adds its pieces in position order, then applies
//              the optimizer.  Both orders are fixed, so results are deterministic.
constexpr int kPiece = kCoalescePiece;
constexpr int kRowWaves = 4;

__device__ __forceinline__ const float* dA_row(const RowUpdateArgs& A, int64_t r) {
    // the fields as values first: a select between the two pointer FIELDS of the by-value kernel
    // argument compiled to a select of their addresses, copying the argument to scratch (24 B per
    // lane in row_update_kernel)
    const float* const lo = A.dA_lo;
    const float* const hi = A.dA_hi;
    const int64_t ld = A.ld_dA;
    if (const int64_t* xu = A.xu) {
        const int64_t u = xu[r];
        return u >= 0 ? lo + u * ld : hi + (~u) * ld;
    }
    return (r < A.split_row ? lo : hi) + r * ld;
}

// SDA: each position's dA row resolved once into LDS (compact exchange unit maps: their dependent
// load); otherwise per column from its row (TTAMM_PIECE_SDA=1 forces SDA)
template <bool SDA>
__global__ __launch_bounds__(64 * kRowWaves) void piece_sum_kernel(RowUpdateArgs A) {
    __shared__ int64_t srows[kRowWaves][kPiece];
    __shared__ const float* sda[kRowWaves][kPiece];  // each position's dA row (resolved once: GateTower::xu)
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t chunk = (int64_t)blockIdx.x * kRowWaves + w;
    const int64_t k0 = chunk * kPiece;
    if (k0 >= A.n) return;
    const int cnt = (int)min((int64_t)kPiece, A.n - k0);
    // only segments longer than a piece are summed in two levels (row_update sums the rest)
    if (__ballot(lane < cnt && A.seglong[k0 + lane] != 0) == 0ull) return;
    // positions of the chunk: lane p holds row / key / "last of a run" for position k0 + p
    int64_t my_row = 0;
    int my_key = 0, my_last = 1;
    if (lane < cnt) {
        my_row = A.rows[k0 + lane];
        my_key = A.keys[k0 + lane];
    }
    const int next_key = __shfl_down(my_key, 1, 64);
    if (lane + 1 < cnt) my_last = next_key != my_key;
    const uint64_t last_mask = __ballot(lane < cnt && my_last);
    const bool mimic = A.mimic.weight != nullptr;
    if (lane < kPiece) {  // read back uniformly inside the d loop
        srows[w][lane] = my_row;
        if (SDA) sda[w][lane] = mimic && lane < cnt ? dA_row(A, my_row) : nullptr;
    }
    __builtin_amdgcn_wave_barrier();
    const int D = A.dim;
    const bool idt = A.id.weight != nullptr;  // (a mimic-only pass leaves the ID table out)
    // SDA = false (no unit maps, launch_row_update): buffer loads, the position's row offset in the
    // scalar offset (the row is wave-uniform) and the column in one shared voffset — 64-bit
    // addresses per load had held the kernel at 288 registers, one wave per SIMD
    [[maybe_unused]] __amdgpu_buffer_rsrc_t rE, rAlo, rAhi;
    if constexpr (!SDA) {
        rE = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(A.dE), 0, 0x7fffffff, 0x00020000);
        rAlo = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(A.dA_lo), 0, 0x7fffffff, 0x00020000);
        rAhi = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(A.dA_hi), 0, 0x7fffffff, 0x00020000);
    }
    for (int d = lane; d < D; d += 64) {
        float ve[kPiece], va[kPiece];
#pragma unroll
        for (int p = 0; p < kPiece; ++p) {  // issue every load of the chunk before adding
            if constexpr (SDA) {
                const int64_t r = srows[w][p];
                ve[p] = (idt && p < cnt) ? A.dE[r * A.ld_dE + d] : 0.f;
                va[p] = (mimic && p < cnt) ? sda[w][p][d] : 0.f;
            } else {
                const int r = __builtin_amdgcn_readfirstlane((int)srows[w][p]);
                ve[p] = (idt && p < cnt)
                    ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rE, 4 * d, (int)(4 * r * A.ld_dE), 0))
                    : 0.f;
                va[p] = (mimic && p < cnt)
                    ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r < A.split_row ? rAlo : rAhi, 4 * d,
                                                                                     (int)(4 * r * A.ld_dA), 0))
                    : 0.f;
            }
        }
        float ge = 0.f, ga = 0.f;
        int start = 0;
#pragma unroll
        for (int p = 0; p < kPiece; ++p) {
            if (p < cnt) {
                ge += ve[p];
                ga += va[p];
                if ((last_mask >> p) & 1ull) {
                    if (idt) A.piece_e[(k0 + start) * D + d] = ge;
                    if (mimic) A.piece_a[(k0 + start) * D + d] = ga;
                    ge = ga = 0.f;
                    start = p + 1;
                }
            }
        }
    }
}

// float4 views of table / gradient rows (dim % 4 == 0, 16-byte aligned rows: checked by the
// launcher)
__device__ __forceinline__ float4 ldf4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void stf4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ float4 addf4(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }

// One unique row per `lanes_per_row` lanes, NV float4 columns per lane (lanes_per_row = dim /
// (4 NV), a power of two: D = 96 -> 8 lanes x 3 float4s, eight rows per wave, every lane busy),
// all of a row's table and gradient loads issued before its arithmetic (developer variant, measured
// slower: launch_row_update).  NV = 0 (default): any dim, lanes_per_row the power of two >= dim / 4
// (at most 64), one float4 column per trip of a runtime loop.
template <int NV>
__global__ __launch_bounds__(64 * kRowWaves) void row_update_kernel(RowUpdateArgs A) {
    constexpr int C = NV > 0 ? NV : 1;
    const int lane = threadIdx.x & 63;
    const int lpr = A.lanes_per_row, rpw = 64 / lpr;
    const int64_t u = ((int64_t)blockIdx.x * kRowWaves + (threadIdx.x >> 6)) * rpw + lane / lpr;
    const int sub = lane % lpr;
    if (u >= A.n || u >= (int64_t)A.n_unique[0] || step_poisoned(A.status)) return;
    const int64_t k0 = A.seg_start[u], k1 = A.seg_start[u + 1];
    const int64_t key = A.keys[k0];
    const int D = A.dim;
    const bool mimic = A.mimic.weight != nullptr;
    const bool idt = A.id.weight != nullptr;  // (a mimic-only pass leaves the ID table out)
    const bool direct = k1 - k0 <= kPiece;
    // nn.Embedding padding_idx: no gradient into that row (SparseAdam: not in the sparse gradient at
    // all, so the row is left as it is; AdamW: a zero gradient row)
    const bool pad_row = idt && A.id.has_padding_idx && key == A.id.padding_idx;
    auto each = [](float4& p, float4& m, float4& v, float4 g, auto&& f) {
        f(p.x, m.x, v.x, g.x);
        f(p.y, m.y, v.y, g.y);
        f(p.z, m.z, v.z, g.z);
        f(p.w, m.w, v.w, g.w);
    };
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int d0 = 4 * sub; d0 < D; d0 += 4 * lpr * C) {  // NV > 0: one trip
        int dc[C];
        float4 ip[C], im[C], iv[C], mp[C], mm[C], mv[C], ge[C], ga[C];
        // the table rows first: they do not depend on the gradient sums below
#pragma unroll
        for (int i = 0; i < C; ++i) {
            dc[i] = d0 + i * 4 * lpr;
            const int64_t o = key * D + dc[i];
            ip[i] = idt ? ldf4(A.id.weight + o) : z4;
            im[i] = idt ? ldf4(A.id.exp_avg + o) : z4;
            iv[i] = idt ? ldf4(A.id.exp_avg_sq + o) : z4;
            mp[i] = mimic ? ldf4(A.mimic.weight + o) : z4;
            mm[i] = mimic ? ldf4(A.mimic.exp_avg + o) : z4;
            mv[i] = mimic ? ldf4(A.mimic.exp_avg_sq + o) : z4;
        }
        if (direct) {  // the row's contributions in batch order
            const int64_t r0 = A.rows[k0];
            const float* e0 = A.dE + r0 * A.ld_dE;
            const float* a0 = mimic ? dA_row(A, r0) : nullptr;
#pragma unroll
            for (int i = 0; i < C; ++i) {
                ge[i] = idt ? ldf4(e0 + dc[i]) : z4;
                ga[i] = mimic ? ldf4(a0 + dc[i]) : z4;
            }
            for (int64_t k = k0 + 1; k < k1; ++k) {
                const int64_t r = A.rows[k];
                const float* er = A.dE + r * A.ld_dE;
                const float* ar = mimic ? dA_row(A, r) : nullptr;
#pragma unroll
                for (int i = 0; i < C; ++i) {
                    if (idt) ge[i] = addf4(ge[i], ldf4(er + dc[i]));
                    if (mimic) ga[i] = addf4(ga[i], ldf4(ar + dc[i]));
                }
            }
        } else {  // pieces (piece_sum_kernel), then the pieces in order
#pragma unroll
            for (int i = 0; i < C; ++i) {
                ge[i] = idt ? ldf4(A.piece_e + k0 * D + dc[i]) : z4;
                ga[i] = mimic ? ldf4(A.piece_a + k0 * D + dc[i]) : z4;
            }
            for (int64_t k = (k0 / kPiece + 1) * kPiece; k < k1; k += kPiece) {
#pragma unroll
                for (int i = 0; i < C; ++i) {
                    if (idt) ge[i] = addf4(ge[i], ldf4(A.piece_e + k * D + dc[i]));
                    if (mimic) ga[i] = addf4(ga[i], ldf4(A.piece_a + k * D + dc[i]));
                }
            }
        }
#pragma unroll
        for (int i = 0; i < C; ++i) {
            const int d = dc[i];
            const int64_t o = key * D + d;
            if (A.grad_scale) {  // clip_grad_norm_: g *= coef (training.py:824-825)
                const float c = *A.grad_scale;
                ge[i] = make_float4(ge[i].x * c, ge[i].y * c, ge[i].z * c, ge[i].w * c);
                ga[i] = make_float4(ga[i].x * c, ga[i].y * c, ga[i].z * c, ga[i].w * c);
            }
            if (pad_row) ge[i] = z4;
            if (!idt) {
                // mimic-only pass
            } else if (A.id.optimizer == TTAMM_OPT_SPARSE_ADAM) {
                if (!pad_row)
                    each(ip[i], im[i], iv[i], ge[i],
                         [&](float& p, float& m, float& v, float g) { sparse_adam_elem(p, m, v, g, A.sp); });
            } else {
                each(ip[i], im[i], iv[i], ge[i], [&](float& p, float& m, float& v, float g) { adam_elem(p, m, v, g, A.ad); });
            }
            if (!idt || (A.id.optimizer == TTAMM_OPT_SPARSE_ADAM && pad_row)) {
                // untouched
            } else if (A.id.optimizer == TTAMM_OPT_SPARSE_ADAM || A.id.last_step) {
                // SparseAdam, or deferred mode: the row was caught up before the forward
                stf4(A.id.weight + o, ip[i]);
                stf4(A.id.exp_avg + o, im[i]);
                stf4(A.id.exp_avg_sq + o, iv[i]);
            } else {
                float* sd = A.side_id + u * 3 * D;
                stf4(sd + d, ip[i]);
                stf4(sd + D + d, im[i]);
                stf4(sd + 2 * D + d, iv[i]);
            }
            if (mimic) {
                each(mp[i], mm[i], mv[i], ga[i], [&](float& p, float& m, float& v, float g) { adam_elem(p, m, v, g, A.ad); });
                if (A.mimic.last_step) {
                    stf4(A.mimic.weight + o, mp[i]);
                    stf4(A.mimic.exp_avg + o, mm[i]);
                    stf4(A.mimic.exp_avg_sq + o, mv[i]);
                } else {
                    float* sd = A.side_mimic + u * 3 * D;
                    stf4(sd + d, mp[i]);
                    stf4(sd + D + d, mm[i]);
                    stf4(sd + 2 * D + d, mv[i]);
                }
            }
        }
    }
    if (sub == 0) {
        if (idt && A.id.optimizer != TTAMM_OPT_SPARSE_ADAM && A.id.last_step) {
            A.id.last_step[key] = A.dense_step;
            if (A.id.touched && !pad_row) A.id.touched[key] = 1;
        }
        if (mimic && A.mimic.last_step) {
            A.mimic.last_step[key] = A.dense_step;
            if (A.mimic.touched) A.mimic.touched[key] = 1;
        }
    }
}

// Streaming AdamW(g = 0) over whole tables: 12 B read + 12 B written per element.
__global__ __launch_bounds__(256) void dense_sweep_kernel(SweepArgs A) {
    if (step_poisoned(A.status)) return;
    for (int s = 0; s < A.count; ++s) {
        const SweepSeg& S = A.seg[s];
        const int64_t n4 = S.n >> 2;
        float4* P = reinterpret_cast<float4*>(S.p);
        float4* Mm = reinterpret_cast<float4*>(S.m);
        float4* V = reinterpret_cast<float4*>(S.v);
        const int64_t stride = (int64_t)gridDim.x * blockDim.x;
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
            float4 p = P[i], m = Mm[i], v = V[i];
            adam_elem_g0(p.x, m.x, v.x, A.ad);
            adam_elem_g0(p.y, m.y, v.y, A.ad);
            adam_elem_g0(p.z, m.z, v.z, A.ad);
            adam_elem_g0(p.w, m.w, v.w, A.ad);
            P[i] = p;
            Mm[i] = m;
            V[i] = v;
        }
        // scalar tail
        for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < S.n; i += stride) {
            float p = S.p[i], m = S.m[i], v = S.v[i];
            adam_elem_g0(p, m, v, A.ad);
            S.p[i] = p;
            S.m[i] = m;
            S.v[i] = v;
        }
    }
}

// ---- deferred exact AdamW(g = 0) ----------------------------------------------------------
constexpr int kMaxHistory = kMaxAdamHistory;

__global__ void step_begin_kernel(const uint32_t* status, int64_t* applied, AdamConsts* hist, int cap, int64_t step,
                                  AdamConsts c) {
    if (threadIdx.x != 0 || blockIdx.x != 0 || step_poisoned(status)) return;
    if (applied) applied[0] += 1;
    if (hist) hist[step % cap] = c;
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

// The per-step constants a g = 0 replay reads (the AdamW fast path loads the first 24 B)
struct ReplayConsts {
    float decay, w1, b2, eps, neg_step, inv_bc2_sqrt, bc2_sqrt, wd, w2, fast_ibc, fast_eps, pad0;
};
// The fast decoupled replay's constants as element pairs (each value twice), read as whole 64-bit
// operands by the packed loop.  Built from one float, the compiler broadcast it into both halves
// of a v_pk_* with op_sel, and picked a destination pair whose low register was that broadcast
// source (v_pk_fma_f32 v[48:49], v[54:55], v[48:49], v[48:49] op_sel_hi:[1,0,1]); run beside the
// feature MLP's GEMMs on the main stream, that replay gave run-to-run different parameters
// (tools/diag/deferred_c2.py, profiles/r04_replay_pk_overlap.txt).  With pair operands the halves
// of every packed instruction read only their own lane.
struct ReplayPairs {
    f32x2 decay, w1, b2, ibc, eps;
    float pad0, pad1;
};
static_assert(sizeof(ReplayPairs) == sizeof(ReplayConsts), "one LDS ring size for both layouts");

__device__ __forceinline__ float lo_of(float x) { return x; }
__device__ __forceinline__ float lo_of(f32x2 x) { return x.x; }

// One thread per V float4s of a row (dim % (4 V) == 0: 4 V independent dependency chains per
// thread sharing each step's constants, at float4 columns q and q + dim / (4 V)); blockIdx.y =
// segment.  A row current to step l is brought to A.target by replaying adam_elem(g = 0) with
// the constants of steps l+1 .. target — the operations the eager sweep applies, so the bits
// agree.  Rows come from a range (the rolling slice, the flush: untouched rows of one slice share
// their lag) or from a catch-up list sorted by lag (launch_catchup_list), so the lanes of a wave
// run one trip count.
template <bool DECOUPLED, bool FAST, int V>
__global__ __launch_bounds__(256) void replay_kernel(ReplayArgs) {
    constexpr bool PKL = DECOUPLED && FAST;  // the packed-pair loop
    using HC = typename std::conditional<PKL, ReplayPairs, ReplayConsts>::type;
    const KArg(ReplayArgs)* ka = (const KArg(ReplayArgs)*)(__builtin_amdgcn_kernarg_segment_ptr());
    const KArg(ReplaySeg)& S = ka->seg[blockIdx.y];
    if (step_poisoned(ka->status)) return;
    // the history ring unrolled twice in LDS (2 cap entries, sized at launch: ~6 KB by default),
    // so a row's steps l+1 .. target are consecutive entries from (l + 1) % cap — no wrap test
    // and no address arithmetic beyond a pointer increment in the VALU-bound loop
    extern __shared__ __attribute__((aligned(16))) unsigned char replay_lds[];
    HC* H2 = reinterpret_cast<HC*>(replay_lds);
    const int cap = ka->cap;
    for (int i = threadIdx.x; i < 2 * cap; i += blockDim.x) {
        const AdamConsts& h = ka->hist[i < cap ? i : i - cap];
        if constexpr (PKL)
            H2[i] = ReplayPairs{f32x2{h.decay, h.decay}, f32x2{h.w1, h.w1}, f32x2{h.b2, h.b2},
                                f32x2{h.fast_ibc, h.fast_ibc}, f32x2{h.fast_eps, h.fast_eps}, 0.f, 0.f};
        else
            H2[i] = ReplayConsts{h.decay, h.w1, h.b2, h.eps, h.neg_step, h.inv_bc2_sqrt, h.bc2_sqrt, h.wd, h.w2,
                                 h.fast_ibc, h.fast_eps, 0.f};
    }
    __syncthreads();
    const int dim = S.dim;
    const uint32_t per_row = (uint32_t)(dim >> 2) / V;  // threads per row
    const int32_t target = ka->target;
    const bool by_list = S.list_rows != nullptr;
    const uint32_t nrows = by_list ? (uint32_t)S.list_cnt[0] : (uint32_t)(S.row_hi - S.row_lo);
    const uint32_t total = nrows * per_row;
    for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
        const uint32_t r = e / per_row, q = e - r * per_row;
        int64_t row;
        int32_t l;
        if (by_list) {
            row = S.list_rows[r];
            l = target - S.list_lag[r];
        } else {
            row = S.row_lo + r;
            l = S.last[row];
            if (l >= target) continue;
        }
        const int64_t o = row * dim + 4 * (int64_t)q;
        const HC* hc = H2 + (l + 1) % cap;
        const HC* const hend = hc + (target - l);
        if (DECOUPLED && S.touched && S.touched[row] == 0) {
            // a row never given a gradient: m = v = +0.0 stay so, and each step is p *= decay
            // (the cold path below, bit for bit) — only the parameter row moves
            float4 p[V];
#pragma unroll
            for (int i = 0; i < V; ++i) p[i] = *reinterpret_cast<const float4*>(S.p + o + (int64_t)(4 * per_row) * i);
            for (; hc != hend; ++hc) {
                const float decay = lo_of(hc->decay);
#pragma unroll
                for (int i = 0; i < V; ++i)
                    p[i].x = p[i].x * decay, p[i].y = p[i].y * decay, p[i].z = p[i].z * decay, p[i].w = p[i].w * decay;
            }
#pragma unroll
            for (int i = 0; i < V; ++i) *reinterpret_cast<float4*>(S.p + o + (int64_t)(4 * per_row) * i) = p[i];
            continue;
        }
        float4 p[V], m[V], v[V];
#pragma unroll
        for (int i = 0; i < V; ++i) {
            const int64_t oi = o + (int64_t)(4 * per_row) * i;
            p[i] = *reinterpret_cast<const float4*>(S.p + oi);
            m[i] = *reinterpret_cast<const float4*>(S.m + oi);
            v[i] = *reinterpret_cast<const float4*>(S.v + oi);
        }
        // A cold row (first moment +0.0: never given a gradient) stays cold under g = 0 (m = fma(w1,
        // -0, 0) = +0), and its update term neg_step * (0 * r) is -0.0, which leaves p * decay
        // unchanged for every p — so its replay is p *= decay, v *= b2 per step, bit for bit what
        // the full update computes, without the two transcendentals.  Most rows of a large table
        // are cold for many steps (C4: the in-batch positives touch ~8 K of 6.25 M rows a step).
        uint32_t mbits = 0u, vbits = 0u;
#pragma unroll
        for (int i = 0; i < V; ++i) {
            mbits |= __float_as_uint(m[i].x) | __float_as_uint(m[i].y) | __float_as_uint(m[i].z) | __float_as_uint(m[i].w);
            vbits |= __float_as_uint(v[i].x) | __float_as_uint(v[i].y) | __float_as_uint(v[i].z) | __float_as_uint(v[i].w);
        }
        // a cold row's m is unchanged (+0.0), and a virgin row's v too (+0.0 * b2 = +0.0): their
        // stores are skipped (the flush after a short run is mostly such rows: 24 -> 16 B per element)
        const bool keep_m = DECOUPLED && mbits == 0u, keep_v = keep_m && vbits == 0u;
        if (DECOUPLED && mbits == 0u) {
            for (; hc != hend; ++hc) {
                const float decay = lo_of(hc->decay), b2 = lo_of(hc->b2);
#pragma unroll
                for (int i = 0; i < V; ++i) {
                    p[i].x = p[i].x * decay, p[i].y = p[i].y * decay, p[i].z = p[i].z * decay, p[i].w = p[i].w * decay;
                    v[i].x = v[i].x * b2, v[i].y = v[i].y * b2, v[i].z = v[i].z * b2, v[i].w = v[i].w * b2;
                }
            }
        }
        if constexpr (PKL) {
            // adam_elem_t<true, true, true> on element pairs, written with 2-wide vectors so every
            // multiply / fma issues as one v_pk_* for two elements (the denominator's fma included):
            // the same IEEE operations per element, so the dense sweep's scalar form gives the same bits
            for (; hc != hend; ++hc) {
                const f32x2 decay = hc->decay, w1 = hc->w1, b2 = hc->b2, ibc = hc->ibc, eps = hc->eps;
#pragma unroll
                for (int i = 0; i < V; ++i) {
#pragma unroll
                    for (int half = 0; half < 2; ++half) {
                        f32x2 P = half ? f32x2{p[i].z, p[i].w} : f32x2{p[i].x, p[i].y};
                        f32x2 M = half ? f32x2{m[i].z, m[i].w} : f32x2{m[i].x, m[i].y};
                        f32x2 Q = half ? f32x2{v[i].z, v[i].w} : f32x2{v[i].x, v[i].y};
                        P = P * decay;
                        M = __builtin_elementwise_fma(w1, -M, M);
                        Q = Q * b2;
                        const f32x2 Sq = {__builtin_amdgcn_sqrtf(Q.x), __builtin_amdgcn_sqrtf(Q.y)};
                        const f32x2 Dn = __builtin_elementwise_fma(Sq, ibc, eps);
                        const f32x2 R = {__builtin_amdgcn_rcpf(Dn.x), __builtin_amdgcn_rcpf(Dn.y)};
                        P = __builtin_elementwise_fma(M, R, P);
                        if (half) {
                            p[i].z = P.x, p[i].w = P.y, m[i].z = M.x, m[i].w = M.y, v[i].z = Q.x, v[i].w = Q.y;
                        } else {
                            p[i].x = P.x, p[i].y = P.y, m[i].x = M.x, m[i].y = M.y, v[i].x = Q.x, v[i].y = Q.y;
                        }
                    }
                }
            }
        } else {
            for (; hc != hend; ++hc) {
                AdamConsts c;
                c.decay = hc->decay, c.w1 = hc->w1, c.b2 = hc->b2, c.eps = hc->eps, c.neg_step = hc->neg_step;
                c.bc2_sqrt = hc->bc2_sqrt, c.inv_bc2_sqrt = hc->inv_bc2_sqrt, c.wd = hc->wd, c.w2 = hc->w2;
                c.fast_ibc = hc->fast_ibc, c.fast_eps = hc->fast_eps;
                c.decoupled = DECOUPLED ? 1 : 0, c.fast_g0 = FAST ? 1 : 0;
#pragma unroll
                for (int i = 0; i < V; ++i) {
                    adam_elem_t<DECOUPLED, true, FAST>(p[i].x, m[i].x, v[i].x, 0.f, c);
                    adam_elem_t<DECOUPLED, true, FAST>(p[i].y, m[i].y, v[i].y, 0.f, c);
                    adam_elem_t<DECOUPLED, true, FAST>(p[i].z, m[i].z, v[i].z, 0.f, c);
                    adam_elem_t<DECOUPLED, true, FAST>(p[i].w, m[i].w, v[i].w, 0.f, c);
                }
            }
        }
#pragma unroll
        for (int i = 0; i < V; ++i) {
            const int64_t oi = o + (int64_t)(4 * per_row) * i;
            *reinterpret_cast<float4*>(S.p + oi) = p[i];
            if (!keep_m) *reinterpret_cast<float4*>(S.m + oi) = m[i];
            if (!keep_v) *reinterpret_cast<float4*>(S.v + oi) = v[i];
        }
    }
}

// The same replay with the per-step constants in scalar registers.  A wave whose active lanes
// share one start step l (the slice: untouched rows of a slice share their lag; the catch-up
// lists: sorted by lag) reads step k's constants once for the wave with s_load from the history
// ring (constant address space, wave-uniform index), the next step's load issued before the
// current step's arithmetic — no LDS ring fill, no per-lane ds_read and pointer arithmetic in
// the VALU-bound loop.  Waves whose lanes straddle two lags take each lane's constants with
// vector loads (a few waves per launch).  Arithmetic and constants are replay_kernel's, bit for
// bit.
template <bool DECOUPLED, bool FAST>
__device__ __forceinline__ void replay_steps_g0(float4& p, float4& m, float4& v, const AdamConsts& c) {
    adam_elem_t<DECOUPLED, true, FAST>(p.x, m.x, v.x, 0.f, c);
    adam_elem_t<DECOUPLED, true, FAST>(p.y, m.y, v.y, 0.f, c);
    adam_elem_t<DECOUPLED, true, FAST>(p.z, m.z, v.z, 0.f, c);
    adam_elem_t<DECOUPLED, true, FAST>(p.w, m.w, v.w, 0.f, c);
}

template <typename H>
__device__ __forceinline__ AdamConsts consts_at(H h) {
    AdamConsts c;
    c.decay = h->decay, c.w1 = h->w1, c.b2 = h->b2, c.eps = h->eps, c.neg_step = h->neg_step;
    c.bc2_sqrt = h->bc2_sqrt, c.inv_bc2_sqrt = h->inv_bc2_sqrt, c.wd = h->wd, c.w2 = h->w2;
    c.fast_ibc = h->fast_ibc, c.fast_eps = h->fast_eps;
    c.decoupled = 0, c.fast_g0 = 0;
    return c;
}

template <bool DECOUPLED, bool FAST, int V>
__global__ __launch_bounds__(256) void replay_s_kernel(ReplayArgs) {
    const KArg(ReplayArgs)* ka = (const KArg(ReplayArgs)*)(__builtin_amdgcn_kernarg_segment_ptr());
    const KArg(ReplaySeg)& S = ka->seg[blockIdx.y];
    if (step_poisoned(ka->status)) return;
    const KArg(AdamConsts)* hist = (const KArg(AdamConsts)*)ka->hist;
    const int cap = ka->cap;
    const int dim = S.dim;
    const uint32_t per_row = (uint32_t)(dim >> 2) / V;  // threads per row
    const int32_t target = ka->target;
    const bool by_list = S.list_rows != nullptr;
    const uint32_t nrows = by_list ? (uint32_t)S.list_cnt[0] : (uint32_t)(S.row_hi - S.row_lo);
    const uint32_t total = nrows * per_row;
    for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
        const uint32_t r = e / per_row, q = e - r * per_row;
        int64_t row;
        int32_t l;
        if (by_list) {
            row = S.list_rows[r];
            l = target - S.list_lag[r];
        } else {
            row = S.row_lo + r;
            l = S.last[row];
            if (l >= target) continue;
        }
        const int64_t o = row * dim + 4 * (int64_t)q;
        float4 p[V], m[V], v[V];
#pragma unroll
        for (int i = 0; i < V; ++i) {
            const int64_t oi = o + (int64_t)(4 * per_row) * i;
            p[i] = *reinterpret_cast<const float4*>(S.p + oi);
            m[i] = *reinterpret_cast<const float4*>(S.m + oi);
            v[i] = *reinterpret_cast<const float4*>(S.v + oi);
        }
        uint32_t mbits = 0u;
#pragma unroll
        for (int i = 0; i < V; ++i)
            mbits |= __float_as_uint(m[i].x) | __float_as_uint(m[i].y) | __float_as_uint(m[i].z) | __float_as_uint(m[i].w);
        const bool cold = DECOUPLED && mbits == 0u;  // see replay_kernel: p *= decay, v *= b2
        const int32_t l0 = __builtin_amdgcn_readfirstlane(l);
        if (__builtin_amdgcn_ballot_w64(l != l0) == 0) {
            // wave-uniform start step: constants in SGPRs, step k + 1's loaded during step k
            const int32_t n = target - l0;
            int j = (l0 + 1) % cap;
            if (cold) {
                float decay = hist[j].decay, b2 = hist[j].b2;
                for (int32_t k = 0; k < n; ++k) {
                    j = j + 1 == cap ? 0 : j + 1;
                    const float nd = hist[j].decay, nb = hist[j].b2;
#pragma unroll
                    for (int i = 0; i < V; ++i) {
                        p[i].x = p[i].x * decay, p[i].y = p[i].y * decay, p[i].z = p[i].z * decay, p[i].w = p[i].w * decay;
                        v[i].x = v[i].x * b2, v[i].y = v[i].y * b2, v[i].z = v[i].z * b2, v[i].w = v[i].w * b2;
                    }
                    decay = nd, b2 = nb;
                }
            } else {
                AdamConsts c = consts_at(hist + j);
                for (int32_t k = 0; k < n; ++k) {
                    j = j + 1 == cap ? 0 : j + 1;
                    const AdamConsts nc = consts_at(hist + j);
#pragma unroll
                    for (int i = 0; i < V; ++i) replay_steps_g0<DECOUPLED, FAST>(p[i], m[i], v[i], c);
                    c = nc;
                }
            }
        } else {
            // lanes of two or more start steps: per-lane constants
            int j = (l + 1) % cap;
            for (int32_t k = l; k < target; ++k) {
                const AdamConsts c = consts_at((const AdamConsts*)ka->hist + j);
                j = j + 1 == cap ? 0 : j + 1;
#pragma unroll
                for (int i = 0; i < V; ++i) replay_steps_g0<DECOUPLED, FAST>(p[i], m[i], v[i], c);
            }
        }
#pragma unroll
        for (int i = 0; i < V; ++i) {
            const int64_t oi = o + (int64_t)(4 * per_row) * i;
            *reinterpret_cast<float4*>(S.p + oi) = p[i];
            *reinterpret_cast<float4*>(S.m + oi) = m[i];
            *reinterpret_cast<float4*>(S.v + oi) = v[i];
        }
    }
}

// The deferred SGD(g = 0) replay (torch.optim.SGD in the dense group, training.py:1324-1330): an
// untouched row's step is p' = p + lr-scaled momentum of its own decay term,
//     g = p wd;  buf = fma(g, 1 - dampening, buf momentum) (buf = g on a first step);
//     p = fma(nesterov ? fma(buf, momentum, g) : buf, -lr, p)
// — linear in (p, buf), no transcendentals.  Each replayed step applies sgd_elem(g = 0) with that
// step's constants from the history ring (AdamConsts: sgd_neg_lr, sgd_mom, sgd_damp1, sgd_first,
// sgd_nesterov, wd), exactly the operations the eager sweep applies, so deferred == eager bit for
// bit.  momentum == 0: m and v alias the parameter (no state), the stores write p three times.
// Constants are read per lane from the ring in global memory (L1/L2-resident, a few dozen bytes a
// step); the loop is a handful of FMAs per element-step, so it is HBM-bound like the row traffic.
template <int V>
__global__ __launch_bounds__(256) void replay_sgd_kernel(ReplayArgs) {
    const KArg(ReplayArgs)* ka = (const KArg(ReplayArgs)*)(__builtin_amdgcn_kernarg_segment_ptr());
    const KArg(ReplaySeg)& S = ka->seg[blockIdx.y];
    if (step_poisoned(ka->status)) return;
    const AdamConsts* hist = ka->hist;
    const int cap = ka->cap;
    const int dim = S.dim;
    const uint32_t per_row = (uint32_t)(dim >> 2) / V;
    const int32_t target = ka->target;
    const bool by_list = S.list_rows != nullptr;
    const uint32_t nrows = by_list ? (uint32_t)S.list_cnt[0] : (uint32_t)(S.row_hi - S.row_lo);
    const uint32_t total = nrows * per_row;
    for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
        const uint32_t r = e / per_row, q = e - r * per_row;
        int64_t row;
        int32_t l;
        if (by_list) {
            row = S.list_rows[r];
            l = target - S.list_lag[r];
        } else {
            row = S.row_lo + r;
            l = S.last[row];
            if (l >= target) continue;
        }
        const int64_t o = row * dim + 4 * (int64_t)q;
        float4 p[V], m[V], v[V];
#pragma unroll
        for (int i = 0; i < V; ++i) {
            const int64_t oi = o + (int64_t)(4 * per_row) * i;
            p[i] = *reinterpret_cast<const float4*>(S.p + oi);
            m[i] = *reinterpret_cast<const float4*>(S.m + oi);
            v[i] = *reinterpret_cast<const float4*>(S.v + oi);
        }
        int j = (l + 1) % cap;
        for (int32_t k = l; k < target; ++k) {
            AdamConsts c = hist[j];
            c.sgd = 1;
            j = j + 1 == cap ? 0 : j + 1;
#pragma unroll
            for (int i = 0; i < V; ++i) {
                sgd_elem(p[i].x, m[i].x, v[i].x, 0.f, c);
                sgd_elem(p[i].y, m[i].y, v[i].y, 0.f, c);
                sgd_elem(p[i].z, m[i].z, v[i].z, 0.f, c);
                sgd_elem(p[i].w, m[i].w, v[i].w, 0.f, c);
            }
        }
#pragma unroll
        for (int i = 0; i < V; ++i) {
            const int64_t oi = o + (int64_t)(4 * per_row) * i;
            *reinterpret_cast<float4*>(S.p + oi) = p[i];
            *reinterpret_cast<float4*>(S.m + oi) = m[i];
            *reinterpret_cast<float4*>(S.v + oi) = v[i];
        }
    }
}

// row ranges only: last[row] = target (stamp 1) or max(last[row], target) (stamp 2) after the
// replay (list segments were stamped by their build)
__global__ void stamp_kernel(ReplayArgs) {
    const KArg(ReplayArgs)* ka = (const KArg(ReplayArgs)*)(__builtin_amdgcn_kernarg_segment_ptr());
    const KArg(ReplaySeg)& S = ka->seg[blockIdx.y];
    if (step_poisoned(ka->status) || S.list_rows != nullptr) return;
    const bool at_least = ka->stamp == 2;
    for (int64_t r = S.row_lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < S.row_hi;
         r += (int64_t)gridDim.x * blockDim.x) {
        if (at_least) atomicMax(&S.last[r], ka->target);
        else S.last[r] = ka->target;
    }
}

// ---- catch-up list (launch_catchup_list) ----------------------------------------------------
// lag of batch position p, or 0 when p is not its row's first occurrence or the row is current
__device__ __forceinline__ int32_t catchup_lag(const int64_t* __restrict__ idx, int64_t p, int64_t n,
                                               const int32_t* __restrict__ first, const int32_t* __restrict__ last,
                                               int32_t target, int64_t& row) {
    if (p >= n) return 0;
    row = idx[p];
    if (first[row] != (int32_t)(INT_MAX - p)) return 0;
    const int32_t lag = target - last[row];
    return lag > 0 ? lag : 0;
}

// rows per lag: a block histogram in LDS, then one atomic per (block, lag); cnt[0] = all rows
__device__ __forceinline__ void catchup_count_block(const int64_t* __restrict__ idx, int64_t n,
                                                    const int32_t* __restrict__ first, const int32_t* __restrict__ last,
                                                    int32_t target, int cap, int32_t* __restrict__ cnt, int32_t* h) {
    for (int i = threadIdx.x; i <= cap; i += blockDim.x) h[i] = 0;
    __syncthreads();
    int64_t row = 0;
    const int32_t lag = catchup_lag(idx, (int64_t)blockIdx.x * blockDim.x + threadIdx.x, n, first, last, target, row);
    if (lag > 0) {
        atomicAdd(&h[lag], 1);
        atomicAdd(&h[0], 1);
    }
    __syncthreads();
    for (int i = threadIdx.x; i <= cap; i += blockDim.x)
        if (h[i]) atomicAdd(&cnt[i], h[i]);
}

__global__ __launch_bounds__(256) void catchup_count_kernel(const int64_t* __restrict__ idx, int64_t n,
                                                            const int32_t* __restrict__ first,
                                                            const int32_t* __restrict__ last, int32_t target, int cap,
                                                            int32_t* __restrict__ cnt, const uint32_t* status) {
    __shared__ int32_t h[kMaxHistory + 1];
    if (step_poisoned(status)) return;
    catchup_count_block(idx, n, first, last, target, cap, cnt, h);
}

// both towers' lists in one launch (blockIdx.y = tower)
__global__ __launch_bounds__(256) void catchup_count_seg_kernel(PrepSegs) {
    const KArg(PrepSegs)* ka = (const KArg(PrepSegs)*)(__builtin_amdgcn_kernarg_segment_ptr());
    const KArg(PrepSeg)& S = ka->seg[blockIdx.y];
    __shared__ int32_t h[kMaxHistory + 1];
    if (step_poisoned(ka->status) || S.list_cnt == nullptr) return;
    catchup_count_block(S.idx, S.n, S.first, S.last[0], ka->target, ka->cap, S.list_cnt, h);
}

struct LastPtrs {
    int32_t* p[2];
};

// each listed row into its lag's range of the list (longest lag first: lag b starts at
// sum_{b' > b} cnt[b']), in block order within a lag (atomics: any order — every row's replay is
// independent of the others), then stamped current in every table of the tower
__device__ __forceinline__ void catchup_scatter_block(const int64_t* __restrict__ idx, int64_t n,
                                                      const int32_t* __restrict__ first, int32_t* const* last,
                                                      int nlast, int32_t target, int cap,
                                                      const int32_t* __restrict__ cnt, int32_t* __restrict__ fill,
                                                      int32_t* __restrict__ rows, int32_t* __restrict__ lags,
                                                      int32_t (*suf)[kMaxHistory + 2], int32_t* h, int32_t* base) {
    const int tid = threadIdx.x;
    for (int i = tid; i <= cap + 1; i += blockDim.x) {
        suf[0][i] = (i >= 1 && i <= cap) ? cnt[i] : 0;
        if (i <= cap) h[i] = 0;
    }
    __syncthreads();
    int cur = 0;
    for (int off = 1; off <= cap; off <<= 1) {  // Hillis-Steele suffix scan
        for (int i = tid; i <= cap + 1; i += blockDim.x)
            suf[cur ^ 1][i] = suf[cur][i] + (i + off <= cap ? suf[cur][i + off] : 0);
        cur ^= 1;
        __syncthreads();
    }
    int64_t row = 0;
    const int32_t lag = catchup_lag(idx, (int64_t)blockIdx.x * blockDim.x + tid, n, first, last[0], target, row);
    int32_t rank = 0;
    if (lag > 0) rank = atomicAdd(&h[lag], 1);
    __syncthreads();
    for (int i = tid + 1; i <= cap; i += blockDim.x)
        if (h[i]) base[i] = atomicAdd(&fill[i], h[i]);
    __syncthreads();
    if (lag > 0) {
        const int32_t slot = suf[cur][lag + 1] + base[lag] + rank;
        rows[slot] = (int32_t)row;
        lags[slot] = lag;
        for (int t = 0; t < nlast; ++t) last[t][row] = target;
    }
}

__global__ __launch_bounds__(256) void catchup_scatter_kernel(const int64_t* __restrict__ idx, int64_t n,
                                                              const int32_t* __restrict__ first, LastPtrs last,
                                                              int nlast, int32_t target, int cap,
                                                              const int32_t* __restrict__ cnt,
                                                              int32_t* __restrict__ fill, int32_t* __restrict__ rows,
                                                              int32_t* __restrict__ lags, const uint32_t* status) {
    __shared__ int32_t suf[2][kMaxHistory + 2];  // suffix sums of cnt[1..cap] (double buffered)
    __shared__ int32_t h[kMaxHistory + 1], base[kMaxHistory + 1];
    if (step_poisoned(status)) return;
    catchup_scatter_block(idx, n, first, last.p, nlast, target, cap, cnt, fill, rows, lags, suf, h, base);
}

__global__ __launch_bounds__(256) void catchup_scatter_seg_kernel(PrepSegs) {
    const KArg(PrepSegs)* ka = (const KArg(PrepSegs)*)(__builtin_amdgcn_kernarg_segment_ptr());
    const KArg(PrepSeg)& S = ka->seg[blockIdx.y];
    __shared__ int32_t suf[2][kMaxHistory + 2];
    __shared__ int32_t h[kMaxHistory + 1], base[kMaxHistory + 1];
    if (step_poisoned(ka->status) || S.list_cnt == nullptr) return;
    int32_t* last[2] = {S.last[0], S.last[1]};
    catchup_scatter_block(S.idx, S.n, S.first, last, S.nlast, ka->target, ka->cap, S.list_cnt,
                          S.list_cnt + (ka->cap + 1), S.list_rows, S.list_lag, suf, h, base);
}

__global__ void side_scatter_kernel(const int32_t* __restrict__ n_unique, const int32_t* __restrict__ keys,
                                    const int32_t* __restrict__ seg_start, const float* __restrict__ side, int64_t n,
                                    int dim, ttamm_table t, const uint32_t* __restrict__ status) {
    if (step_poisoned(status)) return;
    const int64_t total = n * dim;
    const int64_t nu = n_unique[0];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t u = i / dim;
        if (u >= nu) return;
        const int d = (int)(i - u * dim);
        const int64_t key = keys[seg_start[u]];
        const float* sd = side + u * 3 * dim;
        const int64_t o = key * dim + d;
        t.weight[o] = sd[d];
        t.exp_avg[o] = sd[dim + d];
        t.exp_avg_sq[o] = sd[2 * dim + d];
    }
}

__global__ void dense_adam_kernel(DenseAdamArgs A, int64_t total) {
    if (step_poisoned(A.status)) return;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        int64_t off = i;
        int t = 0;
        while (t < A.count - 1 && off >= A.t[t].n) {
            off -= A.t[t].n;
            ++t;
        }
        const DenseTensor& T = A.t[t];
        float p = T.p[off], m = T.m[off], v = T.v[off];
        adam_elem(p, m, v, A.grad_scale ? T.g[off] * *A.grad_scale : T.g[off], A.ad);
        T.p[off] = p;
        T.m[off] = m;
        T.v[off] = v;
    }
}

// ---- clip_grad_norm_ (training.py:824-825; torch/nn/utils/clip_grad.py) ---------------------
// sum over a tower table pair's touched rows of |sum of the row's gradient contributions|^2
// (the dense gradient tensor's rows; the padding row's ID gradient is zero), one thread per
// (row, 4 columns), the row's contributions summed in batch order
__global__ void rows_sumsq_kernel(RowUpdateArgs A, float* __restrict__ partials) {
    __shared__ float red[4];
    const int dim4 = A.dim >> 2;
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t u = e / dim4;
    float acc = 0.f;
    if (u < A.n && u < (int64_t)A.n_unique[0]) {
        const int d = (int)(e - u * dim4) * 4;
        const int64_t k0 = A.seg_start[u], k1 = A.seg_start[u + 1];
        const int64_t key = A.keys[k0];
        const bool mimic = A.mimic.weight != nullptr;
        float4 ge = make_float4(0.f, 0.f, 0.f, 0.f), ga = ge;
        for (int64_t k = k0; k < k1; ++k) {
            const int64_t r = A.rows[k];
            ge = addf4(ge, ldf4(A.dE + r * A.ld_dE + d));
            if (mimic) ga = addf4(ga, ldf4(dA_row(A, r) + d));
        }
        if (A.id.has_padding_idx && key == A.id.padding_idx) ge = make_float4(0.f, 0.f, 0.f, 0.f);
        acc = (ge.x * ge.x + ge.y * ge.y) + (ge.z * ge.z + ge.w * ge.w) +
              ((ga.x * ga.x + ga.y * ga.y) + (ga.z * ga.z + ga.w * ga.w));
    }
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) partials[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ void dense_sumsq_kernel(DenseAdamArgs A, int64_t total, float* __restrict__ partials) {
    __shared__ float red[4];
    float acc = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t off = i;
        int t = 0;
        while (t < A.count - 1 && off >= A.t[t].n) {
            off -= A.t[t].n;
            ++t;
        }
        const float g = A.t[t].g[off];
        acc += g * g;
    }
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) partials[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// one block: the partials summed in a fixed order (fp64), then torch's fp32 coefficient
// clip_coef = max_norm / (total_norm + 1e-6), clamped to <= 1
__global__ void clip_coef_kernel(const float* __restrict__ partials, int n, float max_norm, float* coef) {
    __shared__ double red[256];
    double acc = 0.0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) acc += (double)partials[i];
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const float total = (float)sqrt(red[0]);
        const float c = max_norm / (total + 1e-6f);
        *coef = c < 1.0f ? c : 1.0f;
    }
}


__global__ void sum_partials_kernel(const float* __restrict__ partials, int n, float* out) {
    __shared__ double red[256];
    double acc = 0.0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) acc += (double)partials[i];
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) *out = (float)red[0];
}

__global__ void sparse_adam_rows_kernel(float* __restrict__ w, float* __restrict__ m, float* __restrict__ v,
                                        int dim, const int64_t* __restrict__ rows, const float* __restrict__ grad,
                                        int64_t n, SparseConsts c) {
    const int64_t total = n * dim;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t u = i / dim;
        const int d = (int)(i - u * dim);
        const int64_t o = rows[u] * dim + d;
        float p = w[o], mm = m[o], vv = v[o];
        sparse_adam_elem(p, mm, vv, grad[i], c);
        w[o] = p;
        m[o] = mm;
        v[o] = vv;
    }
}

inline unsigned grid_for(int64_t work, int threads = 256, int64_t cap = 65536) {
    int64_t g = ceil_div(work, threads);
    if (g > cap) g = cap;
    if (g < 1) g = 1;
    return (unsigned)g;
}


}  // namespace

// RN(1/c) for a positive normal fp32 c: the double quotient rounded to fp32 may be off by one
// ulp (double rounding), so pick among it and its neighbours the one with the smallest
// |1 - y*c|, evaluated exactly in double (24-bit x 24-bit products fit in 53 bits).
float correctly_rounded_reciprocal(float c) {
    const float y0 = (float)(1.0 / (double)c);
    float best = y0;
    double err = std::fabs(1.0 - (double)y0 * (double)c);
    for (float y : {std::nextafter(y0, 0.f), std::nextafter(y0, INFINITY)}) {
        const double e = std::fabs(1.0 - (double)y * (double)c);
        if (e < err) {
            err = e;
            best = y;
        }
    }
    return best;
}

AdamConsts make_adam_consts(double lr, double beta1, double beta2, double eps, double wd, int decoupled,
                            int64_t step) {
    AdamConsts c;
    const double bc1 = 1.0 - std::pow(beta1, (double)step);
    const double bc2 = 1.0 - std::pow(beta2, (double)step);
    c.decay = (float)(1.0 - lr * wd);
    c.w1 = (float)(1.0 - beta1);
    c.b2 = (float)beta2;
    c.w2 = (float)(1.0 - beta2);
    c.eps = (float)eps;
    c.neg_step = (float)(-(lr / bc1));
    c.bc2_sqrt = (float)std::pow(bc2, 0.5);
    c.inv_bc2_sqrt = correctly_rounded_reciprocal(c.bc2_sqrt);
    const double ns = -(lr / bc1);
    if (ns != 0.0) {
        c.fast_ibc = (float)(1.0 / (std::sqrt(bc2) * ns));
        c.fast_eps = (float)(eps / ns);
    } else {  // lr = 0: r = rcp(+inf) = +0, p = fma(m, 0, p) = p (torch: p + (-0) * (m / denom))
        c.fast_ibc = 0.f;
        c.fast_eps = INFINITY;
    }
    c.wd = (float)wd;
    c.decoupled = decoupled;
    c.fast_g0 = 0;
    c.sgd = 0, c.sgd_neg_lr = 0.f, c.sgd_mom = 0.f, c.sgd_damp1 = 0.f, c.sgd_first = 0, c.sgd_nesterov = 0;
    return c;
}

AdamConsts make_sgd_consts(double lr, double wd, double momentum, double dampening, int nesterov, int first) {
    AdamConsts c;
    std::memset(&c, 0, sizeof(c));
    c.sgd = 1;
    c.sgd_neg_lr = (float)(-lr);
    c.wd = (float)wd;
    c.sgd_mom = (float)momentum;
    c.sgd_damp1 = (float)(1.0 - dampening);
    c.sgd_first = first ? 1 : 0;
    c.sgd_nesterov = nesterov ? 1 : 0;
    return c;
}

SparseConsts make_sparse_consts(double lr, double beta1, double beta2, double eps, int64_t step) {
    SparseConsts c;
    const double bc1 = 1.0 - std::pow(beta1, (double)step);
    const double bc2 = 1.0 - std::pow(beta2, (double)step);
    c.w1 = (float)(1.0 - beta1);
    c.w2 = (float)(1.0 - beta2);
    c.eps = (float)eps;
    c.neg_step = (float)(-(lr * std::sqrt(bc2) / bc1));
    return c;
}

size_t coalesce_scratch_ints(int64_t key_range) { return (size_t)3 * (size_t)(key_range > 0 ? key_range : 1); }

void coalesce_bind_scratch(CoalesceWs& ws, int32_t* scratch, int64_t key_range) {
    const int64_t r = key_range > 0 ? key_range : 1;
    ws.cnt = scratch;
    ws.first = scratch ? scratch + r : nullptr;
    ws.fill = scratch ? scratch + 2 * r : nullptr;
    ws.key_range = key_range;
}

int launch_coalesce_count(const int64_t* idx, int64_t n, int64_t table_rows, CoalesceWs& ws, hipStream_t s) {
    TTAMM_REQUIRE(table_rows < (int64_t(1) << 31) && n < (int64_t(1) << 31) - 1, "coalesce: table or batch too large");
    TTAMM_REQUIRE(ws.key_range >= table_rows && ws.cnt && ws.first && ws.fill, "coalesce: per-row scratch missing");
    TTAMM_REQUIRE(!ws.sorted || table_rows <= 65536, "coalesce: sorted grouping needs <= 65536 keys");
    if (n <= 0) return TTAMM_OK;
    hipLaunchKernelGGL(co_count_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, idx, n, ws.cnt, ws.first);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

int launch_coalesce_group(const int64_t* idx, int64_t n, int64_t table_rows, CoalesceWs& ws, hipStream_t s) {
    if (n <= 0) {
        TTAMM_HIP(hipMemsetAsync(ws.n_unique, 0, sizeof(int32_t), s));
        return TTAMM_OK;
    }
    const unsigned g = (unsigned)ceil_div(n, 256);
    // segment scan over positions (first-occurrence order) or over the key range (sorted)
    const int64_t entries = ws.sorted ? table_rows : n;
    const int64_t tiles = ceil_div(entries, 256);
    TTAMM_REQUIRE(tiles <= std::max<int64_t>(n, 257), "coalesce: tile scratch too small");
    hipLaunchKernelGGL(co_tile_sum_kernel, dim3((unsigned)tiles), dim3(256), 0, s, entries, ws.sorted, idx, ws.cnt,
                       ws.first, ws.lead_cnt, ws.seglong);
    TTAMM_LAUNCH_CHECK();
    hipLaunchKernelGGL(co_tile_scan_kernel, dim3(1), dim3(1024), 0, s, tiles, ws.lead_cnt, ws.seglong, ws.seg_start,
                       ws.n_unique);
    TTAMM_LAUNCH_CHECK();
    hipLaunchKernelGGL(co_tile_write_kernel, dim3((unsigned)tiles), dim3(256), 0, s, entries, ws.sorted, idx, ws.cnt,
                       ws.first, ws.lead_cnt, ws.seglong, ws.lead, ws.seg_start);
    TTAMM_LAUNCH_CHECK();
    hipLaunchKernelGGL(co_fill_kernel, dim3(g), dim3(256), 0, s, idx, n, ws.sorted, ws.lead, ws.first, ws.fill,
                       ws.seg_start, ws.vals_tmp, ws.keys_out, ws.lead_cnt);
    TTAMM_LAUNCH_CHECK();
    // segments longer than kOrderSmall: their ids in `lead` (free again), their count in
    // lead_cnt[0] (zeroed by co_fill)
    hipLaunchKernelGGL(co_order_small_kernel, dim3(g), dim3(256), 0, s, ws, ws.lead, ws.lead_cnt);
    TTAMM_LAUNCH_CHECK();
    hipLaunchKernelGGL(co_order_big_kernel, dim3(256), dim3(256), 0, s, ws, ws.lead, ws.lead_cnt);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

int launch_coalesce(const int64_t* idx, int64_t n, int64_t table_rows, CoalesceWs& ws, hipStream_t s) {
    int rc;
    if ((rc = launch_coalesce_count(idx, n, table_rows, ws, s))) return rc;
    return launch_coalesce_group(idx, n, table_rows, ws, s);
}

namespace {
constexpr int kScanThreads = 1024;
__global__ __launch_bounds__(kScanThreads) void block_exclusive_scan_kernel(const int32_t* __restrict__ in,
                                                                            int32_t* __restrict__ out, int64_t n) {
    __shared__ int32_t sc[kScanThreads];
    const int t = threadIdx.x;
    const int64_t chunk = (n + kScanThreads - 1) / kScanThreads;
    const int64_t lo = min(n, t * chunk), hi = min(n, lo + chunk);
    int32_t sum = 0;
    for (int64_t i = lo; i < hi; ++i) sum += in[i];
    sc[t] = sum;
    __syncthreads();
    for (int o = 1; o < kScanThreads; o <<= 1) {
        const int32_t a = t >= o ? sc[t - o] : 0;
        __syncthreads();
        sc[t] += a;
        __syncthreads();
    }
    int32_t run = sc[t] - sum;
    for (int64_t i = lo; i < hi; ++i) {
        const int32_t v = in[i];
        out[i] = run;
        run += v;
    }
}
}  // namespace

int launch_block_exclusive_scan(const int32_t* in, int32_t* out, int64_t n, hipStream_t s) {
    if (n <= 0) return TTAMM_OK;
    hipLaunchKernelGGL(block_exclusive_scan_kernel, dim3(1), dim3(kScanThreads), 0, s, in, out, n);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

int launch_row_update(const RowUpdateArgs& args, hipStream_t s) {
    if (args.n <= 0) return TTAMM_OK;
    RowUpdateArgs a = args;
    TTAMM_REQUIRE(a.dim % 4 == 0 && (!a.id.weight || a.ld_dE % 4 == 0) && (!a.mimic.weight || a.ld_dA % 4 == 0),
                  "row update: dim and gradient leading dims must be multiples of 4");
    // NV float4 columns per lane when dim / (4 NV) is a power of two <= 64 (row_update_kernel<NV>):
    // measured slower in the C2 step (the item launch 70 -> 91 us: eight rows per wave run the wave's
    // longest Zipf segment, and 183 registers halve the waves per SIMD), so developer-only
    // (TTAMM_ROW_UPDATE_NV=1); the default is one float4 per lane (NV = 0)
    static const bool nv_env = [] { const char* e = dev_env("TTAMM_ROW_UPDATE_NV"); return e && e[0] == '1'; }();
    int nv = 0;
    for (int c = 4; c >= 1 && nv == 0 && nv_env; --c) {
        const int q = a.dim / 4;
        if (q % c == 0 && (q / c & (q / c - 1)) == 0 && q / c <= 64) nv = c;
    }
    if (nv) {
        a.lanes_per_row = a.dim / (4 * nv);
    } else {
        a.lanes_per_row = 1;
        while (a.lanes_per_row < a.dim / 4 && a.lanes_per_row < 64) a.lanes_per_row *= 2;
    }
    // per-column dA rows unless the unit maps are on (their dependent load): the LDS-resolved form
    // cost the one-process C2 step 7 us (0.6616 vs 0.6545 ms, profiles/r05_s42_piece_sum.txt)
    static const bool sda_env = [] { const char* e = dev_env("TTAMM_PIECE_SDA"); return e && e[0] == '1'; }();
    // (the buffer-load form takes 32-bit byte offsets of the gradient rows: positions index them)
    const bool small = 4 * a.n * std::max<int64_t>(a.ld_dE, a.ld_dA) < (int64_t(1) << 31);
    const bool sda = sda_env || a.xu != nullptr || !small;
    if (sda) hipLaunchKernelGGL(piece_sum_kernel<true>, dim3((unsigned)ceil_div(ceil_div(a.n, kPiece), kRowWaves)),
                       dim3(64 * kRowWaves), 0, s, a);
    else hipLaunchKernelGGL(piece_sum_kernel<false>, dim3((unsigned)ceil_div(ceil_div(a.n, kPiece), kRowWaves)),
                       dim3(64 * kRowWaves), 0, s, a);
    TTAMM_LAUNCH_CHECK();
    const int64_t rows_per_block = (int64_t)kRowWaves * (64 / a.lanes_per_row);
    const dim3 grid((unsigned)ceil_div(a.n, rows_per_block));
    switch (nv) {
        case 4: hipLaunchKernelGGL(row_update_kernel<4>, grid, dim3(64 * kRowWaves), 0, s, a); break;
        case 3: hipLaunchKernelGGL(row_update_kernel<3>, grid, dim3(64 * kRowWaves), 0, s, a); break;
        case 2: hipLaunchKernelGGL(row_update_kernel<2>, grid, dim3(64 * kRowWaves), 0, s, a); break;
        case 1: hipLaunchKernelGGL(row_update_kernel<1>, grid, dim3(64 * kRowWaves), 0, s, a); break;
        default: hipLaunchKernelGGL(row_update_kernel<0>, grid, dim3(64 * kRowWaves), 0, s, a); break;
    }
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

int launch_dense_sweep(const SweepArgs& a, hipStream_t s) {
    int64_t total4 = 0;
    for (int i = 0; i < a.count; ++i) {
        TTAMM_REQUIRE(((uintptr_t)a.seg[i].p | (uintptr_t)a.seg[i].m | (uintptr_t)a.seg[i].v) % 16 == 0,
                      "dense sweep: tables must be 16-byte aligned");
        total4 += a.seg[i].n >> 2;
    }
    if (a.count == 0) return TTAMM_OK;
    // 2048 blocks x 256 threads: 8 blocks per CU, grid-stride over the tables
    hipLaunchKernelGGL(dense_sweep_kernel, dim3(grid_for(total4, 256, 2048)), dim3(256), 0, s, a);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

int launch_step_begin(const uint32_t* status, int64_t* applied, AdamConsts* hist, int cap, int64_t step,
                      const AdamConsts& c, hipStream_t s) {
    TTAMM_REQUIRE(!hist || (cap > 1 && cap <= kMaxHistory), "adam history: capacity must be in [2, 512]");
    if (!hist && !applied) return TTAMM_OK;
    hipLaunchKernelGGL(step_begin_kernel, dim3(1), dim3(64), 0, s, status, applied, hist, hist ? cap : 2, step, c);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

template <int V>
static void launch_replay_v(const ReplayArgs& a, dim3 grid, size_t lds, hipStream_t s) {
    // TTAMM_REPLAY_SCALAR=1: constants in scalar registers (replay_s_kernel); default: the
    // history ring staged in LDS per block (replay_kernel)
    static const bool scalar = [] {
        const char* e = dev_env("TTAMM_REPLAY_SCALAR");
        return e && e[0] == '1';
    }();
    if (a.sgd) {
        hipLaunchKernelGGL((replay_sgd_kernel<V>), grid, dim3(256), 0, s, a);
        return;
    }
    if (scalar) {
        if (a.fast_g0) {
            if (a.decoupled) hipLaunchKernelGGL((replay_s_kernel<true, true, V>), grid, dim3(256), 0, s, a);
            else hipLaunchKernelGGL((replay_s_kernel<false, true, V>), grid, dim3(256), 0, s, a);
        } else if (a.decoupled) {
            hipLaunchKernelGGL((replay_s_kernel<true, false, V>), grid, dim3(256), 0, s, a);
        } else {
            hipLaunchKernelGGL((replay_s_kernel<false, false, V>), grid, dim3(256), 0, s, a);
        }
        return;
    }
    if (a.fast_g0) {
        if (a.decoupled) hipLaunchKernelGGL((replay_kernel<true, true, V>), grid, dim3(256), lds, s, a);
        else hipLaunchKernelGGL((replay_kernel<false, true, V>), grid, dim3(256), lds, s, a);
    } else if (a.decoupled) {
        hipLaunchKernelGGL((replay_kernel<true, false, V>), grid, dim3(256), lds, s, a);
    } else {
        hipLaunchKernelGGL((replay_kernel<false, false, V>), grid, dim3(256), lds, s, a);
    }
}

int launch_replay(const ReplayArgs& a, hipStream_t s, void* const* ev) {
    if (a.count == 0) return TTAMM_OK;
    TTAMM_REQUIRE(a.count <= kMaxReplaySegs && a.hist && a.cap > 1 && a.cap <= kMaxHistory,
                  "replay: bad arguments");
    int64_t most = 0;
    bool v2 = true;  // two float4s per thread when every segment's dim is a multiple of 8
    for (int i = 0; i < a.count; ++i) v2 = v2 && a.seg[i].dim % 8 == 0;
    const int V = v2 ? 2 : 1;
    for (int i = 0; i < a.count; ++i) {
        const ReplaySeg& g = a.seg[i];
        TTAMM_REQUIRE(g.p && g.m && g.v && (g.last || g.list_rows), "replay: table without deferred state");
        TTAMM_REQUIRE(!g.list_rows || (g.list_lag && g.list_cnt), "replay: catch-up list incomplete");
        TTAMM_REQUIRE(g.dim % 4 == 0 && ((uintptr_t)g.p | (uintptr_t)g.m | (uintptr_t)g.v) % 16 == 0,
                      "replay: tables must be 16-byte aligned with dim % 4 == 0");
        const int64_t n = g.row_hi - g.row_lo;  // lists: the batch positions bound the listed rows
        TTAMM_REQUIRE(n >= 0 && n * (g.dim / 4) < (int64_t(1) << 31), "replay: more than 2^31 float4s in a segment");
        most = n * (g.dim / 4 / V) > most ? n * (g.dim / 4 / V) : most;
    }
    if (most == 0) return TTAMM_OK;
    const dim3 grid(grid_for(most, 256, 16384), a.count);
    const size_t lds = (size_t)2 * a.cap * sizeof(ReplayConsts);
    if (ev && ev[0]) TTAMM_HIP(hipEventRecord((hipEvent_t)ev[0], s));
    if (v2) launch_replay_v<2>(a, grid, lds, s);
    else launch_replay_v<1>(a, grid, lds, s);
    TTAMM_LAUNCH_CHECK();
    if (ev && ev[1]) TTAMM_HIP(hipEventRecord((hipEvent_t)ev[1], s));
    if (a.stamp) {
        int64_t rows = 0;
        for (int i = 0; i < a.count; ++i) rows = a.seg[i].row_hi - a.seg[i].row_lo > rows ? a.seg[i].row_hi - a.seg[i].row_lo : rows;
        hipLaunchKernelGGL(stamp_kernel, dim3(grid_for(rows, 256, 4096), a.count), dim3(256), 0, s, a);
        TTAMM_LAUNCH_CHECK();
    }
    return TTAMM_OK;
}

size_t catchup_list_ints(int64_t n, int cap) { return (size_t)2 * (cap + 1) + (size_t)2 * (n > 0 ? n : 1) + 64; }

void catchup_bind(CatchupList& cl, int32_t* ints, int64_t n, int cap) {
    cl.cnt = ints;
    cl.fill = ints ? ints + (cap + 1) : nullptr;
    cl.rows = ints ? ints + 2 * (cap + 1) + 64 : nullptr;  // 256-B aligned past the counters
    cl.lag = ints ? cl.rows + (n > 0 ? n : 1) : nullptr;
}

int launch_catchup_list(const int64_t* idx, int64_t n, const int32_t* first, int32_t* const* last, int nlast,
                        int32_t target, int cap, const CatchupList& cl, const uint32_t* status, hipStream_t s) {
    TTAMM_REQUIRE(cl.cnt && cl.fill && cl.rows && cl.lag && first && last && last[0] && nlast >= 1 && nlast <= 2,
                  "catch-up list: bad arguments");
    TTAMM_REQUIRE(cap > 1 && cap <= kMaxHistory && n < (int64_t(1) << 31) - 1, "catch-up list: bad sizes");
    TTAMM_HIP(hipMemsetAsync(cl.cnt, 0, sizeof(int32_t) * 2 * (cap + 1), s));  // cnt and fill
    if (n <= 0) return TTAMM_OK;
    const unsigned g = (unsigned)ceil_div(n, 256);
    hipLaunchKernelGGL(catchup_count_kernel, dim3(g), dim3(256), 0, s, idx, n, first, last[0], target, cap, cl.cnt,
                       status);
    TTAMM_LAUNCH_CHECK();
    LastPtrs lp{{last[0], nlast > 1 ? last[1] : nullptr}};
    hipLaunchKernelGGL(catchup_scatter_kernel, dim3(g), dim3(256), 0, s, idx, n, first, lp, nlast, target, cap, cl.cnt,
                       cl.fill, cl.rows, cl.lag, status);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

int launch_prepare_segs(const PrepSegs& a, hipStream_t s) {
    TTAMM_REQUIRE(a.count >= 1 && a.count <= 2, "prepare: one or two towers");
    int64_t most = 0;
    bool lists = false;
    for (int i = 0; i < a.count; ++i) {
        const PrepSeg& g = a.seg[i];
        TTAMM_REQUIRE(g.idx && g.cnt && g.first && g.n >= 0 && g.n < (int64_t(1) << 31) - 1, "prepare: bad tower");
        TTAMM_REQUIRE(!g.list_cnt || (g.list_rows && g.list_lag && g.last[0] && g.nlast >= 1 && g.nlast <= 2 &&
                                      a.cap > 1 && a.cap <= kMaxHistory),
                      "prepare: catch-up list incomplete");
        most = g.n > most ? g.n : most;
        lists = lists || g.list_cnt;
    }
    const unsigned g = (unsigned)std::max<int64_t>(1, ceil_div(most, 256));
    hipLaunchKernelGGL(co_count_seg_kernel, dim3(g, a.count), dim3(256), 0, s, a);
    TTAMM_LAUNCH_CHECK();
    if (!lists || most == 0) return TTAMM_OK;
    hipLaunchKernelGGL(catchup_count_seg_kernel, dim3(g, a.count), dim3(256), 0, s, a);
    TTAMM_LAUNCH_CHECK();
    hipLaunchKernelGGL(catchup_scatter_seg_kernel, dim3(g, a.count), dim3(256), 0, s, a);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

int launch_side_scatter(const int32_t* n_unique, const int32_t* keys, const int32_t* seg_start, const float* side,
                        int64_t n, int dim, ttamm_table t, const uint32_t* status, hipStream_t s) {
    if (n <= 0) return TTAMM_OK;
    hipLaunchKernelGGL(side_scatter_kernel, dim3(grid_for(n * dim)), dim3(256), 0, s, n_unique, keys, seg_start, side,
                       n, dim, t, status);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

int rows_sumsq_blocks(int64_t n, int dim) { return (int)std::max<int64_t>(1, ceil_div(n * (dim / 4), 256)); }

int launch_rows_sumsq(const RowUpdateArgs& a, float* partials, hipStream_t s) {
    if (a.n <= 0) return TTAMM_OK;
    TTAMM_REQUIRE(a.dim % 4 == 0, "clip: dim must be a multiple of 4");
    hipLaunchKernelGGL(rows_sumsq_kernel, dim3((unsigned)rows_sumsq_blocks(a.n, a.dim)), dim3(256), 0, s, a, partials);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

int launch_dense_sumsq(const DenseAdamArgs& a, float* partials, hipStream_t s) {
    int64_t total = 0;
    for (int i = 0; i < a.count; ++i) total += a.t[i].n;
    if (total == 0) {
        TTAMM_HIP(hipMemsetAsync(partials, 0, kDenseSumsqBlocks * sizeof(float), s));
        return TTAMM_OK;
    }
    hipLaunchKernelGGL(dense_sumsq_kernel, dim3(kDenseSumsqBlocks), dim3(256), 0, s, a, total, partials);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

int launch_clip_coef(const float* partials, int n, float max_norm, float* coef, hipStream_t s) {
    hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(256), 0, s, partials, n, max_norm, coef);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

int launch_sum_partials(const float* partials, int n, float* out, hipStream_t s) {
    hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, s, partials, n, out);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

int launch_dense_adam(const DenseAdamArgs& a, hipStream_t s) {
    int64_t total = 0;
    for (int i = 0; i < a.count; ++i) total += a.t[i].n;
    if (total == 0) return TTAMM_OK;
    hipLaunchKernelGGL(dense_adam_kernel, dim3(grid_for(total, 256, 4096)), dim3(256), 0, s, a, total);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

int launch_sparse_adam_rows(float* w, float* m, float* v, int dim, const int64_t* rows, const float* grad, int64_t n,
                            SparseConsts c, hipStream_t s) {
    if (n <= 0) return TTAMM_OK;
    hipLaunchKernelGGL(sparse_adam_rows_kernel, dim3(grid_for(n * dim)), dim3(256), 0, s, w, m, v, dim, rows, grad,
                       n, c);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

}  // namespace ttamm
