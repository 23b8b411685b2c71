// On-device negative sampler: sample_negative_items (samplers.py:11-85).
//
// Reference semantics per slot (b, j): draw uniformly from [0, num_items); if the draw is
// one of user b's known positives, redraw.  The reference redraws invalid slots in rounds
// and raises once an 11th redraw round has been needed (samplers.py:66-81), so a slot gets at
// most 11 draws (initial + 10 redraws) before the batch fails.  Here every slot is one thread
// that walks its own counter-based Philox stream; a slot that exhausts its 11 draws sets
// TTAMM_STATUS_SAMPLER_EXHAUSTED, which the host raises as RuntimeError.
// Positives are a CSR (per-user sorted item ids), searched by binary search instead of
// torch.isin on a per-user tensor (samplers.py:44-65).
#include "kernels.h"

namespace ttamm {

namespace {

constexpr int kMaxDraws = 11;

__device__ __forceinline__ bool is_positive(const int64_t* __restrict__ vals, int64_t lo, int64_t hi, int64_t x) {
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        const int64_t v = vals[mid];
        if (v == x) return true;
        if (v < x) lo = mid + 1;
        else hi = mid;
    }
    return false;
}

// slot `slot` of the batch's negatives for user row u (a staged, in-range id)
__device__ __forceinline__ void sample_slot(int64_t slot, int64_t u, uint64_t num_items,
                                            const int64_t* __restrict__ pos_offsets,
                                            const int64_t* __restrict__ pos_values, uint32_t k0, uint32_t k1,
                                            uint64_t counter, int64_t slot_base, int64_t* __restrict__ out,
                                            int64_t* __restrict__ out2, uint32_t* __restrict__ status) {
    int64_t lo = 0, hi = 0;
    if (pos_offsets) {
        lo = pos_offsets[u];
        hi = pos_offsets[u + 1];
    }
    int64_t cand = 0;
    bool ok = false;
    const int64_t key = slot_base + slot;  // global slot: a sharded batch draws what one process would
    // a short positive list (the common case: ~20 per user) is loaded whole with independent loads
    // and scanned in registers — one memory round trip instead of a binary search's log2(n)
    // dependent ones on the step's critical path; longer lists keep the binary search
    constexpr int kShort = 32;
    const int64_t n = hi - lo;
    int64_t pv[kShort];
    if (n <= kShort) {
#pragma unroll
        for (int i = 0; i < kShort; ++i) pv[i] = i < n ? pos_values[lo + i] : -1;
    }
    for (int attempt = 0; attempt < kMaxDraws && !ok; ++attempt) {
        const u32x4 r = philox4x32(
            u32x4{(uint32_t)key, (uint32_t)(key >> 32), (uint32_t)counter,
                  RNG_NEGATIVES | ((uint32_t)attempt << 20) | ((uint32_t)(counter >> 32) & 0xFFFFFu)},
            k0, k1);
        const uint64_t r64 = ((uint64_t)r.x << 32) | r.y;
        cand = (int64_t)__umul64hi(r64, num_items);  // uniform in [0, num_items), bias < 2^-40
        if (n <= kShort) {
            bool hit = false;
#pragma unroll
            for (int i = 0; i < kShort; ++i) hit |= pv[i] == cand;  // (-1 never equals a draw)
            ok = !hit;
        } else {
            ok = !is_positive(pos_values, lo, hi, cand);
        }
    }
    out[slot] = cand;
    if (out2) out2[slot] = cand;
    if (!ok) atomicOr(status, TTAMM_STATUS_SAMPLER_EXHAUSTED);
}

__global__ void sample_negatives_kernel(const int64_t* __restrict__ users, int64_t batch, int num_neg,
                                        uint64_t num_items, const int64_t* __restrict__ pos_offsets,
                                        const int64_t* __restrict__ pos_values, int64_t user_rows, uint32_t k0,
                                        uint32_t k1, uint64_t counter, int64_t slot_base, int64_t* __restrict__ out,
                                        int64_t* __restrict__ out2, uint32_t* __restrict__ status) {
    const int64_t slot = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (slot >= batch * num_neg) return;
    const int64_t u = users[slot / num_neg];
    // a user outside the CSR has no positives (the reference's positives.get(user, set()))
    const bool known = u >= 0 && u < user_rows;
    sample_slot(slot, known ? u : 0, num_items, known ? pos_offsets : nullptr, pos_values, k0, k1, counter, slot_base,
                out, out2, status);
}

// The step's prologue in one launch (blockIdx.y < st.count: staging segment y, as
// stage_rows_kernel; y == st.count: the sampler, reading user b's id from the raw batch with the
// staging's range check, so it needs no staged copy; both grid-stride), and the last block to
// finish runs
// step_begin_kernel's work with every block's status bits visible (a completion counter in the
// zero-initialised workspace, reset by that block).
struct StepPrologue {
    StageArgs st;
    PrologueArgs pa;
};
__global__ void step_prologue_kernel(StepPrologue) {
    const KArg(StepPrologue)* kp = (const KArg(StepPrologue)*)(__builtin_amdgcn_kernarg_segment_ptr());
    const KArg(StageArgs)* st = &kp->st;
    const KArg(PrologueArgs)* pa = &kp->pa;
    const int y = blockIdx.y;
    if (y < st->count) {
        const KArg(StageSeg)& S = st->seg[y];
        bool bad = false;
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < S.n; i += (int64_t)gridDim.x * blockDim.x) {
            const int64_t v = S.in[i * (S.ld ? S.ld : 1)];
            const bool ok = v >= 0 && v < S.rows;
            bad |= !ok;
            if (S.out) S.out[i] = ok ? v : 0;
        }
        if (st->status && __ballot(bad) != 0ull && (threadIdx.x & 63) == 0)
            atomicOr(st->status, TTAMM_STATUS_INDEX_OUT_OF_RANGE);
    } else if (y >= st->count + (pa->num_neg > 0 ? 1 : 0)) {
        // weight prep segment: the first feature layer's weight padded / rounded to bf16
        const KArg(WeightPrep)& W = pa->prep[y - st->count - (pa->num_neg > 0 ? 1 : 0)];
        const int64_t total = W.rows * W.ld_dst;
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
            const int64_t r = i / W.ld_dst;
            const int c = (int)(i - r * W.ld_dst);
            const float v = c < W.cols ? W.src[r * W.ld_src + c] : 0.f;
            if (W.bf16) static_cast<uint16_t*>(W.dst)[i] = __builtin_bit_cast(uint16_t, (__bf16)v);  // RNE
            else static_cast<float*>(W.dst)[i] = v;
        }
    } else {
        const int64_t slots = pa->batch * pa->num_neg;
        for (int64_t slot = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; slot < slots;
             slot += (int64_t)gridDim.x * blockDim.x) {
            const int64_t v = pa->users[slot / pa->num_neg];
            const int64_t u = (v >= 0 && v < pa->user_rows) ? v : 0;
            sample_slot(slot, u, pa->num_items, pa->pos_offsets, pa->pos_values, pa->k0, pa->k1, pa->counter,
                        pa->slot_base, pa->out, pa->out2, st->status);
        }
    }
    // completion: the last block counts the step and publishes its AdamW constants (done == null: the
    // caller runs step_begin_kernel on its aux stream instead, off the critical path)
    if (!pa->done) return;
    __syncthreads();
    if (threadIdx.x != 0) return;
    __threadfence();
    const uint32_t blocks = gridDim.x * gridDim.y;
    if (atomicAdd(pa->done, 1u) != blocks - 1) return;
    __threadfence();
    *pa->done = 0u;
    const uint32_t status = st->status ? atomicOr(st->status, 0u) : 0u;
    if (status & kStatusPoison) return;
    if (pa->applied) pa->applied[0] += 1;
    if (pa->hist) {
        AdamConsts c;
        c.decay = pa->c.decay, c.w1 = pa->c.w1, c.b2 = pa->c.b2, c.w2 = pa->c.w2, c.eps = pa->c.eps;
        c.neg_step = pa->c.neg_step, c.bc2_sqrt = pa->c.bc2_sqrt, c.inv_bc2_sqrt = pa->c.inv_bc2_sqrt;
        c.wd = pa->c.wd, c.decoupled = pa->c.decoupled, c.fast_g0 = pa->c.fast_g0;
        c.fast_ibc = pa->c.fast_ibc, c.fast_eps = pa->c.fast_eps;
        c.sgd = pa->c.sgd, c.sgd_neg_lr = pa->c.sgd_neg_lr, c.sgd_mom = pa->c.sgd_mom;  // deferred SGD replay
        c.sgd_damp1 = pa->c.sgd_damp1, c.sgd_first = pa->c.sgd_first, c.sgd_nesterov = pa->c.sgd_nesterov;
        pa->hist[pa->step % pa->cap] = c;
    }
}

}  // namespace

int launch_step_prologue(const StageArgs& st, const PrologueArgs& pa, hipStream_t s) {
    TTAMM_REQUIRE(st.count >= 0 && st.count <= kMaxStageSegs && (pa.done || (!pa.applied && !pa.hist)),
                  "step prologue: bad arguments");
    TTAMM_REQUIRE(pa.num_neg == 0 || (pa.num_items > 1 && pa.users), "step prologue: sampler arguments");
    TTAMM_REQUIRE(!pa.hist || (pa.cap > 1 && pa.cap <= kMaxAdamHistory), "adam history: capacity must be in [2, 512]");
    int64_t most = pa.batch * pa.num_neg;
    for (int i = 0; i < st.count; ++i) most = st.seg[i].n > most ? st.seg[i].n : most;
    // both parts grid-stride: 64 blocks per part keep the closing counter's atomics few (one per
    // block) while a C2 batch is still ~2.5 staging elements or sampler slots per thread
    int64_t gx = ceil_div(most, 256);
    if (gx > 64) gx = 64;
    if (gx < 1) gx = 1;
    TTAMM_REQUIRE(pa.n_prep >= 0 && pa.n_prep <= kMaxWeightPrep, "step prologue: weight prep segments");
    for (int i = 0; i < pa.n_prep; ++i) {
        const WeightPrep& w = pa.prep[i];
        TTAMM_REQUIRE(w.src && w.dst && w.rows > 0 && w.cols > 0 && w.ld_dst >= w.cols && w.ld_src >= w.cols,
                      "step prologue: bad weight prep segment");
        most = w.rows * w.ld_dst > most ? w.rows * w.ld_dst : most;
    }
    const unsigned gy = (unsigned)st.count + (pa.num_neg > 0 ? 1u : 0u) + (unsigned)pa.n_prep;
    TTAMM_REQUIRE(gy >= 1 && gx * gy < (int64_t(1) << 31), "step prologue: grid too large");
    hipLaunchKernelGGL(step_prologue_kernel, dim3((unsigned)gx, gy), dim3(256), 0, s, StepPrologue{st, pa});
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

int launch_sample_negatives(const int64_t* users, int64_t batch, int num_neg, int64_t num_items,
                            const int64_t* pos_offsets, const int64_t* pos_values, int64_t user_rows, uint64_t seed,
                            uint64_t counter, int64_t slot_base, int64_t* out, int64_t* out2, uint32_t* status,
                            hipStream_t s) {
    TTAMM_REQUIRE(num_neg > 0, "num_negatives must be greater than zero.");
    TTAMM_REQUIRE(num_items > 1, "num_items must be greater than one.");
    const int64_t slots = batch * num_neg;
    if (slots <= 0) return TTAMM_OK;
    hipLaunchKernelGGL(sample_negatives_kernel, dim3((unsigned)ceil_div(slots, 256)), dim3(256), 0, s, users, batch,
                       num_neg, (uint64_t)num_items, pos_offsets, pos_values, pos_offsets ? user_rows : 0,
                       (uint32_t)seed, (uint32_t)(seed >> 32), counter, slot_base, out, out2, status);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

}  // namespace ttamm
