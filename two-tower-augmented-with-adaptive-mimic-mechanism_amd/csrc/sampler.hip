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

__global__ void sample_negatives_kernel(const int64_t* __restrict__ users, int64_t batch, int num_neg,
                                        uint64_t num_items, const int64_t* __restrict__ pos_offsets,
                                        const int64_t* __restrict__ pos_values, uint32_t k0, uint32_t k1,
                                        uint64_t counter, int64_t slot_base, int64_t* __restrict__ out,
                                        int64_t* __restrict__ out2, uint32_t* __restrict__ status) {
    const int64_t slot = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (slot >= batch * num_neg) return;
    const int64_t b = slot / num_neg;
    const int64_t u = users[b];
    int64_t lo = 0, hi = 0;
    if (pos_offsets) {
        lo = pos_offsets[u];
        hi = pos_offsets[u + 1];
    }
    int64_t cand = 0;
    bool ok = false;
    const int64_t key = slot_base + slot;  // global slot: a sharded batch draws what one process would
    for (int attempt = 0; attempt < kMaxDraws && !ok; ++attempt) {
        const u32x4 r = philox4x32(
            u32x4{(uint32_t)key, (uint32_t)(key >> 32), (uint32_t)counter,
                  RNG_NEGATIVES | ((uint32_t)attempt << 20) | ((uint32_t)(counter >> 32) & 0xFFFFFu)},
            k0, k1);
        const uint64_t r64 = ((uint64_t)r.x << 32) | r.y;
        cand = (int64_t)__umul64hi(r64, num_items);  // uniform in [0, num_items), bias < 2^-40
        ok = (hi == lo) || !is_positive(pos_values, lo, hi, cand);
    }
    out[slot] = cand;
    if (out2) out2[slot] = cand;
    if (!ok) atomicOr(status, TTAMM_STATUS_SAMPLER_EXHAUSTED);
}

}  // namespace

int launch_sample_negatives(const int64_t* users, int64_t batch, int num_neg, int64_t num_items,
                            const int64_t* pos_offsets, const int64_t* pos_values, uint64_t seed, uint64_t counter,
                            int64_t slot_base, int64_t* out, int64_t* out2, uint32_t* status, hipStream_t s) {
    TTAMM_REQUIRE(num_neg > 0, "num_negatives must be greater than zero.");
    TTAMM_REQUIRE(num_items > 1, "num_items must be greater than one.");
    const int64_t slots = batch * num_neg;
    if (slots <= 0) return TTAMM_OK;
    hipLaunchKernelGGL(sample_negatives_kernel, dim3((unsigned)ceil_div(slots, 256)), dim3(256), 0, s, users, batch,
                       num_neg, (uint64_t)num_items, pos_offsets, pos_values, (uint32_t)seed, (uint32_t)(seed >> 32),
                       counter, slot_base, out, out2, status);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

}  // namespace ttamm
