// On-device epoch order of the interaction pairs: the reference's
//   DataLoader(InteractionDataset(train_df), batch_size, shuffle=True, drop_last=False)
// (datasets.py:12-45, training.py:260-264) with the pairs resident in HBM.
//
// The shuffle is a seeded bijection of [0, n) evaluated per position — no permutation array is
// built or sorted: a 4-round balanced Feistel network on 2h-bit words (2^2h >= n, h >= 1) with
// cycle-walking (positions that map outside [0, n) are mapped again until they land inside; a
// walk stays on the position's own cycle, so it ends, after < 4 rounds on average since
// 2^2h < 4n).  Round keys come from (seed, epoch) on the host (epoch_round_keys), so every
// epoch has its own order and the same (seed, epoch) gives the same order on every device and
// in oracle/data_perm.py, which restates this function for the tests.
#include "kernels.h"

namespace ttamm {

namespace {

__host__ __device__ __forceinline__ uint32_t fmix32(uint32_t x) {  // murmur3 finaliser
    x ^= x >> 16;
    x *= 0x85ebca6bu;
    x ^= x >> 13;
    x *= 0xc2b2ae35u;
    x ^= x >> 16;
    return x;
}

__host__ __device__ __forceinline__ uint64_t feistel(uint64_t x, int h, uint32_t k0, uint32_t k1, uint32_t k2,
                                                     uint32_t k3) {
    const uint64_t mask = h >= 32 ? 0xFFFFFFFFull : ((1ull << h) - 1);
    uint64_t l = x >> h, r = x & mask;
    const uint32_t ks[4] = {k0, k1, k2, k3};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint64_t t = r;
        r = l ^ ((uint64_t)fmix32((uint32_t)r ^ ks[q]) & mask);
        l = t;
    }
    return (l << h) | r;
}

__global__ void epoch_batch_kernel(const int64_t* __restrict__ users, const int64_t* __restrict__ items, int64_t n,
                                   int h, uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3, int shuffle,
                                   int64_t start, int64_t count, int64_t* __restrict__ out_users,
                                   int64_t* __restrict__ out_items) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < count; j += (int64_t)gridDim.x * blockDim.x) {
        uint64_t src = (uint64_t)(start + j);
        if (shuffle) {
            src = feistel(src, h, k0, k1, k2, k3);
            while (src >= (uint64_t)n) src = feistel(src, h, k0, k1, k2, k3);
        }
        out_users[j] = users[src];
        out_items[j] = items[src];
    }
}

uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

}  // namespace

// half width h: the smallest h >= 1 with 4^h >= n
int epoch_half_bits(int64_t n) {
    int h = 1;
    while (h < 32 && (uint64_t)n > (1ull << (2 * h))) ++h;
    return h;
}

void epoch_round_keys(uint64_t seed, int64_t epoch, uint32_t keys[4]) {
    for (int q = 0; q < 4; ++q) keys[q] = (uint32_t)splitmix64(seed ^ splitmix64((uint64_t)epoch * 4u + (uint64_t)q));
}

int launch_epoch_batch(const int64_t* users, const int64_t* items, int64_t n, uint64_t seed, int64_t epoch,
                       int shuffle, int64_t start, int64_t count, int64_t* out_users, int64_t* out_items,
                       hipStream_t s) {
    TTAMM_REQUIRE(n >= 0 && start >= 0 && count >= 0 && start + count <= n, "epoch batch: positions outside [0, n)");
    TTAMM_REQUIRE(count == 0 || (users && items && out_users && out_items), "epoch batch: null pointer");
    if (count == 0) return TTAMM_OK;
    uint32_t k[4];
    epoch_round_keys(seed, epoch, k);
    const int h = epoch_half_bits(n);
    int64_t blocks = ceil_div(count, 256);
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(epoch_batch_kernel, dim3((unsigned)blocks), dim3(256), 0, s, users, items, n, h, k[0], k[1],
                       k[2], k[3], shuffle, start, count, out_users, out_items);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

}  // namespace ttamm
