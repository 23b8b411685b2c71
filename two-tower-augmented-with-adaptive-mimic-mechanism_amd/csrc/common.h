// Shared device/host helpers for libttamm (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>
#include <string>

#include "../../include/ttamm.h"

// A kernel argument viewed in place in the kernarg segment (address space 4): indexing an
// array member of a by-value kernel argument with a runtime index would otherwise copy the
// whole argument to scratch.  Use with __builtin_amdgcn_kernarg_segment_ptr().
#define KArg(T) __attribute__((address_space(4))) T

namespace ttamm {

// ---- error plumbing ---------------------------------------------------------------
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);

#define TTAMM_HIP(expr)                                                                    \
    do {                                                                                   \
        hipError_t _e = (expr);                                                            \
        if (_e != hipSuccess)                                                              \
            return ::ttamm::fail(TTAMM_E_HIP, std::string(#expr " failed: ") +             \
                                                  hipGetErrorString(_e));                  \
    } while (0)

#define TTAMM_LAUNCH_CHECK()                                                               \
    do {                                                                                   \
        hipError_t _e = hipGetLastError();                                                 \
        if (_e != hipSuccess)                                                              \
            return ::ttamm::fail(TTAMM_E_HIP, std::string("kernel launch failed: ") +      \
                                                  hipGetErrorString(_e) + " at " + __FILE__); \
    } while (0)

#define TTAMM_REQUIRE(cond, msg)                                                           \
    do {                                                                                   \
        if (!(cond)) return ::ttamm::fail(TTAMM_E_INVALID, (msg));                         \
    } while (0)

static inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
static inline size_t align_up(size_t a, size_t b) { return (a + b - 1) / b * b; }

// ---- environment switches -----------------------------------------------------------------
// product_env: the documented knobs (INTEGRATION.md "Environment"): TTAMM_FP32_MFMA,
// TTAMM_RETRIEVAL_FP32, TTAMM_GENERIC_GATE.  dev_env: A/B variants, ablations and measured-slower
// opt-ins, honoured only by a developer build (make DEV=1 defines TTAMM_DEV_KNOBS); the default
// library never reads them, so a stray variable cannot change what it computes.
static inline const char* product_env(const char* name) { return std::getenv(name); }
#ifdef TTAMM_DEV_KNOBS
constexpr bool kDevKnobs = true;
static inline const char* dev_env(const char* name) { return std::getenv(name); }
#else
constexpr bool kDevKnobs = false;  // timing ablations inside kernels are compiled out
static inline const char* dev_env(const char*) { return nullptr; }
#endif

// ---- workspace bump allocator (host side) -----------------------------------------------
struct Arena {
    char* base;
    size_t cap;
    size_t off;
    bool measuring;  // when true only sizes are accumulated
    template <typename T>
    T* take(size_t count) {
        off = align_up(off, 256);
        T* p = measuring ? nullptr : reinterpret_cast<T*>(base + off);
        off += count * sizeof(T);
        return p;
    }
    bool ok() const { return measuring || off <= cap; }
};

// ---- device helpers -------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Streaming (non-temporal) 16-byte store, for outputs a LATER kernel reads: the line is not
// kept dirty in this XCD's L2, so the end-of-kernel L2 write-back does not serialise behind
// the launch.  Measured on a 49,152 x 512 B row gather: 22 us with plain stores, 6.8 us with
// these (csrc/tools/gather_bench.cpp, profiles/r01_gather_variants.txt).
typedef float f32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store_nt(float4* p, float4 v) {
    const f32x4_t x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<f32x4_t*>(p));
}
__device__ __forceinline__ void store_nt(float* p, float4 v) { store_nt(reinterpret_cast<float4*>(p), v); }

// x / c correctly rounded (== IEEE x / c, bit for bit) for a per-step constant c > 0 with
// inv_c = RN(1/c), when x is +0 or a normal number and x / c stays normal: two Markstein
// refinements of x * inv_c — the first makes the quotient faithful, so the second residual
// fma(-c, q, x) is exact and q + r * inv_c rounds to the correctly rounded quotient.  Used
// for sqrt(v) / sqrt(bc2): sqrt of any fp32 v >= 0 is 0 or >= 2^-75, bc2_sqrt is in (0, 1].
// 5 VALU ops instead of the ~11 of the general IEEE division sequence.
__device__ __forceinline__ float div_by_const(float x, float c, float inv_c) {
    float q = x * inv_c;
    float r = fmaf(-c, q, x);
    q = fmaf(r, inv_c, q);
    r = fmaf(-c, q, x);
    return fmaf(r, inv_c, q);
}

// Philox4x32-10 counter-based RNG (Salmon et al., SC'11).
struct u32x4 {
    uint32_t x, y, z, w;
};
__device__ __forceinline__ u32x4 philox4x32(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
        const uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
        c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

// RNG stream domains, kept in the high bits of counter word w.
enum : uint32_t {
    RNG_NEGATIVES = 1u << 28,
    RNG_DROPOUT = 2u << 28,
};

}  // namespace ttamm
