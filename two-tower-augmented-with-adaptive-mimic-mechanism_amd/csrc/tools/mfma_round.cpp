// Developer probe: the rounding semantics of v_mfma_f32_32x32x16_bf16 on gfx950, and the bias of
// the split-bf16 fp32 product (six bf16 MFMAs) against an fp32 fma chain, both against fp64.
// Build: hipcc -O3 --offload-arch=gfx950 -x hip tools/mfma_round.cpp -o ../build/mfma_round
//
// Part 1 (one MFMA): D = C + sum_k A[i][k] B[k][j] over k < 16, bf16 A/B.  For every output the
// host forms (a) the exact sum rounded once to fp32 (RNE), (b) a k-ordered fp32 fma chain from C,
// (c) the exact product sum truncated toward zero, and counts which one D equals bit for bit.
// Part 2 (a K = 608 dot product, 38 chained MFMAs from C = 0): the MFMA chain's mean signed error
// and RMS error against fp64, beside a host fp32 fma chain over the same bf16 products, in units
// of 2^-24 * sum |a b| — a systematic (signed) part would bias gradients the same way every step.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

static uint16_t f2bf(float f) {  // RNE
    uint32_t u;
    std::memcpy(&u, &f, 4);
    uint32_t r = u + 0x7fff + ((u >> 16) & 1);
    return (uint16_t)(r >> 16);
}
static float bf2f(uint16_t b) {
    uint32_t u = (uint32_t)b << 16;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

// one 32x32x16 MFMA per block of 64 threads: A [32][16], B [16][32] (bf16 bits), C / D [32][32]
__global__ void one_mfma(const uint16_t* A, const uint16_t* B, const float* C, float* D, int reps) {
    const int lane = threadIdx.x;
    const int t = blockIdx.x;
    A += t * 32 * 16;
    B += t * 16 * 32;
    C += t * 32 * 32;
    D += t * 32 * 32;
    bf16x8 a, b;
    for (int j = 0; j < 8; ++j) {
        const int k = 8 * (lane / 32) + j;
        uint16_t av = A[(lane % 32) * 16 + k], bv = B[k * 32 + (lane % 32)];
        a[j] = __builtin_bit_cast(__bf16, av);
        b[j] = __builtin_bit_cast(__bf16, bv);
    }
    f32x16 acc;
    for (int r = 0; r < 16; ++r) acc[r] = C[(8 * (r / 4) + 4 * (lane / 32) + (r % 4)) * 32 + lane % 32];
    for (int i = 0; i < reps; ++i) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
    for (int r = 0; r < 16; ++r) D[(8 * (r / 4) + 4 * (lane / 32) + (r % 4)) * 32 + lane % 32] = acc[r];
}

// 38 chained MFMAs from C = 0: A [T][32][K], B [T][K][32]
__global__ void chain_mfma(const uint16_t* A, const uint16_t* B, float* D, int K) {
    const int lane = threadIdx.x;
    const int t = blockIdx.x;
    A += (size_t)t * 32 * K;
    B += (size_t)t * K * 32;
    D += t * 32 * 32;
    f32x16 acc;
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    for (int k0 = 0; k0 < K; k0 += 16) {
        bf16x8 a, b;
        for (int j = 0; j < 8; ++j) {
            const int k = k0 + 8 * (lane / 32) + j;
            uint16_t av = A[(lane % 32) * K + k], bv = B[(size_t)k * 32 + (lane % 32)];
            a[j] = __builtin_bit_cast(__bf16, av);
            b[j] = __builtin_bit_cast(__bf16, bv);
        }
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
    }
    for (int r = 0; r < 16; ++r) D[(8 * (r / 4) + 4 * (lane / 32) + (r % 4)) * 32 + lane % 32] = acc[r];
}

int main() {
    std::mt19937 g(7);
    std::normal_distribution<float> nd(0.f, 1.f);
    const int T = 4096;
    std::vector<uint16_t> A(T * 512), B(T * 512);
    std::vector<float> C(T * 1024), D(T * 1024);
    for (auto& x : A) x = f2bf(nd(g));
    for (auto& x : B) x = f2bf(nd(g));
    for (auto& x : C) x = nd(g) * 4.f;
    uint16_t *dA, *dB;
    float *dC, *dD;
    hipMalloc(&dA, A.size() * 2);
    hipMalloc(&dB, B.size() * 2);
    hipMalloc(&dC, C.size() * 4);
    hipMalloc(&dD, D.size() * 4);
    hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(one_mfma, dim3(T), dim3(64), 0, 0, dA, dB, dC, dD, 1);
    hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
    long n = 0, m_once = 0, m_chain = 0, m_trunc = 0, m_chain_rev = 0;
    double bias = 0, rms = 0;
    for (int t = 0; t < T; ++t)
        for (int i = 0; i < 32; ++i)
            for (int j = 0; j < 32; ++j) {
                const float c = C[t * 1024 + i * 32 + j];
                double ex = c;
                float ch = c, chr = c;
                double prod_sum = 0;
                for (int k = 0; k < 16; ++k) {
                    const float a = bf2f(A[t * 512 + i * 16 + k]), b = bf2f(B[t * 512 + k * 32 + j]);
                    ex += (double)a * b;
                    prod_sum += (double)a * b;
                    ch = fmaf(a, b, ch);
                }
                for (int k = 15; k >= 0; --k)
                    chr = fmaf(bf2f(A[t * 512 + i * 16 + k]), bf2f(B[t * 512 + k * 32 + j]), chr);
                const float once = (float)ex;
                const double tr = std::trunc(ex * 0x1p24 / std::pow(2.0, std::floor(std::log2(std::fabs(ex))))) ;
                (void)tr;
                float trunc_f = (float)ex;
                if ((double)trunc_f != ex && std::fabs((double)trunc_f) > std::fabs(ex))
                    trunc_f = std::nextafter(trunc_f, 0.f);
                const float d = D[t * 1024 + i * 32 + j];
                ++n;
                m_once += d == once;
                m_chain += d == ch;
                m_chain_rev += d == chr;
                m_trunc += d == trunc_f;
                const double ulp = std::ldexp(1.0, std::ilogb(ex) - 23);
                const double sg = ex < 0 ? -1.0 : 1.0;
                bias += sg * (d - ex) / ulp;
                rms += ((d - ex) / ulp) * ((d - ex) / ulp);
                (void)prod_sum;
            }
    // part 2
    const int K = 608, T2 = 2048;
    std::vector<uint16_t> A2((size_t)T2 * 32 * K), B2((size_t)T2 * K * 32);
    for (auto& x : A2) x = f2bf(nd(g));
    for (auto& x : B2) x = f2bf(nd(g));
    uint16_t *dA2, *dB2;
    float* dD2;
    hipMalloc(&dA2, A2.size() * 2);
    hipMalloc(&dB2, B2.size() * 2);
    hipMalloc(&dD2, (size_t)T2 * 1024 * 4);
    hipMemcpy(dA2, A2.data(), A2.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dB2, B2.data(), B2.size() * 2, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(chain_mfma, dim3(T2), dim3(64), 0, 0, dA2, dB2, dD2, K);
    std::vector<float> D2((size_t)T2 * 1024);
    hipMemcpy(D2.data(), dD2, D2.size() * 4, hipMemcpyDeviceToHost);
    double mb = 0, mr = 0, cb = 0, cr = 0;
    long n2 = 0;
    for (int t = 0; t < T2; ++t)
        for (int i = 0; i < 32; ++i)
            for (int j = 0; j < 32; ++j) {
                double ex = 0, mag = 0;
                float ch = 0.f;
                for (int k = 0; k < K; ++k) {
                    const float a = bf2f(A2[((size_t)t * 32 + i) * K + k]), b = bf2f(B2[((size_t)t * K + k) * 32 + j]);
                    ex += (double)a * b;
                    mag += std::fabs((double)a * b);
                    ch = fmaf(a, b, ch);
                }
                const double u = mag * 0x1p-24;
                // signed toward the sum's magnitude: a truncating accumulator shows a negative mean
                const double sg = ex < 0 ? -1.0 : 1.0;
                const double e1 = sg * (D2[(size_t)t * 1024 + i * 32 + j] - ex) / u, e2 = sg * (ch - ex) / u;
                mb += e1, mr += e1 * e1, cb += e2, cr += e2 * e2;
                ++n2;
            }
    printf("K = %d chain, %ld outputs, error / (2^-24 sum|ab|), signed toward |exact|: MFMA mean %+.5f rms %.5f | host fp32 fma chain mean %+.5f rms %.5f\n",
           K, n2, mb / n2, std::sqrt(mr / n2), cb / n2, std::sqrt(cr / n2));
    printf("one v_mfma_f32_32x32x16_bf16, %ld outputs: == exact-then-RNE %ld, == fp32 fma chain k 0..15 %ld, "
           "== chain k 15..0 %ld, == exact-then-truncate %ld; error vs exact in ulps of the result (signed toward |exact|): mean %.4f rms %.4f\n",
           n, m_once, m_chain, m_chain_rev, m_trunc, bias / n, std::sqrt(rms / n));
    return 0;
}
