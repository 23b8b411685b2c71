// Developer micro-benchmark: whole-row gather variants at C4 shapes (128-float rows).
// Build: make -C csrc tools ; run on the GPU box: ./build/gather_bench
// Variants: rows in flight per lane (I), non-temporal stores, row-per-wave layout, and the
// table size (6.25M rows = one of 8 C4 shards; 50M rows = the whole C4 table).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <algorithm>
#include <random>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e = (x);                                                                    \
        if (e != hipSuccess) {                                                                 \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);       \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)

// D4 = 32 float4 per row; a wave moves RPW rows per iteration over I instructions
template <int I, bool NT, bool NTL>
__global__ __launch_bounds__(256) void gather_v(const float4* __restrict__ table, const int64_t* __restrict__ idx,
                                                int64_t n, float4* __restrict__ out) {
    constexpr int D4 = 32, RPW = 2 * I;
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (int64_t)gridDim.x * 4;
    for (int64_t r0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW; r0 < n; r0 += nwaves * RPW) {
        int64_t src[I];
#pragma unroll
        for (int u = 0; u < I; ++u) {
            const int64_t r = r0 + (u * 64 + lane) / D4;
            src[u] = r < n ? idx[r] : -1;
        }
        float4 v[I];
#pragma unroll
        for (int u = 0; u < I; ++u)
            if (src[u] >= 0) {
                const float4* p = table + src[u] * D4 + (u * 64 + lane) % D4;
                if (NTL) {
                    v[u].x = __builtin_nontemporal_load(&p->x);
                    v[u].y = __builtin_nontemporal_load(&p->y);
                    v[u].z = __builtin_nontemporal_load(&p->z);
                    v[u].w = __builtin_nontemporal_load(&p->w);
                } else {
                    v[u] = *p;
                }
            }
#pragma unroll
        for (int u = 0; u < I; ++u) {
            const int e = u * 64 + lane;
            const int64_t r = r0 + e / D4;
            if (r < n) {
                float4* q = out + r * D4 + e % D4;
                if (NT) {
                    __builtin_nontemporal_store(v[u].x, &q->x);
                    __builtin_nontemporal_store(v[u].y, &q->y);
                    __builtin_nontemporal_store(v[u].z, &q->z);
                    __builtin_nontemporal_store(v[u].w, &q->w);
                } else {
                    *q = v[u];
                }
            }
        }
    }
}

// read-only variant (the gather fused into a consumer: rows are summed, one float per lane out)
template <int I>
__global__ __launch_bounds__(256) void gather_read(const float4* __restrict__ table, const int64_t* __restrict__ idx,
                                                   int64_t n, float* __restrict__ out) {
    constexpr int D4 = 32, RPW = 2 * I;
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (int64_t)gridDim.x * 4;
    float acc = 0.f;
    for (int64_t r0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW; r0 < n; r0 += nwaves * RPW) {
        int64_t src[I];
#pragma unroll
        for (int u = 0; u < I; ++u) {
            const int64_t r = r0 + (u * 64 + lane) / D4;
            src[u] = r < n ? idx[r] : -1;
        }
#pragma unroll
        for (int u = 0; u < I; ++u)
            if (src[u] >= 0) {
                const float4 v = table[src[u] * D4 + (u * 64 + lane) % D4];
                acc += v.x + v.y + v.z + v.w;
            }
    }
    out[(int64_t)blockIdx.x * 256 + threadIdx.x] = acc;
}

template <class K>
static float time_it(K k, int reps, hipEvent_t e0, hipEvent_t e1) {
    for (int i = 0; i < 3; ++i) k();
    hipEventRecord(e0, 0);
    for (int i = 0; i < reps; ++i) k();
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / reps;
}

int main() {
    const int64_t big = 50000000, D = 128;
    float4* table;
    CK(hipMalloc(&table, big * D * 4));
    CK(hipMemset(table, 0x3c, big * D * 4));
    const int64_t nmax = 2000000;
    float4* out;
    CK(hipMalloc(&out, nmax * D * 4));
    int64_t* idx;
    CK(hipMalloc(&idx, nmax * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::mt19937_64 g(7);
    std::vector<int64_t> h(nmax);
    for (int64_t rows : {big, big / 8}) {
        std::uniform_int_distribution<int64_t> ui(0, rows - 1);
        for (auto& v : h) v = ui(g);
        CK(hipMemcpy(idx, h.data(), nmax * 8, hipMemcpyHostToDevice));
        for (int64_t n : {(int64_t)49152, nmax}) {
            auto run = [&](const char* name, auto kern, int rpw, bool write) {
                int64_t blocks = (n + 4 * rpw - 1) / (4 * rpw);
                if (blocks > 8192) blocks = 8192;
                const float ms = time_it([&] { hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), 0, 0, (const float4*)table, (const int64_t*)idx, n, out); }, 50, e0, e1);
                const double rb = (double)n * D * 4, tb = rb * (write ? 2 : 1) + n * 8.0;
                printf("table %9lld rows  n %8lld  %-18s %8.2f us  read %7.1f GB/s  total %7.1f GB/s\n", (long long)rows,
                       (long long)n, name, ms * 1e3, rb / ms / 1e6, tb / ms / 1e6);
            };
            run("I2", gather_v<2, false, false>, 4, true);
            run("I4", gather_v<4, false, false>, 8, true);
            run("I8", gather_v<8, false, false>, 16, true);
            run("I4 nt-store", gather_v<4, true, false>, 8, true);
            run("I8 nt-store", gather_v<8, true, false>, 16, true);
            run("I4 nt-both", gather_v<4, true, true>, 8, true);
            auto rd4 = [&](const float4* t, const int64_t* i, int64_t nn, float4* o) {
                gather_read<4><<<dim3((unsigned)std::min<int64_t>(8192, (nn + 31) / 32)), dim3(256)>>>(t, i, nn, (float*)o);
            };
            auto rd8 = [&](const float4* t, const int64_t* i, int64_t nn, float4* o) {
                gather_read<8><<<dim3((unsigned)std::min<int64_t>(8192, (nn + 63) / 64)), dim3(256)>>>(t, i, nn, (float*)o);
            };
            {
                const float ms = time_it([&] { rd4(table, idx, n, out); }, 50, e0, e1);
                printf("table %9lld rows  n %8lld  %-18s %8.2f us  read %7.1f GB/s\n", (long long)rows, (long long)n,
                       "read-only I4", ms * 1e3, (double)n * D * 4 / ms / 1e6);
                const float ms8 = time_it([&] { rd8(table, idx, n, out); }, 50, e0, e1);
                printf("table %9lld rows  n %8lld  %-18s %8.2f us  read %7.1f GB/s\n", (long long)rows, (long long)n,
                       "read-only I8", ms8 * 1e3, (double)n * D * 4 / ms8 / 1e6);
            }
            // empty-kernel floor of a back-to-back launch
            const float ms0 = time_it([&] { gather_v<4, false, false><<<1536, 256>>>(table, idx, 0, out); }, 50, e0, e1);
            printf("launch floor %.2f us\n", ms0 * 1e3);
        }
    }
    return 0;
}
