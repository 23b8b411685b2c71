// Developer microbenchmark of the bf16 forward GEMM (ttamm::launch_gemm with A16/B16) in
// isolation: C5 layer-1 shape (M = 57344 rows, N = 512, K = 608), contiguous vs gathered A
// rows, plain store vs the hidden-layer epilogue (bias + ReLU + dropout).  Links the library's
// object files directly (the launcher is not part of the C ABI).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include -I../../<pkg>/csrc gemm_bench.cpp <objs>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "kernels.h"

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                           \
        }                                                                           \
    } while (0)

int main(int argc, char** argv) {
    const int M = argc > 1 ? std::atoi(argv[1]) : 57344;
    const int N = argc > 2 ? std::atoi(argv[2]) : 512;
    const int K = argc > 3 ? std::atoi(argv[3]) : 608;
    const int64_t table_rows = 2000000;
    const int reps = 20;
    uint16_t *A16, *B16;
    float *C, *bias;
    int64_t* idx;
    CK(hipMalloc(&A16, table_rows * K * 2));
    CK(hipMalloc(&B16, (size_t)N * K * 2));
    CK(hipMalloc(&C, (size_t)M * N * 4));
    CK(hipMalloc(&bias, N * 4));
    CK(hipMalloc(&idx, M * 8));
    CK(hipMemset(A16, 0x3c, table_rows * K * 2));  // bf16 ~0.0115
    CK(hipMemset(B16, 0x3c, (size_t)N * K * 2));
    CK(hipMemset(bias, 0, N * 4));
    std::vector<int64_t> h(M);
    std::mt19937_64 g(1);
    for (auto& v : h) v = (int64_t)(g() % table_rows);
    CK(hipMemcpy(idx, h.data(), M * 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int variant = 0; variant < 4; ++variant) {
        const bool gathered = variant & 1, hidden = variant & 2;
        ttamm::GemmBatch b;
        std::memset(&b, 0, sizeof(b));
        ttamm::GemmProblem& p = b.p[0];
        p.A16 = A16;
        p.a_idx = gathered ? idx : nullptr;
        p.lda = K;
        p.B16 = B16;
        p.ldb = K;
        p.M = M;
        p.N = N;
        p.K = K;
        p.C = C;
        p.ldc = N;
        p.bias = bias;
        p.epi = hidden ? ttamm::EPI_HIDDEN : ttamm::EPI_STORE;
        p.keep_prob = 0.85f;
        p.inv_keep = 1.f / 0.85f;
        p.rng_k0 = 1;
        p.key_split = M;
        p.a_ones_col = -1;
        b.count = 1;
        for (int w = 0; w < 3; ++w) {
            ttamm::GemmBatch c = b;
            if (ttamm::launch_gemm(c, 0)) return 2;
        }
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int r = 0; r < reps; ++r) {
            ttamm::GemmBatch c = b;
            if (ttamm::launch_gemm(c, 0)) return 2;
        }
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = 1e3 * ms / reps;
        const double tf = 2.0 * M * N * K / (us * 1e-6) / 1e12;
        std::printf("M=%d N=%d K=%d %-9s %-6s %8.1f us %7.1f TF/s\n", M, N, K, gathered ? "gathered" : "contig",
                    hidden ? "hidden" : "store", us, tf);
    }
    return 0;
}
