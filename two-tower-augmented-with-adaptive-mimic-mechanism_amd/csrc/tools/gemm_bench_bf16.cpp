// Developer micro-benchmark of the bf16-tower (C5) GEMM shapes: R = 57344 tower rows,
// F = 608 (605 padded), H = 512, D = 256, operands bf16, fp32 accumulation.
// Build: make -C csrc tools ; run on the GPU box: ./build/gemm_bench_bf16
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../kernels.h"

using namespace ttamm;

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            return 1;                                                              \
        }                                                                          \
    } while (0)

static float* dev_rand(size_t n, std::mt19937& g, float scale = 1.f) {
    std::vector<float> h(n);
    std::normal_distribution<float> d(0.f, scale);
    for (auto& x : h) x = d(g);
    float* p;
    if (hipMalloc(&p, n * 4) != hipSuccess) return nullptr;
    if (hipMemcpy(p, h.data(), n * 4, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
    return p;
}

int main(int argc, char** argv) {
    std::mt19937 g(1);
    const int R = 57344, F = 608, H = 512, D = 256;
    const int64_t ROWS = 2000000;
    float* X = dev_rand((size_t)ROWS * F, g, 0.3f);
    uint16_t *X16, *W16;
    CK(hipMalloc(&X16, (size_t)ROWS * F * 2));
    float* W1 = dev_rand((size_t)H * F, g, 0.05f);
    CK(hipMalloc(&W16, (size_t)H * F * 2));
    float* b1 = dev_rand(H, g, 0.01f);
    float* Hb = dev_rand((size_t)R * H, g);
    float* dY = dev_rand((size_t)R * H, g);
    float* W2 = dev_rand((size_t)D * H, g, 0.05f);
    float* dF = dev_rand((size_t)R * D, g);
    float *C, *slab, *gw, *gb;
    CK(hipMalloc(&C, (size_t)R * H * 4));
    CK(hipMalloc(&slab, (size_t)256 * (F + 1) * H * 4));
    CK(hipMalloc(&gw, (size_t)H * F * 4));
    CK(hipMalloc(&gb, (size_t)H * 4));
    if (launch_to_bf16(X, ROWS, F, F, X16, F, 0) || launch_to_bf16(W1, H, F, F, W16, F, 0)) {
        printf("to_bf16 failed: %s\n", ttamm_last_error());
        return 1;
    }
    std::vector<int64_t> hidx(R), hsorted(R), hseq(R);
    std::uniform_int_distribution<int64_t> ui(0, ROWS - 1);
    for (auto& v : hidx) v = ui(g);
    hsorted = hidx;
    std::sort(hsorted.begin(), hsorted.end());
    for (int i = 0; i < R; ++i) hseq[i] = i;
    int64_t *idx, *idx_sorted, *idx_seq;
    CK(hipMalloc(&idx, R * 8));
    CK(hipMalloc(&idx_sorted, R * 8));
    CK(hipMalloc(&idx_seq, R * 8));
    CK(hipMemcpy(idx, hidx.data(), R * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(idx_sorted, hsorted.data(), R * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(idx_seq, hseq.data(), R * 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));

    auto base = [] {
        GemmProblem p;
        std::memset(&p, 0, sizeof(p));
        p.keep_prob = 1.f;
        p.inv_keep = 1.f;
        p.a_ones_col = -1;
        p.bf16 = 1;
        return p;
    };
    auto time_one = [&](auto fn) -> double {
        for (int i = 0; i < 3; ++i) fn();
        if (hipEventRecord(e0, 0) != hipSuccess) return -1;
        const int iters = 20;
        for (int i = 0; i < iters; ++i) fn();
        if (hipEventRecord(e1, 0) != hipSuccess || hipEventSynchronize(e1) != hipSuccess) return -1;
        float ms;
        if (hipEventElapsedTime(&ms, e0, e1) != hipSuccess) return -1;
        return ms * 1e3 / iters;
    };
    auto report = [&](const char* name, double flop, double us) {
        printf("%-44s %8.1f us %7.1f TF/s  %5.1f%% of bf16 peak  (%s)\n", name, us, flop / (us * 1e-6) / 1e12,
               100.0 * flop / (us * 1e-6) / 2.5e15, ttamm_last_error());
    };
    auto l1_mem = [&](const int64_t* ix, int epi, float keep) {
        GemmBatch b;
        std::memset(&b, 0, sizeof(b));
        GemmProblem p = base();
        p.A16 = X16, p.a_idx = ix, p.lda = F, p.B16 = W16, p.ldb = F, p.M = R, p.N = H, p.K = F;
        p.A = X, p.B = W1;
        p.epi = epi, p.C = C, p.ldc = H, p.bias = b1, p.keep_prob = keep, p.inv_keep = 1.f / keep;
        b.p[0] = p, b.count = 1;
        launch_gemm(b, 0);
    };
    const double l1 = 2.0 * R * F * H;
    {  // dropout keep rate of the GEMM epilogue: nonzeros with dropout / nonzeros without (ReLU only)
        std::vector<float> h((size_t)R * H);
        auto nonzero = [&]() -> double {
            if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(h.data(), C, h.size() * 4, hipMemcpyDeviceToHost) != hipSuccess)
                return -1;
            size_t nz = 0;
            for (float v : h) nz += v != 0.f;
            return (double)nz;
        };
        l1_mem(idx, EPI_HIDDEN, 1.f);
        const double base = nonzero();
        l1_mem(idx, EPI_HIDDEN, 0.85f);
        const double kept = nonzero();
        printf("dropout keep rate (p = 0.15): %.5f over %.0f ReLU-positive elements (expect 0.85)\n", kept / base, base);
    }
    report("L1 fwd bf16-mem gather, ReLU+dropout", l1, time_one([&] { l1_mem(idx, EPI_HIDDEN, 0.85f); }));
    report("L1 fwd bf16-mem gather, ReLU", l1, time_one([&] { l1_mem(idx, EPI_HIDDEN, 1.f); }));
    report("L1 fwd bf16-mem gather, store", l1, time_one([&] { l1_mem(idx, EPI_STORE, 1.f); }));
    report("L1 fwd bf16-mem sorted gather, store", l1, time_one([&] { l1_mem(idx_sorted, EPI_STORE, 1.f); }));
    report("L1 fwd bf16-mem sequential rows, store", l1, time_one([&] { l1_mem(idx_seq, EPI_STORE, 1.f); }));
    report("L1 fwd bf16-mem no index, store", l1, time_one([&] { l1_mem(nullptr, EPI_STORE, 1.f); }));
    report("L1 fwd fp32-staged (gemm_x PL1) gather, dropout", l1, time_one([&] {
               GemmBatch b;
               std::memset(&b, 0, sizeof(b));
               GemmProblem p = base();
               p.A = X, p.a_idx = idx, p.lda = F, p.B = W1, p.ldb = F, p.M = R, p.N = H, p.K = F;
               p.epi = EPI_HIDDEN, p.C = C, p.ldc = H, p.bias = b1, p.keep_prob = 0.85f, p.inv_keep = 1.f / 0.85f;
               b.p[0] = p, b.count = 1;
               launch_gemm(b, 0);
           }));
    report("L2 fwd R x 512 -> 256", 2.0 * R * H * D, time_one([&] {
               GemmBatch b;
               std::memset(&b, 0, sizeof(b));
               GemmProblem p = base();
               p.A = Hb, p.lda = H, p.B = W2, p.ldb = H, p.M = R, p.N = D, p.K = H;
               p.epi = EPI_STORE, p.C = C, p.ldc = D, p.bias = b1;
               b.p[0] = p, b.count = 1;
               launch_gemm(b, 0);
           }));
    report("dgrad R x 256 -> 512 (W KN) + ReLU'/dropout'", 2.0 * R * H * D, time_one([&] {
               GemmBatch b;
               std::memset(&b, 0, sizeof(b));
               GemmProblem p = base();
               p.A = dF, p.lda = D, p.B = W2, p.ldb = H, p.b_kn = 1, p.M = R, p.N = H, p.K = D;
               p.epi = EPI_DGRAD_HIDDEN, p.C = C, p.ldc = H, p.aux0 = Hb, p.ld_aux0 = H;
               b.p[0] = p, b.count = 1;
               launch_gemm(b, 0);
           }));
    auto wgrad = [&](const float* dy, int ldy, const float* x, const int64_t* xi, int ldx, int M, int N) {
        WgradBatch wb;
        std::memset(&wb, 0, sizeof(wb));
        WgradProblem w{};
        w.dY = dy, w.ld_dy = ldy, w.X = x, w.x_idx = xi, w.ld_x = ldx, w.R = R, w.M = M, w.N = N;
        w.grad_w = gw, w.grad_b = gb, w.slab = slab, w.bf16 = 1;
        const WgradShape sh{w.R, w.M, w.N};
        int rps[kWgradClasses];
        wgrad_rows_per_split(&sh, 1, rps);
        w.rows_per_split = rps[wgrad_class(w.M)];
        wb.p[0] = w, wb.count = 1;
        launch_wgrad(wb, 0);
    };
    report("wgrad W1 512 x 605 over R (gather)", 2.0 * R * (F - 3 + 1) * H,
           time_one([&] { wgrad(dY, H, X, idx, F, H, F - 3); }));
    report("wgrad W2 256 x 512 over R", 2.0 * R * (H + 1) * D, time_one([&] { wgrad(dF, D, Hb, nullptr, H, D, H); }));
    CK(hipDeviceSynchronize());
    printf("done\n");
    (void)argc, (void)argv;
    return 0;
}
