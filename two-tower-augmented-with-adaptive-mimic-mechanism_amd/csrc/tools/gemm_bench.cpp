// Developer micro-benchmark of the step's GEMM shapes (C2: R = 57344 tower rows).
// Build: make -C csrc tools ; run on the GPU box: ./build/gemm_bench
// Each case runs on the split-bf16 kernel and on the exact fp32 MFMA kernel
// (TTAMM_FP32_MFMA=exact) and prints both times and their max output difference relative to
// the output's max magnitude.
#include <hip/hip_runtime.h>

#include <cmath>
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

int main() {
    std::mt19937 g(1);
    const int R = 57344, F = 608, H = 192, D = 96;
    float* X = dev_rand((size_t)2000000 * F, g, 0.3f);
    float* W1 = dev_rand((size_t)H * F, g, 0.05f);
    float* b1 = dev_rand(H, g, 0.01f);
    float* Hb = dev_rand((size_t)R * H, g);
    float* dY = dev_rand((size_t)R * H, g);
    float* W2 = dev_rand((size_t)D * H, g, 0.05f);
    float* dF = dev_rand((size_t)R * D, g);
    float *C, *slab, *gw, *gb;
    CK(hipMalloc(&C, (size_t)R * H * 4));
    CK(hipMalloc(&slab, (size_t)(R / 512 + 1) * (F + 1) * H * 4));
    CK(hipMalloc(&gw, (size_t)H * F * 4));
    CK(hipMalloc(&gb, (size_t)H * 4));
    std::vector<int64_t> hidx(R);
    std::uniform_int_distribution<int64_t> ui(0, 1999999);
    for (auto& v : hidx) v = ui(g);
    int64_t* idx;
    CK(hipMalloc(&idx, R * 8));
    CK(hipMemcpy(idx, hidx.data(), R * 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));

    auto base = [] {
        GemmProblem p;
        std::memset(&p, 0, sizeof(p));
        p.keep_prob = 1.f;
        p.inv_keep = 1.f;
        p.a_ones_col = -1;
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
    // out: the tensor the case writes (n floats), compared between the two kernels
    // fp64 reference of C = A B^T (+ bias) on sampled outputs: max |err| / max |C| of both kernels
    auto fp64_check = [&](const char* name, const float* dA, int lda, const float* dB, int ldb, int Mr, int Nc, int K,
                          const float* dbias, auto fn) -> int {
        std::vector<float> a((size_t)Mr * lda), b((size_t)Nc * ldb), bias(Nc), out((size_t)Mr * Nc);
        CK(hipMemcpy(a.data(), dA, a.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), dB, b.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(bias.data(), dbias, Nc * 4, hipMemcpyDeviceToHost));
        double errs[2];
        for (int mode = 0; mode < 2; ++mode) {
            if (mode == 0) setenv("TTAMM_FP32_MFMA", "exact", 1);
            else unsetenv("TTAMM_FP32_MFMA");
            fn();
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(out.data(), C, out.size() * 4, hipMemcpyDeviceToHost));
            double mx = 0, md = 0;
            for (int r = 0; r < Mr; r += 97)
                for (int c = 0; c < Nc; ++c) {
                    double acc = bias[c];
                    for (int k = 0; k < K; ++k) acc += (double)a[(size_t)r * lda + k] * b[(size_t)c * ldb + k];
                    mx = std::fmax(mx, std::fabs(acc));
                    md = std::fmax(md, std::fabs(acc - out[(size_t)r * Nc + c]));
                }
            errs[mode] = md / mx;
        }
        printf("%-36s fp64 check: exact %.2e  split %.2e (max |err| / max |C|)\n", name, errs[0], errs[1]);
        return 0;
    };
    auto time_it = [&](const char* name, double flop, const float* out, size_t n, auto fn) -> int {
        std::vector<float> ref(n), got(n);
        setenv("TTAMM_FP32_MFMA", "exact", 1);
        const double us_exact = time_one(fn);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(ref.data(), out, n * 4, hipMemcpyDeviceToHost));
        unsetenv("TTAMM_FP32_MFMA");
        const double us = time_one(fn);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(got.data(), out, n * 4, hipMemcpyDeviceToHost));
        double mx = 0, md = 0;
        for (size_t i = 0; i < n; ++i) {
            mx = std::fmax(mx, std::fabs(ref[i]));
            md = std::fmax(md, std::fabs((double)ref[i] - got[i]));
        }
        printf("%-36s split %8.1f us %6.1f TF/s | exact %8.1f us %6.1f TF/s | rel diff %.2e  (%s)\n", name, us,
               flop / (us * 1e-6) / 1e12, us_exact, flop / (us_exact * 1e-6) / 1e12, mx > 0 ? md / mx : md,
               ttamm_last_error());
        return 0;
    };
    // layer-1 forward: [R, F](gathered) x W1^T -> [R, H], bias+ReLU+dropout
    time_it("fwd L1 R x 608 -> 192 (gather)", 2.0 * R * F * H, C, (size_t)R * H, [&] {
        GemmBatch b;
        std::memset(&b, 0, sizeof(b));
        GemmProblem p = base();
        p.A = X, p.a_idx = idx, p.lda = F, p.B = W1, p.ldb = F, p.M = R, p.N = H, p.K = F;
        p.epi = EPI_HIDDEN, p.C = C, p.ldc = H, p.bias = b1, p.keep_prob = 0.85f, p.inv_keep = 1.f / 0.85f;
        b.p[0] = p, b.count = 1;
        launch_gemm(b, 0);
    });
    time_it("fwd L1 (no dropout)", 2.0 * R * F * H, C, (size_t)R * H, [&] {
        GemmBatch b;
        std::memset(&b, 0, sizeof(b));
        GemmProblem p = base();
        p.A = X, p.a_idx = idx, p.lda = F, p.B = W1, p.ldb = F, p.M = R, p.N = H, p.K = F;
        p.epi = EPI_HIDDEN, p.C = C, p.ldc = H, p.bias = b1;
        b.p[0] = p, b.count = 1;
        launch_gemm(b, 0);
    });
    time_it("fwd L1 (no gather, no dropout)", 2.0 * R * F * H, C, (size_t)R * H, [&] {
        GemmBatch b;
        std::memset(&b, 0, sizeof(b));
        GemmProblem p = base();
        p.A = X, p.lda = F, p.B = W1, p.ldb = F, p.M = R, p.N = H, p.K = F;
        p.epi = EPI_HIDDEN, p.C = C, p.ldc = H, p.bias = b1;
        b.p[0] = p, b.count = 1;
        launch_gemm(b, 0);
    });
    fp64_check("fwd L2 R x 192 -> 96", Hb, H, W2, H, R, D, H, b1, [&] {
        GemmBatch b;
        std::memset(&b, 0, sizeof(b));
        GemmProblem p = base();
        p.A = Hb, p.lda = H, p.B = W2, p.ldb = H, p.M = R, p.N = D, p.K = H;
        p.epi = EPI_STORE, p.C = C, p.ldc = D, p.bias = b1;
        b.p[0] = p, b.count = 1;
        launch_gemm(b, 0);
    });
    fp64_check("fwd L1 R x 608 -> 192 (no gather)", X, F, W1, F, R, H, F, b1, [&] {
        GemmBatch b;
        std::memset(&b, 0, sizeof(b));
        GemmProblem p = base();
        p.A = X, p.lda = F, p.B = W1, p.ldb = F, p.M = R, p.N = H, p.K = F;
        p.epi = EPI_STORE, p.C = C, p.ldc = H, p.bias = b1;
        b.p[0] = p, b.count = 1;
        launch_gemm(b, 0);
    });
    time_it("fwd L2 R x 192 -> 96", 2.0 * R * H * D, C, (size_t)R * D, [&] {
        GemmBatch b;
        std::memset(&b, 0, sizeof(b));
        GemmProblem p = base();
        p.A = Hb, p.lda = H, p.B = W2, p.ldb = H, p.M = R, p.N = D, p.K = H;
        p.epi = EPI_STORE, p.C = C, p.ldc = D, p.bias = b1;
        b.p[0] = p, b.count = 1;
        launch_gemm(b, 0);
    });
    time_it("dgrad R x 96 -> 192 (W KN)", 2.0 * R * H * D, C, (size_t)R * H, [&] {
        GemmBatch b;
        std::memset(&b, 0, sizeof(b));
        GemmProblem p = base();
        p.A = dF, p.lda = D, p.B = W2, p.ldb = H, p.b_kn = 1, p.M = R, p.N = H, p.K = D;
        p.epi = EPI_DGRAD_HIDDEN, p.C = C, p.ldc = H, p.aux0 = Hb, p.ld_aux0 = H;
        b.p[0] = p, b.count = 1;
        launch_gemm(b, 0);
    });
    time_it("wgrad W1 192 x 608 over R (gather)", 2.0 * R * (F + 1) * H, gw, (size_t)H * (F - 3), [&] {
        WgradBatch wb;
        std::memset(&wb, 0, sizeof(wb));
        WgradProblem w{};
        w.dY = dY, w.ld_dy = H, w.X = X, w.x_idx = idx, w.ld_x = F, w.R = R, w.M = H, w.N = F - 3;
        w.grad_w = gw, w.grad_b = gb, w.slab = slab;
        const WgradShape sh{w.R, w.M, w.N};
        int rps[kWgradClasses];
        wgrad_rows_per_split(&sh, 1, rps);
        w.rows_per_split = rps[wgrad_class(w.M)];
        wb.p[0] = w, wb.count = 1;
        launch_wgrad(wb, 0);
    });
    time_it("wgrad W2 96 x 192 over R", 2.0 * R * (H + 1) * D, gw, (size_t)D * H, [&] {
        WgradBatch wb;
        std::memset(&wb, 0, sizeof(wb));
        WgradProblem w{};
        w.dY = dF, w.ld_dy = D, w.X = Hb, w.ld_x = H, w.R = R, w.M = D, w.N = H;
        w.grad_w = gw, w.grad_b = gb, w.slab = slab;
        const WgradShape sh{w.R, w.M, w.N};
        int rps[kWgradClasses];
        wgrad_rows_per_split(&sh, 1, rps);
        w.rows_per_split = rps[wgrad_class(w.M)];
        wb.p[0] = w, wb.count = 1;
        launch_wgrad(wb, 0);
    });
    CK(hipDeviceSynchronize());
    printf("done\n");
    return 0;
}
