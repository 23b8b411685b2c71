// Developer micro-benchmark: the deferred AdamW(g = 0) replay (launch_replay) in isolation, at
// the C2 rolling-slice shape (2.2 M x 96 rows of mimic tables, 1/64 of them per launch, lag 64)
// and as a full-table flush.  Rows are warm (first moment != 0) or cold (m = +0) by a given
// fraction.  Run twice to compare the kernels: plain (LDS ring), then TTAMM_REPLAY_SCALAR=1.
// Build: make -C csrc tools ; run on the GPU box: ./build/replay_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../kernels.h"

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e = (x);                                                                    \
        if (e != hipSuccess) {                                                                 \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);       \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)

using namespace ttamm;

static AdamConsts consts_for(int64_t step) {
    const double lr = 1e-3, wd = 0.01, b1 = 0.9, b2 = 0.999, eps = 1e-8;
    const double bc1 = 1.0 - std::pow(b1, (double)step), bc2 = 1.0 - std::pow(b2, (double)step);
    AdamConsts c{};
    c.decay = (float)(1.0 - lr * wd);
    c.w1 = (float)(1.0 - b1);
    c.b2 = (float)b2;
    c.w2 = (float)(1.0 - b2);
    c.eps = (float)eps;
    c.neg_step = (float)(-lr / bc1);
    c.bc2_sqrt = (float)std::sqrt(bc2);
    c.inv_bc2_sqrt = 1.0f / c.bc2_sqrt;
    c.fast_ibc = (float)(1.0 / (std::sqrt(bc2) * (double)c.neg_step));
    c.fast_eps = (float)((double)c.eps / (double)c.neg_step);
    c.wd = (float)wd;
    c.decoupled = 1;
    c.fast_g0 = 1;
    return c;
}

int main(int argc, char** argv) {
    const int64_t R = argc > 1 ? atoll(argv[1]) : 2200000;
    const int D = 96, slices = 64, cap = 128;
    const int64_t n = R * D;
    float *p, *m, *v;
    int32_t* last;
    AdamConsts* hist;
    uint32_t* status;
    CK(hipMalloc(&p, n * 4));
    CK(hipMalloc(&m, n * 4));
    CK(hipMalloc(&v, n * 4));
    CK(hipMalloc(&last, R * 4));
    CK(hipMalloc(&hist, cap * sizeof(AdamConsts)));
    CK(hipMalloc(&status, 64));
    CK(hipMemset(status, 0, 64));
    std::vector<AdamConsts> h(cap);
    const int64_t step0 = 1000;
    for (int i = 0; i < cap; ++i) h[i] = consts_for(step0 + i);  // ring of distinct steps
    CK(hipMemcpy(hist, h.data(), cap * sizeof(AdamConsts), hipMemcpyHostToDevice));
    std::vector<float> hp(n), hm(n), hv(n);
    std::vector<int32_t> hl(R);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* impl = getenv("TTAMM_REPLAY_SCALAR") ? "scalar" : "lds-ring";
    for (double warm : {1.0, 0.5, 0.0}) {
        std::mt19937 g(7);
        std::uniform_real_distribution<float> U(-0.1f, 0.1f), P(1e-9f, 1e-6f), W(0.f, 1.f);
        for (int64_t r = 0; r < R; ++r) {
            const bool w = W(g) < warm;
            for (int d = 0; d < D; ++d) {
                hp[r * D + d] = U(g);
                hm[r * D + d] = w ? U(g) * 1e-3f : 0.f;
                hv[r * D + d] = w ? P(g) : 0.f;
            }
        }
        CK(hipMemcpy(p, hp.data(), n * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(m, hm.data(), n * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(v, hv.data(), n * 4, hipMemcpyHostToDevice));
        // slice: rows [k R / slices, (k+1) R / slices) at lag `slices`; flush: every row, lags 1..slices
        for (int mode = 0; mode < 2; ++mode) {
            const int32_t target = (int32_t)(step0 + cap - 1);
            for (int64_t r = 0; r < R; ++r) hl[r] = mode == 0 ? target - slices : target - 1 - (int32_t)(r % slices);
            CK(hipMemcpy(last, hl.data(), R * 4, hipMemcpyHostToDevice));
            ReplayArgs a{};
            a.count = 1;
            a.hist = hist;
            a.cap = cap;
            a.target = target;
            a.stamp = 0;  // keep the lags: every launch replays the same element-steps
            a.decoupled = 1;
            a.fast_g0 = 1;
            a.status = status;
            ReplaySeg& s = a.seg[0];
            s.p = p, s.m = m, s.v = v, s.last = last, s.dim = D;
            const int64_t rows = mode == 0 ? R / slices : R;
            double esteps = 0;
            for (int64_t r = 0; r < rows; ++r) esteps += (double)(target - hl[r]) * D;
            const int reps = mode == 0 ? 50 : 5;
            double best = 1e30, sum = 0;
            for (int it = 0; it < reps + 2; ++it) {
                const int64_t lo = mode == 0 ? (it % slices) * (R / slices) : 0;
                s.row_lo = lo, s.row_hi = lo + rows;
                CK(hipEventRecord(e0, 0));
                if (launch_replay(a, 0) != 0) {
                    printf("launch failed\n");
                    return 1;
                }
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (it >= 2) {
                    sum += ms;
                    best = ms < best ? ms : best;
                }
            }
            const double avg = sum / reps;
            printf("%-8s warm=%.1f %-5s rows=%lld element-steps=%.3g  avg %.4f ms  best %.4f ms  %.3g element-steps/s  "
                   "bytes %.1f MB -> %.0f GB/s\n",
                   impl, warm, mode == 0 ? "slice" : "flush", (long long)rows, esteps, avg, best, esteps / (avg * 1e-3),
                   rows * D * 24.0 / 1e6, rows * D * 24.0 / (avg * 1e-3) / 1e9);
        }
    }
    return 0;
}
