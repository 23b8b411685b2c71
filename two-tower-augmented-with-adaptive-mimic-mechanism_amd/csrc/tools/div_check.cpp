// Developer check: div_by_const (common.h) against the IEEE fp32 division, bit for bit, over
// the Adam bias-correction constants of steps 1..200000 (beta2 = 0.999 and 0.99), random
// c in (0, 1], and x = 0 or normal numbers spanning 2^-75 .. 2^60 (sqrt of any fp32 v >= 0).
// Build: make -C csrc tools ; run on the GPU box: ./build/div_check
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "../kernels.h"

__global__ void check(const float* cs, const float* ics, int nc, const float* xs, int nx, unsigned long long* bad,
                      float* example) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)nc * nx) return;
    const float c = cs[i / nx], ic = ics[i / nx], x = xs[i % nx];
    const float a = ttamm::div_by_const(x, c, ic);
    const float b = x / c;
    if (__float_as_uint(a) != __float_as_uint(b)) {
        if (atomicAdd(bad, 1ull) == 0) {
            example[0] = x;
            example[1] = c;
            example[2] = a;
            example[3] = b;
        }
    }
}

int main() {
    std::vector<float> cs, ics;
    for (double b2 : {0.999, 0.99, 0.9999})
        for (int t = 1; t <= 200000; t += (t < 5000 ? 1 : 37)) cs.push_back((float)std::pow(1.0 - std::pow(b2, t), 0.5));
    std::mt19937 g(5);
    std::uniform_real_distribution<float> u(1e-4f, 1.f);
    for (int i = 0; i < 20000; ++i) cs.push_back(u(g));
    for (float c : cs) ics.push_back(ttamm::correctly_rounded_reciprocal(c));
    std::vector<float> xs = {0.f};
    std::uniform_real_distribution<float> e(-75.f, 60.f), mnt(1.f, 2.f);
    for (int i = 0; i < 4096; ++i) xs.push_back(std::ldexp(mnt(g), (int)std::floor(e(g))));
    for (int k = -75; k <= 60; ++k) xs.push_back(std::ldexp(1.f, k));
    const int nc = (int)cs.size(), nx = (int)xs.size();
    float *dc, *dic, *dx, *ex;
    unsigned long long* bad;
    hipMalloc(&dc, nc * 4);
    hipMalloc(&dic, nc * 4);
    hipMalloc(&dx, nx * 4);
    hipMalloc(&ex, 16);
    hipMalloc(&bad, 8);
    hipMemcpy(dc, cs.data(), nc * 4, hipMemcpyHostToDevice);
    hipMemcpy(dic, ics.data(), nc * 4, hipMemcpyHostToDevice);
    hipMemcpy(dx, xs.data(), nx * 4, hipMemcpyHostToDevice);
    hipMemset(bad, 0, 8);
    const int64_t total = (int64_t)nc * nx;
    hipLaunchKernelGGL(check, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, 0, dc, dic, nc, dx, nx, bad, ex);
    unsigned long long nbad = 0;
    float exh[4] = {};
    hipMemcpy(&nbad, bad, 8, hipMemcpyDeviceToHost);
    hipMemcpy(exh, ex, 16, hipMemcpyDeviceToHost);
    printf("div_by_const vs IEEE division: %lld (x, c) pairs, %llu mismatches\n", (long long)total, nbad);
    if (nbad) printf("example x=%a c=%a got %a want %a\n", exh[0], exh[1], exh[2], exh[3]);
    return nbad ? 1 : 0;
}
