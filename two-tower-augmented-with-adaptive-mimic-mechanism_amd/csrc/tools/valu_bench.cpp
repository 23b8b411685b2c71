// Developer micro-benchmark: sustained VALU issue rate of the instructions the deferred AdamW
// replay is made of (v_fma_f32, v_pk_fma_f32, v_pk_mul_f32, v_sqrt_f32, v_rcp_f32), with the
// chip full of waves (8 independent chains per lane, 8 waves per SIMD).  Prints wave64
// instructions per second and the implied SIMD cycles per instruction at the measured clock
// (s_memtime-free: cycles = 2.4e9 x wall / (instructions per SIMD)).
// Build: make -C csrc tools ; run on the GPU box: ./build/valu_bench
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e = (x);                                                                    \
        if (e != hipSuccess) {                                                                 \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);       \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int kChains = 8, kIters = 4096;

template <int OP>
__global__ __launch_bounds__(256) void valu_kernel(float* out, float a, float b) {
    float x[kChains];
    f2 y[kChains];
#pragma unroll
    for (int i = 0; i < kChains; ++i) {
        x[i] = threadIdx.x * 1e-3f + i;
        y[i] = f2{x[i], x[i] + 0.5f};
    }
    const f2 a2 = {a, a}, b2 = {b, b};
    for (int k = 0; k < kIters; ++k) {
#pragma unroll
        for (int i = 0; i < kChains; ++i) {
            if (OP == 0) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(a), "v"(b));
            if (OP == 1) y[i] = y[i] * a2 + b2;  // v_pk_fma_f32
            if (OP == 2) y[i] = y[i] * a2;       // v_pk_mul_f32
            if (OP == 3) x[i] = __builtin_amdgcn_sqrtf(x[i]);
            if (OP == 4) x[i] = __builtin_amdgcn_rcpf(x[i]);
            if (OP == 6) asm volatile("v_mul_f32_e32 %0, %1, %0" : "+v"(x[i]) : "v"(a));
            if (OP == 7) asm volatile("v_fmac_f32_e32 %0, %1, %2" : "+v"(x[i]) : "v"(a), "v"(b));
            if (OP == 8) asm volatile("v_add_f32_e32 %0, %1, %0" : "+v"(x[i]) : "v"(b));
            if (OP == 9) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(y[i]) : "v"(a2));
            if (OP == 5) {  // the replay's warm mix per element pair: 3 pk + 2 sqrt + 2 fma + 2 rcp + ...
                x[i] = __builtin_amdgcn_rcpf(fmaf(__builtin_amdgcn_sqrtf(x[i]), a, b));
            }
        }
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < kChains; ++i) s += x[i] + y[i].x + y[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OP>
int run(const char* name, int per_iter, float* out, int cus) {
    const int blocks = cus * 8;  // 8 blocks x 4 waves = 32 waves per CU (8 per SIMD)
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(valu_kernel<OP>, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 1e-8f);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    const int reps = 5;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(valu_kernel<OP>, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 1e-8f);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double waves = (double)blocks * 4 * reps;
    const double instr = waves * kIters * kChains * per_iter;  // wave64 instructions
    const double per_simd = instr / (cus * 4.0);
    printf("%-28s %.3e wave-instr/s   %.2f cycles per wave-instr per SIMD at 2.4 GHz\n", name,
           instr / (ms * 1e-3), 2.4e9 * ms * 1e-3 / per_simd);
    return 0;
}

int main() {
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    float* out;
    CK(hipMalloc(&out, (size_t)cus * 8 * 256 * 4));
    run<0>("v_fma_f32", 1, out, cus);
    run<1>("v_pk_fma_f32", 1, out, cus);
    run<2>("v_pk_mul_f32", 1, out, cus);
    run<3>("v_sqrt_f32", 1, out, cus);
    run<4>("v_rcp_f32", 1, out, cus);
    run<5>("sqrt+fma+rcp (3 instr)", 3, out, cus);
    run<6>("v_mul_f32_e32 (VOP2)", 1, out, cus);
    run<7>("v_fmac_f32_e32 (VOP2)", 1, out, cus);
    run<8>("v_add_f32_e32 (VOP2)", 1, out, cus);
    run<9>("v_pk_mul_f32 (asm)", 1, out, cus);
    return 0;
}
