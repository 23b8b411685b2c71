// Developer micro-benchmark: what a dependent kernel boundary costs on the step's main stream.
// Build: make -C csrc tools ; run on the GPU box: ./build/gap_bench
// One iteration = a writer kernel (R bytes, float4 stores of one cache policy) + [a sync op] + a
// one-block kernel; 200 iterations timed with events, per-iteration time printed.  The variants
// separate the end-of-kernel L2 write-back of dirty lines (plain vs nt vs sc1 stores) from the
// cost of an event record / a cross-stream wait between the two kernels.
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

typedef float f32x4 __attribute__((ext_vector_type(4)));

// MODE 0 plain, 1 nontemporal, 2 sc1 (write-through), 3 sc0 sc1
template <int MODE>
__global__ __launch_bounds__(256) void writer(f32x4* __restrict__ out, int64_t n4, float v) {
    const f32x4 x = {v, v + 1.f, v + 2.f, v + 3.f};
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
        f32x4* p = out + i;
        if constexpr (MODE == 0) *p = x;
        else if constexpr (MODE == 1) __builtin_nontemporal_store(x, p);
        else if constexpr (MODE == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(x) : "memory");
        else asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(x) : "memory");
    }
}

__global__ void tiny(float* out) {
    if (threadIdx.x == 0) out[blockIdx.x] += 1.f;
}

int main() {
    const int64_t big = 44LL << 20, small = 1LL << 20;
    f32x4* buf;
    float* t;
    CK(hipMalloc(&buf, big));
    CK(hipMalloc(&t, 4096));
    hipStream_t s, aux;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&aux, hipStreamNonBlocking));
    hipEvent_t e0, e1, nt_ev, aux_ev, fork_ev, join_ev;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreate(&nt_ev));  // timing-enabled event recorded between the kernels
    CK(hipEventCreateWithFlags(&aux_ev, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&fork_ev, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&join_ev, hipEventDisableTiming));
    const int iters = 200;
    auto launch_writer = [&](int mode, int64_t bytes) {
        const int64_t n4 = bytes / 16;
        const int blocks = 2048;
        switch (mode) {
            case 0: hipLaunchKernelGGL(writer<0>, dim3(blocks), dim3(256), 0, s, buf, n4, 1.f); break;
            case 1: hipLaunchKernelGGL(writer<1>, dim3(blocks), dim3(256), 0, s, buf, n4, 1.f); break;
            case 2: hipLaunchKernelGGL(writer<2>, dim3(blocks), dim3(256), 0, s, buf, n4, 1.f); break;
            default: hipLaunchKernelGGL(writer<3>, dim3(blocks), dim3(256), 0, s, buf, n4, 1.f); break;
        }
    };
    // sync: 0 none, 1 record (no timing), 2 record (timing), 3 wait on a long-done aux event,
    // 4 fork + join through an aux-stream tiny kernel, 5 no tiny kernel at all (writer alone)
    auto run = [&](const char* name, int mode, int64_t bytes, int sync) -> int {
        auto one = [&] {
            launch_writer(mode, bytes);
            if (sync == 1) (void)hipEventRecord(aux_ev, s);
            if (sync == 2) (void)hipEventRecord(nt_ev, s);
            if (sync == 3) (void)hipStreamWaitEvent(s, aux_ev, 0);
            if (sync == 4) {
                (void)hipEventRecord(fork_ev, s);
                (void)hipStreamWaitEvent(aux, fork_ev, 0);
                hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, aux, t + 64);
                (void)hipEventRecord(join_ev, aux);
                (void)hipStreamWaitEvent(s, join_ev, 0);
            }
            if (sync != 5) hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, t);
        };
        if (sync == 3) {
            CK(hipEventRecord(aux_ev, aux));
            CK(hipStreamSynchronize(aux));
        }
        for (int i = 0; i < 20; ++i) one();
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < iters; ++i) one();
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-44s %8.2f us/iter\n", name, ms * 1e3 / iters);
        return 0;
    };
    const char* modes[4] = {"plain", "nt", "sc1", "sc0sc1"};
    char name[128];
    for (int m = 0; m < 4; ++m) {
        for (int64_t bytes : {big, small}) {
            snprintf(name, sizeof name, "writer %s %lld MB alone", modes[m], (long long)(bytes >> 20));
            if (run(name, m, bytes, 5)) return 1;
            snprintf(name, sizeof name, "writer %s %lld MB + tiny", modes[m], (long long)(bytes >> 20));
            if (run(name, m, bytes, 0)) return 1;
        }
    }
    for (int m = 0; m < 2; ++m)
        for (int sync = 1; sync <= 4; ++sync) {
            const char* sn[5] = {"", "record", "record(timing)", "wait(done aux event)", "fork+join(aux tiny)"};
            snprintf(name, sizeof name, "writer %s 44 MB + %s + tiny", modes[m], sn[sync]);
            if (run(name, m, big, sync)) return 1;
        }
    return 0;
}
