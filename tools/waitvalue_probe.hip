// Gate probe (MI355X): how soon does a small kernel run after the host decides
// to run it? (a) the host launches it then (hipLaunchKernelGGL); (b) it was queued
// earlier behind hipStreamWaitValue32 on a host-coherent word, and the host only
// writes the word. Each kernel writes a host-coherent marker; the host spins on it.
// Also with a long kernel occupying part of the GPU on another stream.
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/waitvalue_probe tools/waitvalue_probe.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

__global__ void mark_kernel(volatile int* m, int v) {
    if (blockIdx.x == 0 && threadIdx.x == 0) *m = v;
}

__global__ __launch_bounds__(256) void busy_kernel(float* out, int iters) {
    extern __shared__ float lds[];
    float a = threadIdx.x * 1e-3f, b = blockIdx.x * 1e-4f, c = 1.f, d = 0.5f;
    for (int i = 0; i < iters; i++) {
        a = a * 1.0001f + b;
        b = b * 0.9999f + c;
        c = c * 1.0002f + d;
        d = d * 0.9998f + a;
    }
    if (a + b + c + d == 12345.f) out[blockIdx.x] = a + lds[threadIdx.x];
}

using clk = std::chrono::steady_clock;
static double us_since(clk::time_point t0) { return std::chrono::duration<double, std::micro>(clk::now() - t0).count(); }

int main() {
    int attr = 0;
    CK(hipDeviceGetAttribute(&attr, hipDeviceAttributeCanUseStreamWaitValue, 0));
    std::printf("hipDeviceAttributeCanUseStreamWaitValue = %d\n", attr);
    CK(hipSetDeviceFlags(hipDeviceScheduleSpin));
    int *mark, *gate;
    CK(hipHostMalloc(&mark, 64, hipHostMallocCoherent | hipHostMallocMapped));
    CK(hipHostMalloc(&gate, 64, hipHostMallocCoherent | hipHostMallocMapped));
    *mark = 0;
    *gate = 0;
    float* bout;
    CK(hipMalloc(&bout, 1 << 20));
    hipStream_t s, sb;
    int lo, hi;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    CK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, hi));
    CK(hipStreamCreateWithPriority(&sb, hipStreamNonBlocking, lo));
    const size_t lds = 56 * 1024;  // 2 busy blocks per CU: room left for the small kernel
    CK(hipFuncSetAttribute((const void*)busy_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    volatile int* vm = mark;
    for (int busy = 0; busy < 2; busy++) {
        double la = 0, lb = 0;
        const int reps = 200;
        for (int r = 1; r <= reps; r++) {
            if (busy) hipLaunchKernelGGL(busy_kernel, dim3(512), dim3(256), lds, sb, bout, 20000);
            // (a) launch on demand
            const int va = 2 * r;
            auto t0 = clk::now();
            hipLaunchKernelGGL(mark_kernel, dim3(1), dim3(64), 0, s, mark, va);
            while (*vm != va) {
            }
            la += us_since(t0);
            // (b) pre-queued behind a gate
            const int vb = 2 * r + 1;
            CK(hipStreamWaitValue32(s, gate, (uint32_t)r, hipStreamWaitValueGte, 0xFFFFFFFFu));
            hipLaunchKernelGGL(mark_kernel, dim3(1), dim3(64), 0, s, mark, vb);
            // let the queue reach the wait
            auto tw = clk::now();
            while (us_since(tw) < 50.0) {
            }
            t0 = clk::now();
            __atomic_store_n(gate, r, __ATOMIC_RELEASE);
            while (*vm != vb) {
            }
            lb += us_since(t0);
            if (busy) CK(hipStreamSynchronize(sb));
        }
        CK(hipStreamSynchronize(s));
        std::printf("%s: launch on demand %.1f us, gated (hipStreamWaitValue32) %.1f us (mean of %d)\n",
                    busy ? "beside a long kernel" : "idle GPU", la / reps, lb / reps, reps);
    }
    std::printf("done\n");
    return 0;
}
