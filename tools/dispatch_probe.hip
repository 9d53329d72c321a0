// Dispatch probe (MI355X): why does a small kernel wait ~180 us when it is
// launched beside a long kernel (tools/cumask_probe.hip: CU masks do not help)?
// Hypothesis: the long kernel's dispatch is still in progress -- it has far more
// workgroups than fit, and each waits for a retiring one -- and the small
// kernel's packet waits behind that dispatch. A PERSISTENT long kernel (exactly
// as many workgroups as are resident at once, each looping over its share of
// the work) finishes dispatching at once; the small kernel should then start in
// the resources the long kernel leaves free.
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/dispatch_probe tools/dispatch_probe.hip
//   tools/dispatch_probe
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

__device__ __forceinline__ float spin(float a, float b, int iters) {
    float c = 1.0f, d = 0.5f;
    for (int i = 0; i < iters; i++) {
        a = a * 1.0001f + b;
        b = b * 0.9999f + c;
        c = c * 1.0002f + d;
        d = d * 0.9998f + a;
    }
    return a + b + c + d;
}

// non-persistent: one work item per 256-thread block, `items` blocks
__global__ __launch_bounds__(256) void busy_grid(float* out, int iters) {
    extern __shared__ float lds[];
    const float r = spin(threadIdx.x * 1e-3f, blockIdx.x * 1e-4f, iters);
    if (r == 12345.f) out[blockIdx.x] = r + lds[threadIdx.x];
}

// persistent: gridDim.x blocks loop over `items` work items
__global__ __launch_bounds__(256) void busy_persistent(float* out, int iters, int items) {
    extern __shared__ float lds[];
    float acc = 0.f;
    for (int it = blockIdx.x; it < items; it += gridDim.x)
        acc += spin(threadIdx.x * 1e-3f, it * 1e-4f, iters);
    if (acc == 12345.f) out[blockIdx.x] = acc + lds[threadIdx.x];
}

__global__ __launch_bounds__(256) void small_kernel(const float* in, float* out, int n) {
    __shared__ float s[256];
    float acc = 0.f;
    for (int i = threadIdx.x; i < n; i += 256) acc += in[(size_t)blockIdx.x * n + i];
    s[threadIdx.x] = acc;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) s[threadIdx.x] += s[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[blockIdx.x] = s[0];
}

static double small_latency_us(hipStream_t st, const float* in, float* out, int reps) {
    double tot = 0;
    for (int r = 0; r < reps; r++) {
        auto t0 = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(small_kernel, dim3(64), dim3(256), 0, st, in, out, 2000);
        CK(hipStreamSynchronize(st));
        tot += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    }
    return tot / reps;
}

int main() {
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int ncu = prop.multiProcessorCount;
    float *in, *out, *bout;
    CK(hipMalloc(&in, sizeof(float) * 64 * 2000));
    CK(hipMalloc(&out, sizeof(float) * 64));
    CK(hipMalloc(&bout, sizeof(float) * 65536));
    CK(hipMemset(in, 0, sizeof(float) * 64 * 2000));
    hipStream_t sb, ss;
    int lo, hi;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    CK(hipStreamCreateWithPriority(&sb, hipStreamNonBlocking, lo));
    CK(hipStreamCreateWithPriority(&ss, hipStreamNonBlocking, hi));
    const int iters = 4000, items = 16384;
    // 56 KB of LDS per block: at most 2 blocks (8 waves) per CU, so every CU keeps
    // free wave slots and registers and ~48 KB of LDS for the small kernel
    const size_t lds = 56 * 1024;
    CK(hipFuncSetAttribute((const void*)busy_grid, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CK(hipFuncSetAttribute((const void*)busy_persistent, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    std::printf("CUs %d; small kernel alone %.1f us\n", ncu, small_latency_us(ss, in, out, 50));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int mode = 0; mode < 3; mode++) {
        const int pblocks = mode == 1 ? 2 * ncu : ncu;  // persistent grids: 2 or 1 block per CU
        auto launch = [&]() {
            if (mode == 0)
                hipLaunchKernelGGL(busy_grid, dim3(items), dim3(256), lds, sb, bout, iters);
            else
                hipLaunchKernelGGL(busy_persistent, dim3(pblocks), dim3(256), lds, sb, bout, iters, items);
        };
        CK(hipEventRecord(e0, sb));
        launch();
        CK(hipEventRecord(e1, sb));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        for (int k = 0; k < 3; k++) launch();
        auto t0 = std::chrono::steady_clock::now();
        while (std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() < 1.0) {
        }
        const double lat = small_latency_us(ss, in, out, 20);
        CK(hipStreamSynchronize(sb));
        const char* names[3] = {"grid of 16384 blocks", "persistent, 2 blocks per CU", "persistent, 1 block per CU"};
        std::printf("%-30s busy alone %.3f ms | small kernel latency beside it %.1f us\n", names[mode], ms, lat);
    }
    std::printf("done\n");
    return 0;
}
