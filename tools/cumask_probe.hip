// CU-mask probe (MI355X): does a latency-critical small kernel launched beside a
// long VALU-bound kernel (the LK stand-in) start at once when the long kernel's
// stream is CU-masked to leave a few CUs free? (the front end's
// RANSAC scoring / keyframe kernels waited behind a running LK for CUs, which
// sank the pipelined-slice schedule.)
//
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/cumask_probe tools/cumask_probe.hip
//   /tmp/cumask_probe [reserved_cus_per_xcd]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                              \
        }                                                                              \
    } while (0)

// VALU-bound busy kernel: one wave per block, many blocks, a bounded loop
__global__ __launch_bounds__(64) void busy_kernel(float* out, int iters) {
    float a = threadIdx.x * 1e-3f, b = blockIdx.x * 1e-4f, c = 1.0f, d = 0.5f;
    for (int i = 0; i < iters; i++) {
        a = a * 1.0001f + b;
        b = b * 0.9999f + c;
        c = c * 1.0002f + d;
        d = d * 0.9998f + a;
    }
    if (a + b + c + d == 12345.f) out[blockIdx.x] = a;
}

// small latency-bound kernel: one block per "sequence", a short reduction
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

int main(int argc, char** argv) {
    const int reserve = argc > 1 ? std::atoi(argv[1]) : 2;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int ncu = prop.multiProcessorCount;
    std::printf("CUs %d, reserved per 32-CU word %d\n", ncu, reserve);
    float *in, *out, *bout;
    CK(hipMalloc(&in, sizeof(float) * 64 * 2000));
    CK(hipMalloc(&out, sizeof(float) * 64));
    CK(hipMalloc(&bout, sizeof(float) * 65536));
    CK(hipMemset(in, 0, sizeof(float) * 64 * 2000));
    const int words = (ncu + 31) / 32;
    std::vector<uint32_t> busy_mask(words, 0xffffffffu), crit_mask(words, 0u);
    for (int w = 0; w < words; w++)
        for (int b = 0; b < reserve; b++) {
            busy_mask[w] &= ~(1u << b);
            crit_mask[w] |= 1u << b;
        }
    hipStream_t s_plain, s_busy_masked, s_small, s_small_masked;
    CK(hipStreamCreateWithFlags(&s_plain, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s_small, hipStreamNonBlocking));
    CK(hipExtStreamCreateWithCUMask(&s_busy_masked, words, busy_mask.data()));
    CK(hipExtStreamCreateWithCUMask(&s_small_masked, words, crit_mask.data()));
    const int iters = 20000, blocks = 32768;
    // warm-up and standalone times
    hipLaunchKernelGGL(busy_kernel, dim3(blocks), dim3(64), 0, s_plain, bout, iters);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int m = 0; m < 2; m++) {
        hipStream_t sb = m ? s_busy_masked : s_plain;
        CK(hipEventRecord(e0, sb));
        hipLaunchKernelGGL(busy_kernel, dim3(blocks), dim3(64), 0, sb, bout, iters);
        CK(hipEventRecord(e1, sb));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("busy kernel alone (%s): %.3f ms\n", m ? "masked" : "all CUs", ms);
    }
    std::printf("small kernel alone: %.1f us (unmasked stream), %.1f us (reserved CUs)\n",
                small_latency_us(s_small, in, out, 50), small_latency_us(s_small_masked, in, out, 50));
    // beside a running busy kernel
    const char* names[4] = {"busy all CUs, small unmasked", "busy masked, small unmasked",
                            "busy masked, small on reserved CUs", "busy all CUs, small on reserved CUs"};
    for (int cfg = 0; cfg < 4; cfg++) {
        hipStream_t sb = (cfg == 1 || cfg == 2) ? s_busy_masked : s_plain;
        hipStream_t ss = (cfg == 2 || cfg == 3) ? s_small_masked : s_small;
        for (int k = 0; k < 4; k++) hipLaunchKernelGGL(busy_kernel, dim3(blocks), dim3(64), 0, sb, bout, iters);
        // let it fill the GPU
        auto t0 = std::chrono::steady_clock::now();
        while (std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() < 1.0) {
        }
        const double lat = small_latency_us(ss, in, out, 20);
        CK(hipEventRecord(e1, sb));
        CK(hipEventSynchronize(e1));
        std::printf("%-40s small kernel latency %.1f us\n", names[cfg], lat);
    }
    CK(hipDeviceSynchronize());
    std::printf("done\n");
    return 0;
}
