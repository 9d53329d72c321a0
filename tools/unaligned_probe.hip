// Probe: do global dword / dwordx2 loads at 2-byte-aligned addresses return the
// right bytes on gfx950 (ROCm's unaligned access mode), and what do they cost
// against aligned loads? Decides whether LK may read 16-bit pixel / derivative
// pairs straight from 16-bit planes at any x.
//
//   hipcc --offload-arch=gfx950 -O3 tools/unaligned_probe.hip -o tools/unaligned_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

typedef const __attribute__((address_space(1))) unsigned char* gu8;

template <typename T>
__device__ __forceinline__ T ld(gu8 base, unsigned off) {
    return *reinterpret_cast<const __attribute__((address_space(1))) T*>(base + off);
}

// every lane loads 16 values at byte offset 2 * (lane + 64 * k) + shift
template <int SHIFT>
__global__ __launch_bounds__(256) void load_kernel(const unsigned char* src, unsigned* out, int reps) {
    gu8 b = (gu8)src;
    unsigned acc = 0;
    const unsigned base = (blockIdx.x * 256u + threadIdx.x) * 2u * 16u;
    for (int r = 0; r < reps; r++) {
#pragma unroll
        for (int k = 0; k < 16; k++) acc += ld<unsigned>(b, base + 2u * k + SHIFT + (unsigned)r * 4u);
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

__global__ void check_kernel(const unsigned char* src, unsigned* out2, unsigned long long* out8) {
    gu8 b = (gu8)src;
    const unsigned o = 2u * threadIdx.x + 2u;  // 2 mod 4 for even lanes' halves, all 2-aligned
    out2[threadIdx.x] = ld<unsigned>(b, o);
    typedef unsigned u2 __attribute__((ext_vector_type(2)));
    u2 v = ld<u2>(b, o);
    out8[threadIdx.x] = (unsigned long long)v.x | ((unsigned long long)v.y << 32);
}

int main() {
    const int n = 1 << 26;
    unsigned char* h = new unsigned char[n];
    for (int i = 0; i < n; i++) h[i] = (unsigned char)(i * 37 + (i >> 8));
    unsigned char* d;
    unsigned *o, *o2;
    unsigned long long* o8;
    (void)hipMalloc(&d, n + 4096);
    (void)hipMalloc(&o, sizeof(unsigned) * (n / 32));
    (void)hipMalloc(&o2, 256 * 4);
    (void)hipMalloc(&o8, 256 * 8);
    (void)hipMemcpy(d, h, n, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(check_kernel, dim3(1), dim3(256), 0, 0, d, o2, o8);
    unsigned r2[256];
    unsigned long long r8[256];
    (void)hipMemcpy(r2, o2, sizeof(r2), hipMemcpyDeviceToHost);
    (void)hipMemcpy(r8, o8, sizeof(r8), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int t = 0; t < 256; t++) {
        unsigned e2;
        unsigned long long e8;
        std::memcpy(&e2, h + 2 * t + 2, 4);
        std::memcpy(&e8, h + 2 * t + 2, 8);
        bad += (r2[t] != e2) + (r8[t] != e8);
    }
    printf("unaligned (2-byte) dword / dwordx2 loads: %s (%d mismatches)\n", bad ? "WRONG" : "exact", bad);
    const int blocks = n / (256 * 32 * 2);
    for (int pass = 0; pass < 2; pass++) {
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        float ms0 = 0, ms2 = 0;
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(load_kernel<0>, dim3(blocks), dim3(256), 0, 0, d, o, 8);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms0, e0, e1);
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(load_kernel<2>, dim3(blocks), dim3(256), 0, 0, d, o, 8);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms2, e0, e1);
        if (pass) printf("16 overlapping dword loads per lane x 8 reps: offset 0 mod 4 %.3f ms, 2 mod 4 %.3f ms\n", ms0, ms2);
    }
    return 0;
}
