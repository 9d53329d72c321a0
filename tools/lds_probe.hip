// Micro-probe: cost of unaligned ds_read_b32 and of global_load_lds_dword
// staging on gfx950 (used to choose the LK kernel's LDS layout).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int OFF>
__global__ void lds_read(unsigned* out, int iters) {
    __shared__ uint8_t buf[8192];
    for (int i = threadIdx.x; i < 8192; i += 256) buf[i] = (uint8_t)i;
    __syncthreads();
    unsigned acc = 0;
    const int base = (threadIdx.x & 63) * 36 + OFF;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            unsigned v;
            __builtin_memcpy(&v, buf + base + k * 36 + (it & 3) * 4, 4);
            acc += v;
        }
    }
    if (acc == 0x12345) out[0] = acc;
}

__global__ void dma_stage(const uint8_t* img, unsigned* out, int pitch, int iters) {
    __shared__ uint8_t buf[4][2048];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    unsigned acc = 0;
    for (int it = 0; it < iters; it++) {
        const __attribute__((address_space(1))) uint8_t* src =
            (const __attribute__((address_space(1))) uint8_t*)(img + (size_t)((blockIdx.x * 4 + w + it * 7) & 1023) * 40 * pitch + (lane / 9) * pitch + (lane % 9) * 4);
#pragma unroll
        for (int q = 0; q < 4; q++)
            __builtin_amdgcn_global_load_lds(src + q * 7 * pitch, (__attribute__((address_space(3))) void*)(buf[w] + q * 252), 4, 0, 0);
        __builtin_amdgcn_s_waitcnt(0x0F70);
        unsigned v;
        __builtin_memcpy(&v, buf[w] + lane * 4, 4);
        acc += v;
    }
    if (acc == 0x12345) out[0] = acc;
}

__global__ void reg_stage(const uint8_t* img, unsigned* out, int pitch, int iters) {
    __shared__ unsigned buf[4][512];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    unsigned acc = 0;
    for (int it = 0; it < iters; it++) {
        const uint8_t* src = img + (size_t)((blockIdx.x * 4 + w + it * 7) & 1023) * 40 * pitch + (lane / 9) * pitch + (lane % 9) * 4;
        unsigned v[4];
#pragma unroll
        for (int q = 0; q < 4; q++) v[q] = *(const unsigned*)(src + q * 7 * pitch);
#pragma unroll
        for (int q = 0; q < 4; q++) buf[w][q * 64 + lane] = v[q];
        __builtin_amdgcn_wave_barrier();
        acc += buf[w][(lane * 3) & 255];
    }
    if (acc == 0x12345) out[0] = acc;
}

int main() {
    unsigned* out;
    uint8_t* img;
    const int pitch = 1280;
    (void)hipMalloc(&out, 64);
    (void)hipMalloc(&img, (size_t)pitch * 41000);
    (void)hipMemset(img, 1, (size_t)pitch * 41000);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    float ms;
    auto run = [&](const char* name, auto launch) {
        launch();
        (void)hipEventRecord(a);
        launch();
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms, a, b);
        printf("%-28s %8.3f ms\n", name, ms);
    };
    run("lds_read aligned", [&] { hipLaunchKernelGGL(lds_read<0>, dim3(2048), dim3(256), 0, 0, out, 2000); });
    run("lds_read +1 byte", [&] { hipLaunchKernelGGL(lds_read<1>, dim3(2048), dim3(256), 0, 0, out, 2000); });
    run("lds_read +2 byte", [&] { hipLaunchKernelGGL(lds_read<2>, dim3(2048), dim3(256), 0, 0, out, 2000); });
    run("dma_stage (4 x dword lds)", [&] { hipLaunchKernelGGL(dma_stage, dim3(2048), dim3(256), 0, 0, img, out, pitch, 200); });
    run("reg_stage (4 x dword)", [&] { hipLaunchKernelGGL(reg_stage, dim3(2048), dim3(256), 0, 0, img, out, pitch, 200); });
    return 0;
}
