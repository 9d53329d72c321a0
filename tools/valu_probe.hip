// Micro-probe: sustained VALU issue rate per SIMD on gfx950 (8 waves/SIMD,
// independent chains), for v_add_u32, v_dot2_i32_i16 and DPP adds.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void valu_add(unsigned* out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 ^ 9, a5 = a0 + 11, a6 = a0 + 13, a7 = a0 + 17;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 16; k++) {
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(a0) : "v"(a1));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(a2) : "v"(a3));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(a4) : "v"(a5));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(a6) : "v"(a7));
        }
    }
    if ((a0 ^ a2 ^ a4 ^ a6) == 0x1234567) out[0] = 1;
}
__global__ __launch_bounds__(256) void valu_dot(unsigned* out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 ^ 9, a5 = a0 + 11, a6 = a0 + 13, a7 = a0 + 17;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 16; k++) {
            asm volatile("v_dot2_i32_i16 %0, %1, %1, %0" : "+v"(a0) : "v"(a1));
            asm volatile("v_dot2_i32_i16 %0, %1, %1, %0" : "+v"(a2) : "v"(a3));
            asm volatile("v_dot2_i32_i16 %0, %1, %1, %0" : "+v"(a4) : "v"(a5));
            asm volatile("v_dot2_i32_i16 %0, %1, %1, %0" : "+v"(a6) : "v"(a7));
        }
    }
    if ((a0 ^ a2 ^ a4 ^ a6) == 0x1234567) out[0] = 1;
}
__global__ __launch_bounds__(256) void salu_mix(unsigned* out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 16; k++) {
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(a0) : "v"(a1));
            asm volatile("s_add_u32 s20, s20, 1" ::: "s20", "scc");
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(a2) : "v"(a3));
            asm volatile("s_add_u32 s21, s21, 1" ::: "s21", "scc");
        }
    }
    if ((a0 ^ a2) == 0x1234567) out[0] = 1;
}

int main() {
    unsigned* out;
    (void)hipMalloc(&out, 64);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int blocks = 256 * 8;  // 8 blocks of 4 waves per CU -> 8 waves per SIMD
    const int iters = 2000;
    auto run = [&](const char* name, void (*k)(unsigned*, int), double valu_per_iter) {
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, iters);
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, iters);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        const double waves = blocks * 4.0, valu = waves * iters * valu_per_iter;
        const double per_simd = valu / 1024.0;
        printf("%-10s %8.3f ms  %.3f VALU/ns/SIMD  (%.2f cycles/VALU at 2.4 GHz)\n", name, ms, per_simd / (ms * 1e6),
               ms * 1e6 * 2.4 / per_simd);
    };
    run("v_add", valu_add, 64);
    run("v_dot2", valu_dot, 64);
    run("v+s mix", salu_mix, 32);
    return 0;
}
