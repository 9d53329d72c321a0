// Micro-probe: sustained issue cost of single VALU / SALU instructions on one
// SIMD of gfx950, in shader cycles per wave-instruction (s_memtime around a
// loop of 8 independent chains, 4 waves per SIMD). Decides which integer /
// float forms the LK and FAST inner loops should use.
//
//   hipcc --offload-arch=gfx950 -O3 tools/valu_rates.hip -o tools/valu_rates && ./tools/valu_rates
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHAINS8(OP)                                              \
    asm volatile(OP : "+v"(a0) : "v"(b0), "v"(c0));             \
    asm volatile(OP : "+v"(a1) : "v"(b1), "v"(c0));             \
    asm volatile(OP : "+v"(a2) : "v"(b0), "v"(c1));             \
    asm volatile(OP : "+v"(a3) : "v"(b1), "v"(c1));             \
    asm volatile(OP : "+v"(a4) : "v"(b0), "v"(c0));             \
    asm volatile(OP : "+v"(a5) : "v"(b1), "v"(c0));             \
    asm volatile(OP : "+v"(a6) : "v"(b0), "v"(c1));             \
    asm volatile(OP : "+v"(a7) : "v"(b1), "v"(c1));

#define PROBE(NAME, OP)                                                                         \
    __global__ __launch_bounds__(256) void NAME(unsigned long long* cyc, unsigned* sink, int iters) { \
        unsigned a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 ^ 9, a5 = a0 + 11; \
        unsigned a6 = a0 + 13, a7 = a0 + 17, b0 = a0 | 0x10001, b1 = a0 * 0x10003, c0 = a0 + 1, c1 = a0 + 2; \
        __syncthreads();                                                                        \
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();                             \
        for (int i = 0; i < iters; i++) {                                                       \
            _Pragma("unroll") for (int k = 0; k < 8; k++) { CHAINS8(OP) }                       \
        }                                                                                       \
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();                             \
        if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;          \
        if ((a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7) == 0x1234567u) sink[0] = 1;                 \
    }

PROBE(p_add_u32, "v_add_u32 %0, %1, %0")
PROBE(p_perm, "v_perm_b32 %0, %1, %0, %2")
PROBE(p_lshl, "v_lshlrev_b32 %0, 7, %0")
PROBE(p_lshl_or, "v_lshl_or_b32 %0, %1, 7, %0")
PROBE(p_add3, "v_add3_u32 %0, %1, %2, %0")
PROBE(p_dot2_i16, "v_dot2_i32_i16 %0, %1, %2, %0")
PROBE(p_dot2c_i16, "v_dot2c_i32_i16 %0, %1, %2")
PROBE(p_dot4_i8, "v_dot4_i32_i8 %0, %1, %2, %0")
PROBE(p_dot4_u8, "v_dot4_u32_u8 %0, %1, %2, %0")
PROBE(p_dot4c_i8, "v_dot4c_i32_i8 %0, %1, %2")
PROBE(p_dot8_u4, "v_dot8_u32_u4 %0, %1, %2, %0")
PROBE(p_mad_u24, "v_mad_u32_u24 %0, %1, %2, %0")
PROBE(p_mul_lo, "v_mul_lo_u32 %0, %1, %0")
PROBE(p_fma_f32, "v_fma_f32 %0, %1, %2, %0")
PROBE(p_pk_mad_u16, "v_pk_mad_u16 %0, %1, %2, %0")
PROBE(p_pk_add_u16, "v_pk_add_u16 %0, %1, %0")
PROBE(p_dot2_f32_f16, "v_dot2_f32_f16 %0, %1, %2, %0")
PROBE(p_cvt_f32_i32, "v_cvt_f32_i32 %0, %0")
PROBE(p_add_dpp, "v_add_u32_dpp %0, %1, %0 row_shr:1 row_mask:0xf bank_mask:0xf")
PROBE(p_mov_dpp, "v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf")
PROBE(p_sad_u8, "v_sad_u8 %0, %1, %2, %0")
PROBE(p_msad_u8, "v_msad_u8 %0, %1, %2, %0")
PROBE(p_max3_u32, "v_max3_u32 %0, %1, %2, %0")
PROBE(p_bfe, "v_bfe_u32 %0, %1, 8, 8")
PROBE(p_and_or, "v_and_or_b32 %0, %1, %2, %0")
PROBE(p_cndmask, "v_cndmask_b32 %0, %1, %0, vcc")
PROBE(p_dot2_u32_u16, "v_dot2_u32_u16 %0, %1, %2, %0")
PROBE(p_pk_mad_i16, "v_pk_mad_i16 %0, %1, %2, %0")
PROBE(p_mad_i32_i16, "v_mad_i32_i16 %0, %1, %2, %0")
PROBE(p_mad_i32_i24, "v_mad_i32_i24 %0, %1, %2, %0")
PROBE(p_mul_u32_u24, "v_mul_u32_u24 %0, %1, %0")
PROBE(p_alignbyte, "v_alignbyte_b32 %0, %1, %0, %2")
PROBE(p_pk_sub_i16, "v_pk_sub_i16 %0, %1, %0")
PROBE(p_add_f32, "v_add_f32 %0, %1, %0")
PROBE(p_cvt_i32_f32, "v_cvt_i32_f32 %0, %0")
PROBE(p_rndne_f32, "v_rndne_f32 %0, %0")

typedef void (*probe_t)(unsigned long long*, unsigned*, int);

int main() {
    struct {
        const char* name;
        probe_t fn;
    } P[] = {{"v_add_u32", p_add_u32},     {"v_perm_b32", p_perm},         {"v_lshlrev_b32", p_lshl},
             {"v_lshl_or_b32", p_lshl_or}, {"v_add3_u32", p_add3},         {"v_dot2_i32_i16", p_dot2_i16},
             {"v_dot2c_i32_i16", p_dot2c_i16}, {"v_dot4_i32_i8", p_dot4_i8}, {"v_dot4_u32_u8", p_dot4_u8},
             {"v_dot4c_i32_i8", p_dot4c_i8}, {"v_dot8_u32_u4", p_dot8_u4},  {"v_mad_u32_u24", p_mad_u24},
             {"v_mul_lo_u32", p_mul_lo},   {"v_fma_f32", p_fma_f32},
             {"v_pk_mad_u16", p_pk_mad_u16}, {"v_pk_add_u16", p_pk_add_u16}, {"v_dot2_f32_f16", p_dot2_f32_f16},
             {"v_cvt_f32_i32", p_cvt_f32_i32}, {"v_add_u32_dpp", p_add_dpp}, {"v_mov_b32_dpp", p_mov_dpp},
             {"v_sad_u8", p_sad_u8},       {"v_msad_u8", p_msad_u8},       {"v_max3_u32", p_max3_u32},
             {"v_bfe_u32", p_bfe},         {"v_and_or_b32", p_and_or},     {"v_cndmask_b32", p_cndmask},
             {"v_dot2_u32_u16", p_dot2_u32_u16}, {"v_pk_mad_i16", p_pk_mad_i16}, {"v_mad_i32_i16", p_mad_i32_i16}, {"v_mad_i32_i24", p_mad_i32_i24},
             {"v_mul_u32_u24", p_mul_u32_u24}, {"v_alignbyte_b32", p_alignbyte}, {"v_pk_sub_i16", p_pk_sub_i16},
             {"v_add_f32", p_add_f32}, {"v_cvt_i32_f32", p_cvt_i32_f32}, {"v_rndne_f32", p_rndne_f32}};
    const int blocks = 1024, iters = 2000;  // 1024 x 4 waves = 4 waves per SIMD on 256 CUs
    unsigned long long* cyc;
    unsigned* sink;
    (void)hipMalloc(&cyc, sizeof(unsigned long long) * blocks * 4);
    (void)hipMalloc(&sink, 4);
    unsigned long long* h = new unsigned long long[blocks * 4];
    printf("instruction        s_memtime ticks and wall time per wave-instruction per SIMD (4 waves/SIMD, 8 chains each)\n");
    for (auto& p : P) {
        hipLaunchKernelGGL(p.fn, dim3(blocks), dim3(256), 0, 0, cyc, sink, iters);  // warm
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(p.fn, dim3(blocks), dim3(256), 0, 0, cyc, sink, iters);
        (void)hipEventRecord(e1, 0);
        (void)hipDeviceSynchronize();
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        (void)hipMemcpy(h, cyc, sizeof(unsigned long long) * blocks * 4, hipMemcpyDeviceToHost);
        double s = 0;
        for (int i = 0; i < blocks * 4; i++) s += (double)h[i];
        const double per_wave = s / (blocks * 4);     // cycles (s_memtime ticks) per wave
        const double n = (double)iters * 8 * 8;       // instructions per wave
        // wall: 4096 waves x n instructions on 1024 SIMDs
        const double ns_per = ms * 1e6 / (4.0 * n);
        printf("%-18s %6.2f ticks   %6.3f ns wall (%.2f cycles at 2.4 GHz)\n", p.name, per_wave / n / 4.0, ns_per,
               ns_per * 2.4);
    }
    return 0;
}
