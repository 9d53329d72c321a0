// Second VALU issue-rate probe (companion to valu_rates.hip): which gfx950 VALU
// instructions issue at the "fast" rate (v_add_u32 / v_fma_f32: ~2 cycles per
// wave64 instruction) and which at the "slow" rate (~4 cycles: dot2, perm,
// shifts, cvt ...). 4 waves per SIMD, 8 independent chains each; wall ns per
// wave-instruction per SIMD.
//
//   hipcc --offload-arch=gfx950 -O3 tools/valu_rates2.hip -o tools/bin/valu_rates2
#include <hip/hip_runtime.h>

#include <cstdio>

#define CH8_32(OP)                                                    \
    asm volatile(OP : "+v"(a0) : "v"(b0), "v"(c0));                  \
    asm volatile(OP : "+v"(a1) : "v"(b1), "v"(c0));                  \
    asm volatile(OP : "+v"(a2) : "v"(b0), "v"(c1));                  \
    asm volatile(OP : "+v"(a3) : "v"(b1), "v"(c1));                  \
    asm volatile(OP : "+v"(a4) : "v"(b0), "v"(c0));                  \
    asm volatile(OP : "+v"(a5) : "v"(b1), "v"(c0));                  \
    asm volatile(OP : "+v"(a6) : "v"(b0), "v"(c1));                  \
    asm volatile(OP : "+v"(a7) : "v"(b1), "v"(c1));
#define CH8_64(OP)                                                    \
    asm volatile(OP : "+v"(d0) : "v"(e0), "v"(f0));                  \
    asm volatile(OP : "+v"(d1) : "v"(e1), "v"(f0));                  \
    asm volatile(OP : "+v"(d2) : "v"(e0), "v"(f1));                  \
    asm volatile(OP : "+v"(d3) : "v"(e1), "v"(f1));                  \
    asm volatile(OP : "+v"(d4) : "v"(e0), "v"(f0));                  \
    asm volatile(OP : "+v"(d5) : "v"(e1), "v"(f0));                  \
    asm volatile(OP : "+v"(d6) : "v"(e0), "v"(f1));                  \
    asm volatile(OP : "+v"(d7) : "v"(e1), "v"(f1));

#define PROBE32(NAME, OP)                                                                             \
    __global__ __launch_bounds__(256) void NAME(unsigned* sink, int iters) {                          \
        unsigned a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 ^ 9, a5 = a0 + 11;  \
        unsigned a6 = a0 + 13, a7 = a0 + 17, b0 = a0 | 0x10001, b1 = a0 * 0x10003, c0 = a0 + 1, c1 = a0 + 2; \
        for (int i = 0; i < iters; i++) {                                                             \
            _Pragma("unroll") for (int k = 0; k < 8; k++) { CH8_32(OP) }                              \
        }                                                                                             \
        if ((a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7) == 0x1234567u) sink[0] = 1;                       \
    }
#define PROBE64(NAME, OP)                                                                             \
    __global__ __launch_bounds__(256) void NAME(unsigned* sink, int iters) {                          \
        double d0 = threadIdx.x, d1 = d0 * 3, d2 = d0 * 5, d3 = d0 * 7, d4 = d0 + 9, d5 = d0 + 11;    \
        double d6 = d0 + 13, d7 = d0 + 17, e0 = d0 + 0.5, e1 = d0 * 0.25, f0 = d0 + 1, f1 = d0 + 2;   \
        for (int i = 0; i < iters; i++) {                                                             \
            _Pragma("unroll") for (int k = 0; k < 8; k++) { CH8_64(OP) }                              \
        }                                                                                             \
        if (d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7 == 1234.5) sink[0] = 1;                             \
    }

PROBE32(p_add_u32, "v_add_u32 %0, %1, %0")
PROBE32(p_sub_u32, "v_sub_u32 %0, %1, %0")
PROBE32(p_add_co, "v_add_co_u32 %0, vcc, %1, %0")
PROBE32(p_mul_f32, "v_mul_f32 %0, %1, %0")
PROBE32(p_add_f32, "v_add_f32 %0, %1, %0")
PROBE32(p_fmac_f32, "v_fmac_f32 %0, %1, %2")
PROBE32(p_max_f32, "v_max_f32 %0, %1, %0")
PROBE32(p_and_b32, "v_and_b32 %0, %1, %0")
PROBE32(p_or_b32, "v_or_b32 %0, %1, %0")
PROBE32(p_xor_b32, "v_xor_b32 %0, %1, %0")
PROBE32(p_mov_b32, "v_mov_b32 %0, %1")
PROBE32(p_lshr, "v_lshrrev_b32 %0, %1, %0")
PROBE32(p_ashr, "v_ashrrev_i32 %0, 16, %0")
PROBE32(p_lshl7, "v_lshlrev_b32 %0, 7, %0")
PROBE32(p_lshl_v, "v_lshlrev_b32 %0, %1, %0")
PROBE32(p_lshr1, "v_lshrrev_b32 %0, 1, %0")
PROBE32(p_perm_c, "v_perm_b32 %0, %1, %0, %2")
PROBE32(p_max_i32, "v_max_i32 %0, %1, %0")
PROBE32(p_min_u32, "v_min_u32 %0, %1, %0")
PROBE32(p_mul_i24, "v_mul_i32_i24 %0, %1, %0")
PROBE32(p_mul_hi, "v_mul_hi_u32 %0, %1, %0")
PROBE32(p_floor, "v_floor_f32 %0, %0")
PROBE32(p_cvt_u32, "v_cvt_f32_u32 %0, %0")
PROBE32(p_med3, "v_med3_f32 %0, %1, %2, %0")
PROBE32(p_fma_vop3, "v_fma_f32 %0, %1, %2, %0")
PROBE32(p_add_f32_dpp, "v_add_f32_dpp %0, %1, %0 row_shr:1 row_mask:0xf bank_mask:0xf")
PROBE32(p_add_u32_dpp, "v_add_u32_dpp %0, %1, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")
PROBE32(p_pk_add_u16, "v_pk_add_u16 %0, %1, %0")
PROBE32(p_dot2c_f32_bf16, "v_dot2c_f32_bf16 %0, %1, %2")
PROBE32(p_bfi, "v_bfi_b32 %0, %1, %2, %0")
PROBE32(p_lshl_add, "v_lshl_add_u32 %0, %1, 3, %0")
PROBE32(p_cmp, "v_cmp_gt_u32 vcc, %1, %0")
PROBE32(p_cndmask_s, "v_cndmask_b32_e64 %0, %1, %0, s[0:1]")
PROBE32(p_readfirstlane_mix, "v_sub_f32 %0, %1, %0")
PROBE64(p_pk_fma_f32, "v_pk_fma_f32 %0, %1, %2, %0")
PROBE64(p_pk_mul_f32, "v_pk_mul_f32 %0, %1, %0")
PROBE64(p_pk_add_f32, "v_pk_add_f32 %0, %1, %0")
PROBE64(p_fma_f64, "v_fma_f64 %0, %1, %2, %0")
PROBE64(p_add_f64, "v_add_f64 %0, %1, %0")
PROBE64(p_mul_f64, "v_mul_f64 %0, %1, %0")
PROBE64(p_lshl_b64, "v_lshlrev_b64 %0, 1, %0")
PROBE64(p_mov_b64, "v_mov_b64 %0, %1")

typedef void (*probe_t)(unsigned*, int);

int main() {
    struct {
        const char* name;
        probe_t fn;
    } P[] = {
#define E(n, f) {n, f},
        E("v_add_u32", p_add_u32) E("v_sub_u32", p_sub_u32) E("v_add_co_u32", p_add_co) E("v_mul_f32", p_mul_f32)
        E("v_add_f32", p_add_f32) E("v_fmac_f32", p_fmac_f32) E("v_max_f32", p_max_f32) E("v_and_b32", p_and_b32)
        E("v_or_b32", p_or_b32) E("v_xor_b32", p_xor_b32) E("v_mov_b32", p_mov_b32) E("v_lshrrev_b32", p_lshr)
        E("v_ashrrev_i32", p_ashr) E("v_lshlrev_b32(7)", p_lshl7) E("v_lshlrev_b32(v)", p_lshl_v)
        E("v_lshrrev_b32(1)", p_lshr1) E("v_perm_b32", p_perm_c) E("v_max_i32", p_max_i32) E("v_min_u32", p_min_u32) E("v_mul_i32_i24", p_mul_i24)
        E("v_mul_hi_u32", p_mul_hi) E("v_floor_f32", p_floor) E("v_cvt_f32_u32", p_cvt_u32) E("v_med3_f32", p_med3)
        E("v_fma_f32(vop3)", p_fma_vop3) E("v_add_f32_dpp", p_add_f32_dpp) E("v_add_u32_dpp(quad)", p_add_u32_dpp)
        E("v_pk_add_u16", p_pk_add_u16) E("v_dot2c_f32_bf16", p_dot2c_f32_bf16) E("v_bfi_b32", p_bfi)
        E("v_lshl_add_u32", p_lshl_add) E("v_cmp_gt_u32", p_cmp) E("v_cndmask(sgpr)", p_cndmask_s)
        E("v_sub_f32", p_readfirstlane_mix) E("v_pk_fma_f32", p_pk_fma_f32) E("v_pk_mul_f32", p_pk_mul_f32)
        E("v_pk_add_f32", p_pk_add_f32) E("v_fma_f64", p_fma_f64) E("v_add_f64", p_add_f64) E("v_mul_f64", p_mul_f64)
        E("v_lshlrev_b64", p_lshl_b64) E("v_mov_b64", p_mov_b64)
#undef E
    };
    const int blocks = 1024, iters = 2000;
    unsigned* sink;
    (void)hipMalloc(&sink, 4);
    printf("instruction            wall ns per wave-instruction per SIMD (4 waves/SIMD x 8 chains)\n");
    for (auto& p : P) {
        hipLaunchKernelGGL(p.fn, dim3(blocks), dim3(256), 0, 0, sink, iters);
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(p.fn, dim3(blocks), dim3(256), 0, 0, sink, iters);
        (void)hipEventRecord(e1, 0);
        (void)hipDeviceSynchronize();
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double n = (double)iters * 64;
        printf("%-22s %6.3f ns\n", p.name, ms * 1e6 / (4.0 * n));
    }
    return 0;
}
