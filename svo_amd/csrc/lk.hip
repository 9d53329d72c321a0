// Pyramidal Lucas-Kanade sparse optical flow for gfx950: one wave64 per feature,
// all pyramid levels in one launch.
//
// Replaces cv::calcOpticalFlowPyrLK at R:src/tracking.cpp:160-165 (temporal,
// 21x21, maxLevel 3, {COUNT+EPS, 50, 1e-3}, OPTFLOW_LK_GET_MIN_EIGENVALS) and
// :101-105 (stereo, 11x11, maxLevel 3, {COUNT+EPS, 30, 1e-3}, flags 0).
// Semantics follow OpenCV 4.x lkpyramid.cpp LKTrackerInvoker: identical
// fixed-point sampling (W_BITS 14, I stored x32, CV_DESCALE), identical float
// solve, exit and oscillation rules, identical status/err rules.
//
// MI355X design:
//  * A feature's levels are independent of every other feature, so the whole
//    coarse-to-fine pass is one launch: no grid sync between levels.
//  * The Scharr derivatives of the previous image come from its derivative
//    pyramid (scharr.hip / pyr_scharr_kernel: packed Ix | Iy << 16 per pixel,
//    stored x4, zero-padded borders as OpenCV's derivative levels), built once
//    per frame and reused by every LK call on it (OpenCV recomputes it per
//    call); the prev / next u8 pyramid levels are stored with 32-px REFLECT_101
//    borders (kPyrPad), so window reads near the image edge are branch-free.
//  * Lane <-> pixel map: lane = g*win_w + c owns column c, rows [g*RPG,
//    (g+1)*RPG): vertically adjacent window pixels share J rows, so one GN
//    iteration reads RPG+1 rows x 2 bytes per lane instead of 4 per pixel.
//    21x21 -> 63 lanes x 7 rows exactly.
//  * The normal-equation sums are integer products; they are summed EXACTLY
//    (per-lane int32, wave sum by DPP on 16-bit halves, int64 total) and then
//    rounded to float once, so the result is order-independent and bit-exact
//    against the oracle's EXACT mode (OpenCV's own float accumulation order
//    differs only by rounding of the sums).
#include "common.hpp"
#include "xcd_tile.hpp"

#include <cfloat>
#include <cstdlib>

namespace svo {

namespace {

constexpr int W_BITS = 14;
constexpr float FLT_SCALE = 1.f / (1 << 20);

__device__ __forceinline__ int descale(int x, int n) { return (x + (1 << (n - 1))) >> n; }

// OpenCV's `delta.ddot(delta) <= criteria.epsilon^2` (double products of float
// deltas) decided in float where the float sum is far enough from eps2, in double
// only inside the 2^-20 band around it
__device__ __forceinline__ bool converged(float dx, float dy, float lo, float hi, double eps2) {
    const float sf = dx * dx + dy * dy;
    bool c = sf < lo;
    if (__builtin_expect(sf >= lo && sf <= hi, 0)) {
        // (a real branch: if-converted, the double products cost every iteration of
        // every wave ~10 VALU issue slots for a band no lane is in)
        asm volatile("" ::: "memory");
        c = (double)dx * dx + (double)dy * dy <= eps2;
    }
    return c;
}
// `std::abs(a + b) < 0.01` with a float sum promoted to double: the largest float
// below 0.01 is the bound
__device__ __forceinline__ bool below_001(float v) { return fabsf(v) <= 0x1.47ae14p-7f; }

__device__ __forceinline__ int refl101(int p, int len) {
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        p = p < 0 ? -p : 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

__device__ __forceinline__ int ufloor(float v) {  // cvFloor (identical for |v| < 2^31)
    return (int)__builtin_floorf(v);
}
__device__ __forceinline__ int uround(float v) { return (int)__builtin_rintf(v); }  // cvRound
__device__ __forceinline__ float uni_f(float v) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}
__device__ __forceinline__ int uni_i(int v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// Exact wave sum of int32 values whose 64-lane total may exceed int32: sum the
// high and low 16-bit halves separately with DPP adds (exact), combine in int64.
__device__ __forceinline__ int dpp_sum(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0xb1, 0xf, 0xf, true);   // quad_perm 1,0,3,2
    v += __builtin_amdgcn_update_dpp(0, v, 0x4e, 0xf, 0xf, true);   // quad_perm 2,3,0,1
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, true);  // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, true);  // row_bcast:31
    return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ double wave_sum_exact(int v) {
    int hi = dpp_sum(v >> 16);
    int lo = dpp_sum(v & 0xFFFF);
    return (double)((long long)hi * 65536 + (long long)lo);
}

struct LKDev {
    int win_w, win_h, groups;      // strip map: groups = lanes/win_w, RPG rows each
    int ip_w, ip_h, jr_w, jr_h;    // staged prev / next pair regions (entries x rows)
    int ip_bytes, lds_wave;        // per-wave LDS carve
    int max_level, max_count;
    double eps2;
    float eps2_lo, eps2_hi;  // float brackets of eps2 (see converged())
    int flags, want_err;
    float min_eig;
    int xcd;  // lk_multi_kernel: blocks in XCD order (xcd_tile.hpp; SVO_LK_XCD=0: raster)
    int tail;  // lk_multi_kernel (21 x 21): a wave's last active feature on all 64 lanes (SVO_LK_TAIL=0: off)
};

constexpr int JM = 3;  // margin (px) of the staged next-image region around the window
// the temporal lk_multi_kernel's launch bound (waves per SIMD) and strips loaded per
// setup group (A/B builds: make EXTRA=-DSVO_LK_KKS=4 ...)
#ifndef SVO_LK_MINW
#define SVO_LK_MINW 3
#endif
#ifndef SVO_LK_KKS
#define SVO_LK_KKS 2
#endif

typedef const __attribute__((address_space(1))) uint8_t* gu8;  // global (not flat) loads
typedef const __attribute__((address_space(1))) uint32_t* gu32;
typedef short s16x2 __attribute__((ext_vector_type(2)));

// v_dot2_i32_i16: both operands signed 16-bit -- OpenCV's rounded bilinear weights
// can be -1 (iw11 = 2^14 - iw00 - iw01 - iw10), pixels 0..255 and Scharr values
// |v| <= 4080 fit, and every partial sum fits int32.
__device__ __forceinline__ int sdot2(unsigned a, unsigned b, int c) {
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(s16x2, a), __builtin_bit_cast(s16x2, b), c, false);
}
__device__ __forceinline__ unsigned pack16(int lo, int hi) {
    return ((unsigned)lo & 0xFFFFu) | ((unsigned)hi << 16);
}

// Image region at (x0, y0) as horizontal pixel pairs: entry (r, e) =
// L(x0+e, y0+r) | L(x0+e+1, y0+r) << 16, ready for one v_dot2_i32_i16 per row;
// REFLECT_101 outside the image, as OpenCV's padded pyramid levels.
__device__ __forceinline__ void stage_pairs(unsigned* dst, const ImgLevel& L, int x0, int y0, int rw,
                                            int rh, int lr, int lc, int rpp) {
    if (lr >= rpp) return;
    gu8 src = (gu8)L.data;
    const bool inside = x0 >= 0 && y0 >= 0 && x0 + rw + 1 <= L.w && y0 + rh <= L.h;
    if (inside) {
        gu8 q = src + (size_t)(y0 + lr) * L.pitch + (x0 + lc);
        const size_t step = (size_t)rpp * L.pitch;
        for (int r = lr; r < rh; r += rpp, q += step) dst[r * rw + lc] = (unsigned)q[0] | ((unsigned)q[1] << 16);
    } else {
        const int sx0 = refl101(x0 + lc, L.w), sx1 = refl101(x0 + lc + 1, L.w);
        for (int r = lr; r < rh; r += rpp) {
            gu8 row = src + (size_t)refl101(y0 + r, L.h) * L.pitch;
            dst[r * rw + lc] = (unsigned)row[sx0] | ((unsigned)row[sx1] << 16);
        }
    }
}

template <int RPG, bool FULL>
__global__ __launch_bounds__(256) void lk_kernel(LKBatch B, LKDev p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int seq = blockIdx.y;
    const int n = B.counts ? B.counts[seq] : B.n;
    const int pt = blockIdx.x * 4 + wid;
    if (pt >= n) return;
    const size_t base = (size_t)seq * B.cap;
    const float* __restrict__ prev_xy = B.prev_xy + 2 * base;
    float* __restrict__ next_xy = B.next_xy + 2 * base;
    const PyrDesc& prev = B.prev[seq];
    const PyrDesc& next = B.next[seq];
    const DerivDesc& dprev = B.dprev[seq];
    unsigned* ipair = reinterpret_cast<unsigned*>(lds + wid * p.lds_wave);
    unsigned* jreg = reinterpret_cast<unsigned*>(lds + wid * p.lds_wave + p.ip_bytes);

    const int win_w = p.win_w, win_h = p.win_h;
    const int sc = lane % win_w;
    const int sg = lane / win_w;
    const bool strip = sg < p.groups;
    const int r0 = sg * RPG;
    const int i_rpp = 64 / p.ip_w, i_lr = lane / p.ip_w, i_lc = lane - i_lr * p.ip_w;
    const int j_rpp = 64 / p.jr_w, j_lr = lane / p.jr_w, j_lc = lane - j_lr * p.jr_w;

    const float halfWx = (win_w - 1) * 0.5f, halfWy = (win_h - 1) * 0.5f;
    const float px = uni_f(prev_xy[2 * pt]), py = uni_f(prev_xy[2 * pt + 1]);
    float nx = 0.f, ny = 0.f;
    if (p.flags & SVO_LK_USE_INITIAL_FLOW) {
        nx = uni_f(next_xy[2 * pt]);
        ny = uni_f(next_xy[2 * pt + 1]);
    }
    int st = 1;
    float errv = 0.f;
    int itcount = 0;
    const int max_level = p.max_level;

    for (int level = max_level; level >= 0; level--) {
        const ImgLevel I = prev.lv[level];
        const ImgLevel J = next.lv[level];
        const float lscale = (float)(1. / (1 << level));
        float prevx = px * lscale, prevy = py * lscale;
        float nextx, nexty;
        if (level == max_level) {
            if (p.flags & SVO_LK_USE_INITIAL_FLOW) {
                nextx = nx * lscale;
                nexty = ny * lscale;
            } else {
                nextx = prevx;
                nexty = prevy;
            }
        } else {
            nextx = nx * 2.f;
            nexty = ny * 2.f;
        }
        nx = nextx;
        ny = nexty;
        prevx -= halfWx;
        prevy -= halfWy;
        const int ipx = uni_i(ufloor(prevx)), ipy = uni_i(ufloor(prevy));
        if (ipx < -win_w || ipx >= I.w || ipy < -win_h || ipy >= I.h) {
            if (level == 0) {
                st = 0;
                errv = 0.f;
            }
            continue;
        }
        float a = prevx - ipx, b = prevy - ipy;
        const int iw00 = uround((1.f - a) * (1.f - b) * (1 << W_BITS));
        const int iw01 = uround(a * (1.f - b) * (1 << W_BITS));
        const int iw10 = uround((1.f - a) * b * (1 << W_BITS));
        const int iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;
        const unsigned IW0 = pack16(iw00, iw01), IW1 = pack16(iw10, iw11);

        // ---- stage the prev window (+1 row/col, as pixel pairs) and the next-image
        //      region around the initial window: one load burst, one LDS sync.
        //      The Scharr derivative comes from the precomputed derivative pyramid
        //      (zero outside the image, as OpenCV's zero-padded derivative level). ----
        int jx0 = uni_i(ufloor(nextx - halfWx)) - JM, jy0 = uni_i(ufloor(nexty - halfWy)) - JM;
        stage_pairs(ipair, I, ipx, ipy, p.ip_w, p.ip_h, i_lr, i_lc, i_rpp);
        stage_pairs(jreg, J, jx0, jy0, p.jr_w, p.jr_h, j_lr, j_lc, j_rpp);
        uint32_t dv[RPG + 1][2];
        {
            const int dpitch = dprev.pitch[level];
            gu32 dsrc = (gu32)dprev.data[level];
            const bool full_in = ipx >= 0 && ipy >= 0 && ipx + win_w < I.w && ipy + win_h < I.h;
            const int X = ipx + sc;
            if (full_in) {
                gu32 q = dsrc + (size_t)(ipy + r0) * dpitch + X;
#pragma unroll
                for (int k = 0; k <= RPG; k++) {
                    dv[k][0] = dv[k][1] = 0;
                    if (strip && (FULL || r0 + k <= win_h)) {
                        dv[k][0] = q[(size_t)k * dpitch];
                        dv[k][1] = q[(size_t)k * dpitch + 1];
                    }
                }
            } else {
                const bool c0 = X >= 0 && X < I.w, c1 = X + 1 >= 0 && X + 1 < I.w;
#pragma unroll
                for (int k = 0; k <= RPG; k++) {
                    dv[k][0] = dv[k][1] = 0;
                    const int Y = ipy + r0 + k;
                    if (strip && (FULL || r0 + k <= win_h) && Y >= 0 && Y < I.h) {
                        gu32 q = dsrc + (size_t)Y * dpitch + X;
                        if (c0) dv[k][0] = q[0];
                        if (c1) dv[k][1] = q[1];
                    }
                }
            }
        }
        wave_lds_sync();

        // ---- per-lane strip: bilinear I (x32), Ix, Iy at its window pixels ----
        int ival[RPG], gix[RPG], giy[RPG];
        int a11 = 0, a12 = 0, a22 = 0;
        {
            const unsigned* ip = ipair + r0 * p.ip_w + sc;
            unsigned P0 = strip ? ip[0] : 0u;
#pragma unroll
            for (int j = 0; j < RPG; j++) {
                ival[j] = gix[j] = giy[j] = 0;
                if (strip && (FULL || r0 + j < win_h)) {
                    const unsigned P1 = ip[(j + 1) * p.ip_w];
                    ival[j] = sdot2(P0, IW0, sdot2(P1, IW1, 1 << (W_BITS - 6))) >> (W_BITS - 5);
                    P0 = P1;
                    const unsigned X0 = __builtin_amdgcn_perm(dv[j][1], dv[j][0], 0x05040100u);
                    const unsigned X1 = __builtin_amdgcn_perm(dv[j + 1][1], dv[j + 1][0], 0x05040100u);
                    const unsigned Y0 = __builtin_amdgcn_perm(dv[j][1], dv[j][0], 0x07060302u);
                    const unsigned Y1 = __builtin_amdgcn_perm(dv[j + 1][1], dv[j + 1][0], 0x07060302u);
                    constexpr int DS = W_BITS + kDerShift;  // derivatives are stored x 2^kDerShift
                    const int ix = sdot2(X0, IW0, sdot2(X1, IW1, 1 << (DS - 1))) >> DS;
                    const int iy = sdot2(Y0, IW0, sdot2(Y1, IW1, 1 << (DS - 1))) >> DS;
                    gix[j] = ix;
                    giy[j] = iy;
                    a11 += ix * ix;
                    a12 += ix * iy;
                    a22 += iy * iy;
                }
            }
        }
        const float A11 = (float)wave_sum_exact(a11) * FLT_SCALE;
        const float A12 = (float)wave_sum_exact(a12) * FLT_SCALE;
        const float A22 = (float)wave_sum_exact(a22) * FLT_SCALE;

        float D = A11 * A22 - A12 * A12;
        float minEig = (A22 + A11 - sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) /
                       (float)(2 * win_w * win_h);
        if (p.want_err && (p.flags & SVO_LK_GET_MIN_EIGENVALS)) errv = minEig;
        if (minEig < p.min_eig || D < FLT_EPSILON) {
            if (level == 0) st = 0;
            wave_lds_sync();
            continue;
        }
        D = 1.f / D;

        nextx -= halfWx;
        nexty -= halfWy;
        float pdx = 0.f, pdy = 0.f;
        for (int j = 0; j < p.max_count; j++) {
            const int inx = uni_i(ufloor(nextx)), iny = uni_i(ufloor(nexty));
            if (inx < -win_w || inx >= J.w || iny < -win_h || iny >= J.h) {
                if (level == 0) st = 0;
                break;
            }
            itcount++;
            if (inx < jx0 || inx > jx0 + 2 * JM || iny < jy0 || iny > jy0 + 2 * JM) {
                // the window left the staged region: re-stage around it
                jx0 = inx - JM;
                jy0 = iny - JM;
                wave_lds_sync();
                stage_pairs(jreg, J, jx0, jy0, p.jr_w, p.jr_h, j_lr, j_lc, j_rpp);
                wave_lds_sync();
            }
            a = nextx - inx;
            b = nexty - iny;
            const int w00 = uround((1.f - a) * (1.f - b) * (1 << W_BITS));
            const int w01 = uround(a * (1.f - b) * (1 << W_BITS));
            const int w10 = uround((1.f - a) * b * (1 << W_BITS));
            const int w11 = (1 << W_BITS) - w00 - w01 - w10;
            const unsigned W0 = pack16(w00, w01), W1 = pack16(w10, w11);
            int b1 = 0, b2 = 0;
            if (strip) {
                const unsigned* jp = jreg + (iny - jy0 + r0) * p.jr_w + (inx - jx0 + sc);
                unsigned p0 = jp[0];
#pragma unroll
                for (int k = 0; k < RPG; k++) {
                    if (FULL || r0 + k < win_h) {
                        const unsigned p1 = jp[(k + 1) * p.jr_w];
                        const int jv = sdot2(p0, W0, sdot2(p1, W1, 1 << (W_BITS - 6))) >> (W_BITS - 5);
                        const int diff = jv - ival[k];
                        b1 += diff * gix[k];
                        b2 += diff * giy[k];
                        p0 = p1;
                    }
                }
            }
            const float fb1 = (float)wave_sum_exact(b1) * FLT_SCALE;
            const float fb2 = (float)wave_sum_exact(b2) * FLT_SCALE;
            const float dx = (A12 * fb2 - A22 * fb1) * D;
            const float dy = (A12 * fb1 - A11 * fb2) * D;
            nextx += dx;
            nexty += dy;
            nx = nextx + halfWx;
            ny = nexty + halfWy;
            if ((double)dx * dx + (double)dy * dy <= p.eps2) break;
            if (j > 0 && (double)fabsf(dx + pdx) < 0.01 && (double)fabsf(dy + pdy) < 0.01) {
                nx -= dx * 0.5f;
                ny -= dy * 0.5f;
                break;
            }
            pdx = dx;
            pdy = dy;
        }

        if (st && p.want_err && level == 0 && !(p.flags & SVO_LK_GET_MIN_EIGENVALS)) {
            const float npx = nx - halfWx, npy = ny - halfWy;
            const int ix0 = uni_i(ufloor(npx)), iy0 = uni_i(ufloor(npy));
            if (ix0 < -win_w || ix0 >= J.w || iy0 < -win_h || iy0 >= J.h) {
                st = 0;
                continue;
            }
            if (ix0 < jx0 || ix0 > jx0 + 2 * JM || iy0 < jy0 || iy0 > jy0 + 2 * JM) {
                jx0 = ix0 - JM;
                jy0 = iy0 - JM;
                wave_lds_sync();
                stage_pairs(jreg, J, jx0, jy0, p.jr_w, p.jr_h, j_lr, j_lc, j_rpp);
                wave_lds_sync();
            }
            float aa = npx - ix0, bb = npy - iy0;
            const int w00 = uround((1.f - aa) * (1.f - bb) * (1 << W_BITS));
            const int w01 = uround(aa * (1.f - bb) * (1 << W_BITS));
            const int w10 = uround((1.f - aa) * bb * (1 << W_BITS));
            const int w11 = (1 << W_BITS) - w00 - w01 - w10;
            const unsigned W0 = pack16(w00, w01), W1 = pack16(w10, w11);
            int sad = 0;
            if (strip) {
                const unsigned* jp = jreg + (iy0 - jy0 + r0) * p.jr_w + (ix0 - jx0 + sc);
#pragma unroll
                for (int k = 0; k < RPG; k++) {
                    if (FULL || r0 + k < win_h) {
                        const int jv = sdot2(jp[k * p.jr_w], W0, sdot2(jp[(k + 1) * p.jr_w], W1,
                                                                       1 << (W_BITS - 6))) >> (W_BITS - 5);
                        const int diff = jv - ival[k];
                        sad += diff < 0 ? -diff : diff;
                    }
                }
            }
            // |diff| sums stay < 2^24 for windows <= 2048 px: exact in float
            errv = (float)wave_sum_exact(sad) * 1.f / (float)(32 * win_w * win_h);
        }
        wave_lds_sync();  // this level's LDS reads finish before the next level's staging
    }
    if (lane == 0) {
        next_xy[2 * pt] = nx;
        next_xy[2 * pt + 1] = ny;
        B.status[base + pt] = (uint8_t)st;
        if (B.err) B.err[base + pt] = errv;
        if (B.iters) B.iters[base + pt] = itcount;
    }
}

// ---------------------------------------------------------------------------
// OpenCV's own float accumulation order (SVO_LK_OPENCV_ORDER): the normal
// equations summed exactly as LKTrackerInvoker's SSE build sums them
// (lkpyramid.cpp, the CV_SIMD128 paths; oracle/lk.c:109-157, 186-238 ACC_SSE):
//  * A11 / A12 / A22: four float lanes over the columns x < se4 (lane x & 3,
//    rows in order, columns in order within a row), a scalar float chain over
//    the rest (row by row), then sA + ((q0 + q2) + (q1 + q3));
//  * b1 / b2 per iteration: four float lanes per sum over x < se8, each adding
//    float(d[x] G[x] + d[x+4] G[x+4]) for the 8-column blocks in order
//    (x & 3 = lane), a scalar chain over the rest, then
//    sb + ((c0 + c2 + 0) + (c1 + c3 + 0)).
// Every term is an integer, so a float chain equals the exact integer sum
// whenever the sum of the |terms| of the whole window stays <= 2^24 (every
// partial sum, and every combination of them, is then an exactly representable
// integer): the wave computes that bound beside the exact sums and runs the
// ordered float chains (one lane per chain, the terms staged in LDS in chain
// order) only when the bound fails. One feature per wave, the strip lane map of
// lk_kernel; all else (fixed-point sampling, solve, exits, err) as lk_kernel.
// The chains' term layout in LDS (per quantity, n = win_w * win_h ints):
//   A (3 quantities): lane k < 4 at k*win_h*M4 + y*M4 + m (x = 4m + k),
//                     scalar at 4*win_h*M4 + y*(win_w - se4) + (x - se4);
//   b (2 quantities): lane t < 4 at t*win_h*2*B8 + y*2*B8 + 2*blk + h
//                     (x = 8blk + t + 4h), scalar at win_h*se8 + y*(win_w - se8) + (x - se8).
struct CvOrder {
    int se4, se8;    // OpenCV's SIMD column ends: 4-wide covariance, 8-wide b loop
    int term_off;    // byte offset of the chain terms in the wave's LDS
};

__device__ __forceinline__ float lane_f(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
constexpr int kExact24 = 1 << 24;

template <int RPG, bool FULL>
__global__ __launch_bounds__(64) void lk_cv_kernel(LKBatch B, LKDev p, CvOrder co) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int lane = threadIdx.x;
    const int seq = blockIdx.y;
    const int n = B.counts ? B.counts[seq] : B.n;
    const int pt = blockIdx.x;
    if (pt >= n) return;
    const size_t base = (size_t)seq * B.cap;
    const float* __restrict__ prev_xy = B.prev_xy + 2 * base;
    float* __restrict__ next_xy = B.next_xy + 2 * base;
    const PyrDesc& prev = B.prev[seq];
    const PyrDesc& next = B.next[seq];
    const DerivDesc& dprev = B.dprev[seq];
    unsigned* ipair = reinterpret_cast<unsigned*>(lds);
    unsigned* jreg = reinterpret_cast<unsigned*>(lds + p.ip_bytes);
    int* terms = reinterpret_cast<int*>(lds + co.term_off);

    const int win_w = p.win_w, win_h = p.win_h;
    const int npx = win_w * win_h;
    const int sc = lane % win_w;
    const int sg = lane / win_w;
    const bool strip = sg < p.groups;
    const int r0 = sg * RPG;
    const int i_rpp = 64 / p.ip_w, i_lr = lane / p.ip_w, i_lc = lane - i_lr * p.ip_w;
    const int j_rpp = 64 / p.jr_w, j_lr = lane / p.jr_w, j_lc = lane - j_lr * p.jr_w;

    // this lane's column in the chain layouts (slot of row y = base + y * stride)
    const int se4 = co.se4, se8 = co.se8, M4 = se4 >> 2, B8 = se8 >> 3;
    int a_base, a_stride, b_base, b_stride;
    if (sc < se4) {
        a_base = (sc & 3) * win_h * M4 + (sc >> 2);
        a_stride = M4;
    } else {
        a_base = 4 * win_h * M4 + (sc - se4);
        a_stride = win_w - se4;
    }
    if (sc < se8) {
        b_base = (sc & 3) * win_h * 2 * B8 + 2 * (sc >> 3) + ((sc >> 2) & 1);
        b_stride = 2 * B8;
    } else {
        b_base = win_h * se8 + (sc - se8);
        b_stride = win_w - se8;
    }
    // chain lanes: A: lane = 5q + k (q: A11, A12, A22; k < 4 SIMD lane, 4 scalar);
    // b: lane = 5q + k (q: b1, b2)
    const int cq = lane / 5, ck = lane - 5 * (lane / 5);
    const int a_len = ck < 4 ? win_h * M4 : win_h * (win_w - se4);
    const int* a_src = terms + cq * npx + (ck < 4 ? ck * win_h * M4 : 4 * win_h * M4);
    const int b_len = ck < 4 ? win_h * B8 : win_h * (win_w - se8);
    const int* b_src = terms + cq * npx + (ck < 4 ? ck * win_h * 2 * B8 : win_h * se8);

    const float halfWx = (win_w - 1) * 0.5f, halfWy = (win_h - 1) * 0.5f;
    const float px = uni_f(prev_xy[2 * pt]), py = uni_f(prev_xy[2 * pt + 1]);
    float nx = 0.f, ny = 0.f;
    if (p.flags & SVO_LK_USE_INITIAL_FLOW) {
        nx = uni_f(next_xy[2 * pt]);
        ny = uni_f(next_xy[2 * pt + 1]);
    }
    int st = 1;
    float errv = 0.f;
    int itcount = 0;
    const int max_level = p.max_level;

    for (int level = max_level; level >= 0; level--) {
        const ImgLevel I = prev.lv[level];
        const ImgLevel J = next.lv[level];
        const float lscale = (float)(1. / (1 << level));
        float prevx = px * lscale, prevy = py * lscale;
        float nextx, nexty;
        if (level == max_level) {
            if (p.flags & SVO_LK_USE_INITIAL_FLOW) {
                nextx = nx * lscale;
                nexty = ny * lscale;
            } else {
                nextx = prevx;
                nexty = prevy;
            }
        } else {
            nextx = nx * 2.f;
            nexty = ny * 2.f;
        }
        nx = nextx;
        ny = nexty;
        prevx -= halfWx;
        prevy -= halfWy;
        const int ipx = uni_i(ufloor(prevx)), ipy = uni_i(ufloor(prevy));
        if (ipx < -win_w || ipx >= I.w || ipy < -win_h || ipy >= I.h) {
            if (level == 0) {
                st = 0;
                errv = 0.f;
            }
            continue;
        }
        float a = prevx - ipx, b = prevy - ipy;
        const int iw00 = uround((1.f - a) * (1.f - b) * (1 << W_BITS));
        const int iw01 = uround(a * (1.f - b) * (1 << W_BITS));
        const int iw10 = uround((1.f - a) * b * (1 << W_BITS));
        const int iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;
        const unsigned IW0 = pack16(iw00, iw01), IW1 = pack16(iw10, iw11);

        int jx0 = uni_i(ufloor(nextx - halfWx)) - JM, jy0 = uni_i(ufloor(nexty - halfWy)) - JM;
        stage_pairs(ipair, I, ipx, ipy, p.ip_w, p.ip_h, i_lr, i_lc, i_rpp);
        stage_pairs(jreg, J, jx0, jy0, p.jr_w, p.jr_h, j_lr, j_lc, j_rpp);
        uint32_t dv[RPG + 1][2];
        {
            const int dpitch = dprev.pitch[level];
            gu32 dsrc = (gu32)dprev.data[level];
            const bool full_in = ipx >= 0 && ipy >= 0 && ipx + win_w < I.w && ipy + win_h < I.h;
            const int X = ipx + sc;
            if (full_in) {
                gu32 q = dsrc + (size_t)(ipy + r0) * dpitch + X;
#pragma unroll
                for (int k = 0; k <= RPG; k++) {
                    dv[k][0] = dv[k][1] = 0;
                    if (strip && (FULL || r0 + k <= win_h)) {
                        dv[k][0] = q[(size_t)k * dpitch];
                        dv[k][1] = q[(size_t)k * dpitch + 1];
                    }
                }
            } else {
                const bool c0 = X >= 0 && X < I.w, c1 = X + 1 >= 0 && X + 1 < I.w;
#pragma unroll
                for (int k = 0; k <= RPG; k++) {
                    dv[k][0] = dv[k][1] = 0;
                    const int Y = ipy + r0 + k;
                    if (strip && (FULL || r0 + k <= win_h) && Y >= 0 && Y < I.h) {
                        gu32 q = dsrc + (size_t)Y * dpitch + X;
                        if (c0) dv[k][0] = q[0];
                        if (c1) dv[k][1] = q[1];
                    }
                }
            }
        }
        wave_lds_sync();

        int ival[RPG], gix[RPG], giy[RPG];
        int a11 = 0, a12 = 0, a22 = 0;
        {
            const unsigned* ip = ipair + r0 * p.ip_w + sc;
            unsigned P0 = strip ? ip[0] : 0u;
#pragma unroll
            for (int j = 0; j < RPG; j++) {
                ival[j] = gix[j] = giy[j] = 0;
                if (strip && (FULL || r0 + j < win_h)) {
                    const unsigned P1 = ip[(j + 1) * p.ip_w];
                    ival[j] = sdot2(P0, IW0, sdot2(P1, IW1, 1 << (W_BITS - 6))) >> (W_BITS - 5);
                    P0 = P1;
                    const unsigned X0 = __builtin_amdgcn_perm(dv[j][1], dv[j][0], 0x05040100u);
                    const unsigned X1 = __builtin_amdgcn_perm(dv[j + 1][1], dv[j + 1][0], 0x05040100u);
                    const unsigned Y0 = __builtin_amdgcn_perm(dv[j][1], dv[j][0], 0x07060302u);
                    const unsigned Y1 = __builtin_amdgcn_perm(dv[j + 1][1], dv[j + 1][0], 0x07060302u);
                    constexpr int DS = W_BITS + kDerShift;
                    const int ix = sdot2(X0, IW0, sdot2(X1, IW1, 1 << (DS - 1))) >> DS;
                    const int iy = sdot2(Y0, IW0, sdot2(Y1, IW1, 1 << (DS - 1))) >> DS;
                    gix[j] = ix;
                    giy[j] = iy;
                    a11 += ix * ix;
                    a12 += ix * iy;
                    a22 += iy * iy;
                }
            }
        }
        const double e11 = wave_sum_exact(a11), e12 = wave_sum_exact(a12), e22 = wave_sum_exact(a22);
        float A11, A12, A22;
        // sum |Ix Iy| <= (sum Ix^2 + sum Iy^2) / 2: every chain exact under these bounds
        if (e11 <= kExact24 && e22 <= kExact24 && e11 + e22 <= 2.0 * kExact24) {
            A11 = (float)e11 * FLT_SCALE;
            A12 = (float)e12 * FLT_SCALE;
            A22 = (float)e22 * FLT_SCALE;
        } else {
            if (strip) {
#pragma unroll
                for (int j = 0; j < RPG; j++) {
                    if (FULL || r0 + j < win_h) {
                        const int s = a_base + (r0 + j) * a_stride;
                        terms[s] = gix[j] * gix[j];
                        terms[npx + s] = gix[j] * giy[j];
                        terms[2 * npx + s] = giy[j] * giy[j];
                    }
                }
            }
            wave_lds_sync();
            float acc = 0.f;
            if (lane < 15)
                for (int i = 0; i < a_len; i++) acc += (float)a_src[i];
            wave_lds_sync();
            A11 = (lane_f(acc, 4) + ((lane_f(acc, 0) + lane_f(acc, 2)) + (lane_f(acc, 1) + lane_f(acc, 3)))) *
                  FLT_SCALE;
            A12 = (lane_f(acc, 9) + ((lane_f(acc, 5) + lane_f(acc, 7)) + (lane_f(acc, 6) + lane_f(acc, 8)))) *
                  FLT_SCALE;
            A22 = (lane_f(acc, 14) + ((lane_f(acc, 10) + lane_f(acc, 12)) + (lane_f(acc, 11) + lane_f(acc, 13)))) *
                  FLT_SCALE;
        }

        float D = A11 * A22 - A12 * A12;
        float minEig = (A22 + A11 - sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) /
                       (float)(2 * win_w * win_h);
        if (p.want_err && (p.flags & SVO_LK_GET_MIN_EIGENVALS)) errv = minEig;
        if (minEig < p.min_eig || D < FLT_EPSILON) {
            if (level == 0) st = 0;
            wave_lds_sync();
            continue;
        }
        D = 1.f / D;

        nextx -= halfWx;
        nexty -= halfWy;
        float pdx = 0.f, pdy = 0.f;
        for (int j = 0; j < p.max_count; j++) {
            const int inx = uni_i(ufloor(nextx)), iny = uni_i(ufloor(nexty));
            if (inx < -win_w || inx >= J.w || iny < -win_h || iny >= J.h) {
                if (level == 0) st = 0;
                break;
            }
            itcount++;
            if (inx < jx0 || inx > jx0 + 2 * JM || iny < jy0 || iny > jy0 + 2 * JM) {
                jx0 = inx - JM;
                jy0 = iny - JM;
                wave_lds_sync();
                stage_pairs(jreg, J, jx0, jy0, p.jr_w, p.jr_h, j_lr, j_lc, j_rpp);
                wave_lds_sync();
            }
            a = nextx - inx;
            b = nexty - iny;
            const int w00 = uround((1.f - a) * (1.f - b) * (1 << W_BITS));
            const int w01 = uround(a * (1.f - b) * (1 << W_BITS));
            const int w10 = uround((1.f - a) * b * (1 << W_BITS));
            const int w11 = (1 << W_BITS) - w00 - w01 - w10;
            const unsigned W0 = pack16(w00, w01), W1 = pack16(w10, w11);
            int b1 = 0, b2 = 0, babs = 0;
            int pb1[RPG], pb2[RPG];
            if (strip) {
                const unsigned* jp = jreg + (iny - jy0 + r0) * p.jr_w + (inx - jx0 + sc);
                unsigned p0 = jp[0];
#pragma unroll
                for (int k = 0; k < RPG; k++) {
                    pb1[k] = pb2[k] = 0;
                    if (FULL || r0 + k < win_h) {
                        const unsigned p1 = jp[(k + 1) * p.jr_w];
                        const int jv = sdot2(p0, W0, sdot2(p1, W1, 1 << (W_BITS - 6))) >> (W_BITS - 5);
                        const int diff = jv - ival[k];
                        pb1[k] = diff * gix[k];
                        pb2[k] = diff * giy[k];
                        b1 += pb1[k];
                        b2 += pb2[k];
                        // |terms| <= 8160 * 4080 < 2^25: capped per lane so 64 lanes cannot overflow
                        babs = min(babs + abs(pb1[k]) + abs(pb2[k]), kExact24 + 1);
                        p0 = p1;
                    }
                }
            }
            float fb1, fb2;
            if (dpp_sum(babs) <= kExact24) {
                fb1 = (float)wave_sum_exact(b1) * FLT_SCALE;
                fb2 = (float)wave_sum_exact(b2) * FLT_SCALE;
            } else {
                if (strip) {
#pragma unroll
                    for (int k = 0; k < RPG; k++) {
                        if (FULL || r0 + k < win_h) {
                            const int s = b_base + (r0 + k) * b_stride;
                            terms[s] = pb1[k];
                            terms[npx + s] = pb2[k];
                        }
                    }
                }
                wave_lds_sync();
                float acc = 0.f;
                // (two loops: the SIMD-lane chains add a pair per term, the scalar
                // chain single terms; one loop with a per-term branch on the step cost
                // ~10 instructions per term and ran max(len) times for both kinds)
                if (lane < 10) {
                    if (ck < 4) {
#pragma unroll 6
                        for (int i = 0; i < b_len; i++) acc += (float)(b_src[2 * i] + b_src[2 * i + 1]);
                    } else {
#pragma unroll 8
                        for (int i = 0; i < b_len; i++) acc += (float)b_src[i];
                    }
                }
                wave_lds_sync();
                fb1 = (lane_f(acc, 4) + (((lane_f(acc, 0) + lane_f(acc, 2)) + 0.f) +
                                         ((lane_f(acc, 1) + lane_f(acc, 3)) + 0.f))) * FLT_SCALE;
                fb2 = (lane_f(acc, 9) + (((lane_f(acc, 5) + lane_f(acc, 7)) + 0.f) +
                                         ((lane_f(acc, 6) + lane_f(acc, 8)) + 0.f))) * FLT_SCALE;
            }
            const float dx = (A12 * fb2 - A22 * fb1) * D;
            const float dy = (A12 * fb1 - A11 * fb2) * D;
            nextx += dx;
            nexty += dy;
            nx = nextx + halfWx;
            ny = nexty + halfWy;
            if ((double)dx * dx + (double)dy * dy <= p.eps2) break;
            if (j > 0 && (double)fabsf(dx + pdx) < 0.01 && (double)fabsf(dy + pdy) < 0.01) {
                nx -= dx * 0.5f;
                ny -= dy * 0.5f;
                break;
            }
            pdx = dx;
            pdy = dy;
        }

        if (st && p.want_err && level == 0 && !(p.flags & SVO_LK_GET_MIN_EIGENVALS)) {
            // SAD: sum |diff| <= 2048 * 8160 < 2^24, exact in any order
            const float npx_ = nx - halfWx, npy_ = ny - halfWy;
            const int ix0 = uni_i(ufloor(npx_)), iy0 = uni_i(ufloor(npy_));
            if (ix0 < -win_w || ix0 >= J.w || iy0 < -win_h || iy0 >= J.h) {
                st = 0;
                continue;
            }
            if (ix0 < jx0 || ix0 > jx0 + 2 * JM || iy0 < jy0 || iy0 > jy0 + 2 * JM) {
                jx0 = ix0 - JM;
                jy0 = iy0 - JM;
                wave_lds_sync();
                stage_pairs(jreg, J, jx0, jy0, p.jr_w, p.jr_h, j_lr, j_lc, j_rpp);
                wave_lds_sync();
            }
            float aa = npx_ - ix0, bb = npy_ - iy0;
            const int w00 = uround((1.f - aa) * (1.f - bb) * (1 << W_BITS));
            const int w01 = uround(aa * (1.f - bb) * (1 << W_BITS));
            const int w10 = uround((1.f - aa) * bb * (1 << W_BITS));
            const int w11 = (1 << W_BITS) - w00 - w01 - w10;
            const unsigned W0 = pack16(w00, w01), W1 = pack16(w10, w11);
            int sad = 0;
            if (strip) {
                const unsigned* jp = jreg + (iy0 - jy0 + r0) * p.jr_w + (ix0 - jx0 + sc);
#pragma unroll
                for (int k = 0; k < RPG; k++) {
                    if (FULL || r0 + k < win_h) {
                        const int jv = sdot2(jp[k * p.jr_w], W0, sdot2(jp[(k + 1) * p.jr_w], W1,
                                                                       1 << (W_BITS - 6))) >> (W_BITS - 5);
                        const int diff = jv - ival[k];
                        sad += diff < 0 ? -diff : diff;
                    }
                }
            }
            errv = (float)wave_sum_exact(sad) * 1.f / (float)(32 * win_w * win_h);
        }
        wave_lds_sync();
    }
    if (lane == 0) {
        next_xy[2 * pt] = nx;
        next_xy[2 * pt + 1] = ny;
        B.status[base + pt] = (uint8_t)st;
        if (B.err) B.err[base + pt] = errv;
        if (B.iters) B.iters[base + pt] = itcount;
    }
}

// ---------------------------------------------------------------------------
// Specialised kernel for compile-time window sizes (the reference's 21x21 and
// 11x11, plus 15x15 / 31x31). Same semantics and lane map as lk_kernel; the
// differences are all instruction count:
//  * staging loads whole aligned dwords (4 pixels) per lane and builds the 4
//    pixel pairs with v_perm from its dword and the next lane's (ds_bpermute),
//    one ds_write_b128 per lane: 1 VMEM instruction per 4 pairs instead of 8;
//  * LDS strides are compile-time (ds_read2 with immediate offsets);
//  * two window rows are processed per packed op: the J-I differences of a row
//    pair are packed to int16x2 (v_perm + v_pk_sub_i16) and multiplied into the
//    normal equations with one v_dot2_i32_i16 per sum (b1, b2, A11, A12, A22),
//    replacing two quarter-rate v_mul_lo_u32 per pixel and sum.
// All values fit int16 (|J - I| <= 8160, |Ix|, |Iy| <= 4080) and the per-lane
// int32 sums cannot overflow (7 rows x 2 x 8160 x 4080 < 2^31), so the sums are
// the same exact integers as before: bit-identical results.
constexpr int ru4(int v) { return (v + 3) & ~3; }
typedef uint32_t u32x2a4 __attribute__((ext_vector_type(2), aligned(4)));
typedef uint16_t u16a1 __attribute__((aligned(1)));
typedef const __attribute__((address_space(1))) u16a1* gu16u;  // unaligned 2-byte global loads

// Global loads at a wave-uniform base plus an unsigned 32-bit byte offset: the
// saddr + voffset form (no 64-bit address arithmetic per lane). Padded levels:
// the base is the padded origin, so every offset inside the padding is >= 0.
template <typename T>
__device__ __forceinline__ T ldg_off(gu8 base, unsigned off) {
    return *(const __attribute__((address_space(1))) T*)(base + off);
}
__device__ __forceinline__ gu8 pad_origin(const uint8_t* data, int pitch, int pad_px, int elem) {
    return (gu8)data - (size_t)pad_px * ((size_t)pitch + 1) * elem;
}
typedef const __attribute__((address_space(4))) PyrDesc* cpyr;  // scalar (s_load) descriptor reads

template <int WW, int WH>
struct Shape {
    static constexpr int G = 64 / WW;               // row groups of the strip map
    static constexpr int RPG = (WH + G - 1) / G;     // rows per group
    static constexpr bool FULL = G * RPG == WH;
    static constexpr int NP = (RPG + 1) / 2;        // packed row pairs per lane
    static constexpr int IPW = ru4(WW + 3), IPH = WH + 1;           // I pairs: entries x rows
    static constexpr int JRW = ru4(WW + 2 * JM + 3), JRH = WH + 1 + 2 * JM;
    static constexpr int IBYTES = IPW * IPH * 4, JBYTES = JRW * JRH * 4;
    static constexpr int WAVE_BYTES = IBYTES + JBYTES + 16;  // + a sink for the stager's spare lanes
};

// v_perm selector picking bytes sh, sh+1 of the 8-byte pair {hi:lo} into the
// 16-bit lanes of a pixel pair (p[sh] | p[sh+1] << 16).
__device__ __forceinline__ unsigned pair_sel(unsigned sh) {
    return sh | 0x0c00u | ((sh + 1) << 16) | 0x0c000000u;
}

__device__ __forceinline__ unsigned lo16x2(int lo, int hi) {  // (lo & 0xffff) | (hi << 16) in one v_perm
    return __builtin_amdgcn_perm((unsigned)hi, (unsigned)lo, 0x05040100u);
}
// high halves packed: floor(lo / 2^16) | floor(hi / 2^16) << 16, one v_perm
__device__ __forceinline__ unsigned hi16x2(int lo, int hi) {
    return __builtin_amdgcn_perm((unsigned)hi, (unsigned)lo, 0x07060302u);
}
template <int CTRL, int ROW_MASK, bool BC>
__device__ __forceinline__ int dpp_add(int v) {
    return v + __builtin_amdgcn_update_dpp(0, v, CTRL, ROW_MASK, 0xf, BC);
}

// Exact wave sums of int32 values whose per-lane magnitude is below 2^31/8
// (true for b1, b2, A11, A12, A22: <= RPG * 2 * 8160 * 4080): the first three
// DPP steps (8-lane partial sums) run in int32, then each partial is split into
// 16-bit halves for the last three steps, all chains interleaved so that no
// DPP read waits on the write before it (no s_nop padding). The results are
// the FLT_SCALE'd floats: hi * 65536 is exact in float (|hi| < 2^24) and the one
// addition rounds the exact total once -- the same float as
// (float)(double)(int64 total), without the int64 / double detour.
__device__ __forceinline__ float halves_to_float(int hi_lane, int lo_lane) {
    const float h = (float)__builtin_amdgcn_readlane(hi_lane, 63);
    const float l = (float)__builtin_amdgcn_readlane(lo_lane, 63);
    return (h * 65536.f + l) * FLT_SCALE;
}

__device__ __forceinline__ void wave_sum_f2(int x, int y, float& fx, float& fy) {
    x = dpp_add<0xb1, 0xf, true>(x);
    y = dpp_add<0xb1, 0xf, true>(y);
    x = dpp_add<0x4e, 0xf, true>(x);
    y = dpp_add<0x4e, 0xf, true>(y);
    x = dpp_add<0x114, 0xf, true>(x);
    y = dpp_add<0x114, 0xf, true>(y);
    int xh = x >> 16, xl = x & 0xFFFF, yh = y >> 16, yl = y & 0xFFFF;
    xh = dpp_add<0x118, 0xf, true>(xh);
    xl = dpp_add<0x118, 0xf, true>(xl);
    yh = dpp_add<0x118, 0xf, true>(yh);
    yl = dpp_add<0x118, 0xf, true>(yl);
    xh = dpp_add<0x142, 0xa, false>(xh);
    xl = dpp_add<0x142, 0xa, false>(xl);
    yh = dpp_add<0x142, 0xa, false>(yh);
    yl = dpp_add<0x142, 0xa, false>(yl);
    xh = dpp_add<0x143, 0xc, false>(xh);
    xl = dpp_add<0x143, 0xc, false>(xl);
    yh = dpp_add<0x143, 0xc, false>(yh);
    yl = dpp_add<0x143, 0xc, false>(yl);
    fx = halves_to_float(xh, xl);
    fy = halves_to_float(yh, yl);
}

// three chains: the normal matrix (A11, A12, A22) in one pass
__device__ __forceinline__ void wave_sum_f3(int x, int y, int z, float& fx, float& fy, float& fz) {
    x = dpp_add<0xb1, 0xf, true>(x);
    y = dpp_add<0xb1, 0xf, true>(y);
    z = dpp_add<0xb1, 0xf, true>(z);
    x = dpp_add<0x4e, 0xf, true>(x);
    y = dpp_add<0x4e, 0xf, true>(y);
    z = dpp_add<0x4e, 0xf, true>(z);
    x = dpp_add<0x114, 0xf, true>(x);
    y = dpp_add<0x114, 0xf, true>(y);
    z = dpp_add<0x114, 0xf, true>(z);
    int xh = x >> 16, xl = x & 0xFFFF, yh = y >> 16, yl = y & 0xFFFF, zh = z >> 16, zl = z & 0xFFFF;
    xh = dpp_add<0x118, 0xf, true>(xh);
    xl = dpp_add<0x118, 0xf, true>(xl);
    yh = dpp_add<0x118, 0xf, true>(yh);
    yl = dpp_add<0x118, 0xf, true>(yl);
    zh = dpp_add<0x118, 0xf, true>(zh);
    zl = dpp_add<0x118, 0xf, true>(zl);
    xh = dpp_add<0x142, 0xa, false>(xh);
    xl = dpp_add<0x142, 0xa, false>(xl);
    yh = dpp_add<0x142, 0xa, false>(yh);
    yl = dpp_add<0x142, 0xa, false>(yl);
    zh = dpp_add<0x142, 0xa, false>(zh);
    zl = dpp_add<0x142, 0xa, false>(zl);
    xh = dpp_add<0x143, 0xc, false>(xh);
    xl = dpp_add<0x143, 0xc, false>(xl);
    yh = dpp_add<0x143, 0xc, false>(yh);
    yl = dpp_add<0x143, 0xc, false>(yl);
    zh = dpp_add<0x143, 0xc, false>(zh);
    zl = dpp_add<0x143, 0xc, false>(zl);
    fx = halves_to_float(xh, xl);
    fy = halves_to_float(yh, yl);
    fz = halves_to_float(zh, zl);
}

// v_dot2_i32_i16 in its VOP3P form with a register accumulator: the compiler
// otherwise picks v_dot2c (accumulator = destination) plus a v_mov of the
// rounding constant for every use.
__device__ __forceinline__ int sdot2_r(unsigned a, unsigned b, int c) {
    int d;
    asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}
__device__ __forceinline__ unsigned pk_sub16(unsigned a, unsigned b) {
    return __builtin_bit_cast(unsigned, __builtin_bit_cast(s16x2, a) - __builtin_bit_cast(s16x2, b));
}

// Stage rows [0, H) x pair entries [0, W) of the region whose pixel origin is
// (xa, y0), xa a multiple of 4: entry (r, e) = L(xa+e, y0+r) | L(xa+e+1, y0+r) << 16.
// REFLECT_101 outside the image (slow path, border windows only).
template <int W, int H>
__device__ __forceinline__ void stage_aligned(unsigned* dst, const ImgLevel& L, int xa, int y0, int lane) {
    constexpr int LPR = W / 4 + 1;   // lanes per row: W/4 dwords + the one holding the last pair's right pixel
    constexpr int RPP = 64 / LPR;    // rows per pass
    const int lr = lane / LPR, d = lane - lr * LPR;
    gu8 src = (gu8)L.data;
    const bool inside = xa >= 0 && y0 >= 0 && xa + W + 1 <= L.w && y0 + H <= L.h;
    if (inside) {
        // dword loads may run past the row end (never past the allocation: 256 B slack)
        gu32 q = (gu32)(src + (size_t)(y0 + lr) * L.pitch + xa) + d;
        const size_t step = (size_t)RPP * L.pitch / 4;
#pragma unroll
        for (int r = 0; r < H; r += RPP, q += step) {
            const bool act = lr < RPP && r + lr < H;
            const unsigned v = act ? q[0] : 0u;
            const unsigned nv = (unsigned)__builtin_amdgcn_ds_bpermute((lane + 1) << 2, (int)v);
            if (act && d < W / 4) {
                uint4 o;
                o.x = __builtin_amdgcn_perm(nv, v, 0x0c010c00u);
                o.y = __builtin_amdgcn_perm(nv, v, 0x0c020c01u);
                o.z = __builtin_amdgcn_perm(nv, v, 0x0c030c02u);
                o.w = __builtin_amdgcn_perm(nv, v, 0x0c040c03u);
                *reinterpret_cast<uint4*>(dst + (r + lr) * W + 4 * d) = o;
            }
        }
    } else {
        for (int k = lane; k < W * H; k += 64) {
            const int r = k / W, e = k - r * W;
            gu8 row = src + (size_t)refl101(y0 + r, L.h) * L.pitch;
            dst[k] = (unsigned)row[refl101(xa + e, L.w)] | ((unsigned)row[refl101(xa + e + 1, L.w)] << 16);
        }
    }
}

// Branch-free form of stage_aligned (no exec-mask branches, which cost ~5 SALU
// each): every lane loads a valid dword (rows past the region re-read the last
// row, so they carry the same bytes as that row's owner) and every lane writes:
// lanes without a complete set of pairs write to `sink`. A scheduling barrier
// per pass keeps the compiler from hoisting all loads (register pressure).
template <int W, int H>
__device__ __forceinline__ void stage_bf(unsigned* dst, unsigned* sink, const ImgLevel& L, int xa, int y0,
                                         int lane) {
    constexpr int LPR = W / 4 + 1, RPP = 64 / LPR, NP = (H + RPP - 1) / RPP;
    const int lr = lane / LPR, d = lane - lr * LPR;
    const bool inside = xa >= 0 && y0 >= 0 && xa + W + 1 <= L.w && y0 + H <= L.h;
    if (inside) {
        gu8 src = (gu8)L.data + xa + 4 * d;
        unsigned* dpl = (d < W / 4 && lr < RPP) ? dst + 4 * d : sink;
        const int dstride = (d < W / 4 && lr < RPP) ? W : 0;
#pragma unroll
        for (int q = 0; q < NP; q++) {
            int r = q * RPP + lr;
            r = r < H ? r : H - 1;
            const unsigned v = *(gu32)(src + (size_t)(y0 + r) * L.pitch);
            const unsigned nv = (unsigned)__builtin_amdgcn_ds_bpermute((lane + 1) << 2, (int)v);
            uint4 o;
            o.x = __builtin_amdgcn_perm(nv, v, 0x0c010c00u);
            o.y = __builtin_amdgcn_perm(nv, v, 0x0c020c01u);
            o.z = __builtin_amdgcn_perm(nv, v, 0x0c030c02u);
            o.w = __builtin_amdgcn_perm(nv, v, 0x0c040c03u);
            *reinterpret_cast<uint4*>(dpl + r * dstride) = o;
            __builtin_amdgcn_sched_barrier(0);
        }
    } else {
        gu8 src = (gu8)L.data;
        for (int k = lane; k < W * H; k += 64) {
            const int r = k / W, e = k - r * W;
            gu8 row = src + (size_t)refl101(y0 + r, L.h) * L.pitch;
            dst[k] = (unsigned)row[refl101(xa + e, L.w)] | ((unsigned)row[refl101(xa + e + 1, L.w)] << 16);
        }
    }
}

template <int WW, int WH, int MINW>
__global__ __launch_bounds__(256, MINW) void lk_fast_kernel(LKBatch B, LKDev p) {
    using S = Shape<WW, WH>;
    constexpr int RPG = S::RPG, NP = S::NP;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int seq = blockIdx.y;
    const int n = B.counts ? B.counts[seq] : B.n;
    // a wave per feature; a grid smaller than the count (LKBatch::grid_hint) loops
    for (int pt = blockIdx.x * 4 + wid; pt < n; pt += gridDim.x * 4) {
    const size_t base = (size_t)seq * B.cap;
    const float* __restrict__ prev_xy = B.prev_xy + 2 * base;
    float* __restrict__ next_xy = B.next_xy + 2 * base;
    // descriptors through the scalar cache (uniform per wave)
    const cpyr prev = (cpyr)B.prev + seq;
    const cpyr next = (cpyr)B.next + seq;
    const DerivDesc& dprev = B.dprev[seq];
    unsigned* ipair = reinterpret_cast<unsigned*>(lds + wid * S::WAVE_BYTES);
    unsigned* jreg = reinterpret_cast<unsigned*>(lds + wid * S::WAVE_BYTES + S::IBYTES);
    unsigned* sink = reinterpret_cast<unsigned*>(lds + wid * S::WAVE_BYTES + S::IBYTES + S::JBYTES);

    const int sc = lane % WW;
    const int sg = lane / WW;
    const bool strip = sg < S::G;
    // lanes outside the strip map (and rows past the window) run the same code on
    // in-range addresses; their derivatives are zeroed, so they add nothing
    const int r0 = (strip ? sg : 0) * RPG;
    const int rnd_i = 1 << (W_BITS - 6), rnd_d = 1 << (W_BITS + kDerShift - 1);

    constexpr float halfWx = (WW - 1) * 0.5f, halfWy = (WH - 1) * 0.5f;
    const float px = uni_f(prev_xy[2 * pt]), py = uni_f(prev_xy[2 * pt + 1]);
    float nx = 0.f, ny = 0.f;
    if (p.flags & SVO_LK_USE_INITIAL_FLOW) {
        nx = uni_f(next_xy[2 * pt]);
        ny = uni_f(next_xy[2 * pt + 1]);
    }
    int st = 1;
    float errv = 0.f;
    int itcount = 0;
    const int max_level = p.max_level;

    for (int level = max_level; level >= 0; level--) {
        const ImgLevel I{prev->lv[level].data, prev->lv[level].w, prev->lv[level].h, prev->lv[level].pitch};
        const ImgLevel J{next->lv[level].data, next->lv[level].w, next->lv[level].h, next->lv[level].pitch};
        const float lscale = __builtin_amdgcn_ldexpf(1.f, -level);  // == (float)(1. / (1 << level))
        float prevx = px * lscale, prevy = py * lscale;
        float nextx, nexty;
        if (level == max_level) {
            if (p.flags & SVO_LK_USE_INITIAL_FLOW) {
                nextx = nx * lscale;
                nexty = ny * lscale;
            } else {
                nextx = prevx;
                nexty = prevy;
            }
        } else {
            nextx = nx * 2.f;
            nexty = ny * 2.f;
        }
        nx = nextx;
        ny = nexty;
        prevx -= halfWx;
        prevy -= halfWy;
        const int ipx = uni_i(ufloor(prevx)), ipy = uni_i(ufloor(prevy));
        if (ipx < -WW || ipx >= I.w || ipy < -WH || ipy >= I.h) {
            if (level == 0) {
                st = 0;
                errv = 0.f;
            }
            continue;
        }
        float a = prevx - ipx, b = prevy - ipy;
        const int iw00 = uround((1.f - a) * (1.f - b) * (1 << W_BITS));
        const int iw01 = uround(a * (1.f - b) * (1 << W_BITS));
        const int iw10 = uround((1.f - a) * b * (1 << W_BITS));
        const int iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;
        const unsigned IW0 = pack16(iw00, iw01), IW1 = pack16(iw10, iw11);

        const int ixa = ipx & ~3;
        int jx0 = uni_i(ufloor(nextx - halfWx)) - JM, jy0 = uni_i(ufloor(nexty - halfWy)) - JM;
        int jxa = jx0 & ~3;
        // window (and its +1 bilinear row/column) inside the level: I pairs and
        // derivative pairs come straight from HBM; else REFLECT_101 staging / zeros
        const bool full_in = ipx >= 0 && ipy >= 0 && ipx + WW < I.w && ipy + WH < I.h;
        stage_bf<S::JRW, S::JRH>(jreg, sink, J, jxa, jy0, lane);
        unsigned P[RPG + 1];   // I(x, y) | I(x + 1, y) << 16 at the lane's column, rows r0 .. r0 + RPG
        u32x2a4 dv[RPG + 1];   // (Ix|Iy) at columns X, X+1 of each row: one dwordx2 load
        {
            const int dpitch = dprev.pitch[level];
            gu32 dsrc = (gu32)dprev.data[level];
            const int X = ipx + sc;
            if (full_in) {
                gu8 ib = (gu8)I.data + (size_t)(ipy + r0) * I.pitch + X;
                gu32 q = dsrc + (size_t)(ipy + r0) * dpitch + X;
#pragma unroll
                for (int k = 0; k <= RPG; k++) {
                    const int kk = (S::FULL || r0 + k <= WH) ? k : 0;  // stay inside the window
                    const unsigned v = *(gu16u)(ib + (size_t)kk * I.pitch);
                    P[k] = __builtin_amdgcn_perm(0u, v, 0x0c010c00u);
                    dv[k] = *(const __attribute__((address_space(1))) u32x2a4*)(q + (size_t)kk * dpitch);
                }
            } else {
                stage_bf<S::IPW, S::IPH>(ipair, sink, I, ixa, ipy, lane);
                const bool c0 = X >= 0 && X < I.w, c1 = X + 1 >= 0 && X + 1 < I.w;
#pragma unroll
                for (int k = 0; k <= RPG; k++) {
                    dv[k] = u32x2a4{0u, 0u};
                    const int Y = ipy + r0 + k;
                    if ((S::FULL || r0 + k <= WH) && Y >= 0 && Y < I.h) {
                        gu32 q = dsrc + (size_t)Y * dpitch + X;
                        if (c0) dv[k].x = q[0];
                        if (c1) dv[k].y = q[1];
                    }
                }
                wave_lds_sync();
                const unsigned* ip = ipair + r0 * S::IPW + (ipx - ixa) + sc;
#pragma unroll
                for (int k = 0; k <= RPG; k++) P[k] = ip[(S::FULL || r0 + k <= WH ? k : 0) * S::IPW];
            }
        }
        wave_lds_sync();

        // ---- I (x32), Ix, Iy at the lane's RPG window pixels, packed by row pairs ----
        // Lanes outside the strip map get zero derivative weights (their Ix, Iy
        // come out 0: rnd_d >> (W_BITS + kDerShift) == 0), so no branch per row.
        unsigned I2[NP], GX2[NP], GY2[NP];
        int a11 = 0, a12 = 0, a22 = 0;
        {
            const unsigned GW0 = strip ? IW0 : 0u, GW1 = strip ? IW1 : 0u;
            int iv[2 * NP], gx[2 * NP], gy[2 * NP];
#pragma unroll
            for (int j = 0; j < 2 * NP; j++) iv[j] = gx[j] = gy[j] = 0;
#pragma unroll
            for (int j = 0; j < RPG; j++) {
                iv[j] = sdot2(P[j], IW0, sdot2_r(P[j + 1], IW1, rnd_i)) >> (W_BITS - 5);
                const unsigned X0 = __builtin_amdgcn_perm(dv[j].y, dv[j].x, 0x05040100u);
                const unsigned X1 = __builtin_amdgcn_perm(dv[j + 1].y, dv[j + 1].x, 0x05040100u);
                const unsigned Y0 = __builtin_amdgcn_perm(dv[j].y, dv[j].x, 0x07060302u);
                const unsigned Y1 = __builtin_amdgcn_perm(dv[j + 1].y, dv[j + 1].x, 0x07060302u);
                const int gxr = sdot2(X0, GW0, sdot2_r(X1, GW1, rnd_d)) >> (W_BITS + kDerShift);
                const int gyr = sdot2(Y0, GW0, sdot2_r(Y1, GW1, rnd_d)) >> (W_BITS + kDerShift);
                if (S::FULL) {
                    gx[j] = gxr;
                    gy[j] = gyr;
                } else {
                    const int keep = -(int)(r0 + j < WH);
                    gx[j] = gxr & keep;
                    gy[j] = gyr & keep;
                }
            }
#pragma unroll
            for (int m = 0; m < NP; m++) {
                I2[m] = lo16x2(iv[2 * m], iv[2 * m + 1]);
                GX2[m] = lo16x2(gx[2 * m], gx[2 * m + 1]);
                GY2[m] = lo16x2(gy[2 * m], gy[2 * m + 1]);
                a11 = sdot2(GX2[m], GX2[m], a11);
                a12 = sdot2(GX2[m], GY2[m], a12);
                a22 = sdot2(GY2[m], GY2[m], a22);
            }
        }
        float A11, A12, A22;
        wave_sum_f3(a11, a12, a22, A11, A12, A22);

        float D = A11 * A22 - A12 * A12;
        float minEig = (A22 + A11 - sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) / (float)(2 * WW * WH);
        if (p.want_err && (p.flags & SVO_LK_GET_MIN_EIGENVALS)) errv = minEig;
        if (minEig < p.min_eig || D < FLT_EPSILON) {
            if (level == 0) st = 0;
            wave_lds_sync();
            continue;
        }
        D = 1.f / D;

        nextx -= halfWx;
        nexty -= halfWy;
        float pdx = 0.f, pdy = 0.f;
        // every top-left position of the staged region passes the image-bound test
        bool jsafe = jx0 >= -WW && jx0 + 2 * JM < J.w && jy0 >= -WH && jy0 + 2 * JM < J.h;
        for (int j = 0; j < p.max_count; j++) {
            const int inx = uni_i(ufloor(nextx)), iny = uni_i(ufloor(nexty));
            if (!(jsafe && (unsigned)(inx - jx0) <= 2u * JM && (unsigned)(iny - jy0) <= 2u * JM)) {
                if (inx < -WW || inx >= J.w || iny < -WH || iny >= J.h) {
                    if (level == 0) st = 0;
                    break;
                }
                if (inx < jx0 || inx > jx0 + 2 * JM || iny < jy0 || iny > jy0 + 2 * JM) {
                    jx0 = inx - JM;
                    jy0 = iny - JM;
                    jxa = jx0 & ~3;
                    jsafe = jx0 >= -WW && jx0 + 2 * JM < J.w && jy0 >= -WH && jy0 + 2 * JM < J.h;
                    wave_lds_sync();
                    stage_bf<S::JRW, S::JRH>(jreg, sink, J, jxa, jy0, lane);
                    wave_lds_sync();
                }
            }
            itcount++;
            a = nextx - inx;
            b = nexty - iny;
            const int w00 = uround((1.f - a) * (1.f - b) * (1 << W_BITS));
            const int w01 = uround(a * (1.f - b) * (1 << W_BITS));
            const int w10 = uround((1.f - a) * b * (1 << W_BITS));
            const int w11 = (1 << W_BITS) - w00 - w01 - w10;
            const unsigned W0 = pack16(w00, w01), W1 = pack16(w10, w11);
            int b1 = 0, b2 = 0;
            {
                const unsigned* jp = jreg + (iny - jy0 + r0) * S::JRW + (inx - jxa + sc);
                unsigned q[RPG + 1];
#pragma unroll
                for (int k = 0; k <= RPG; k++) q[k] = jp[k * S::JRW];
                int jv[2 * NP];
#pragma unroll
                for (int k = 0; k < 2 * NP; k++)
                    jv[k] = k < RPG ? sdot2(q[k], W0, sdot2_r(q[k + 1], W1, rnd_i)) >> (W_BITS - 5) : 0;
#pragma unroll
                for (int m = 0; m < NP; m++) {
                    const unsigned d2 = pk_sub16(lo16x2(jv[2 * m], jv[2 * m + 1]), I2[m]);
                    b1 = sdot2(d2, GX2[m], b1);
                    b2 = sdot2(d2, GY2[m], b2);
                }
            }
            float fb1, fb2;
            wave_sum_f2(b1, b2, fb1, fb2);
            const float dx = (A12 * fb2 - A22 * fb1) * D;
            const float dy = (A12 * fb1 - A11 * fb2) * D;
            nextx += dx;
            nexty += dy;
            nx = nextx + halfWx;
            ny = nexty + halfWy;
            if ((double)dx * dx + (double)dy * dy <= p.eps2) break;
            if (j > 0 && (double)fabsf(dx + pdx) < 0.01 && (double)fabsf(dy + pdy) < 0.01) {
                nx -= dx * 0.5f;
                ny -= dy * 0.5f;
                break;
            }
            pdx = dx;
            pdy = dy;
        }

        if (st && p.want_err && level == 0 && !(p.flags & SVO_LK_GET_MIN_EIGENVALS)) {
            const float npx = nx - halfWx, npy = ny - halfWy;
            const int ix0 = uni_i(ufloor(npx)), iy0 = uni_i(ufloor(npy));
            if (ix0 < -WW || ix0 >= J.w || iy0 < -WH || iy0 >= J.h) {
                st = 0;
                continue;
            }
            if (ix0 < jx0 || ix0 > jx0 + 2 * JM || iy0 < jy0 || iy0 > jy0 + 2 * JM) {
                jx0 = ix0 - JM;
                jy0 = iy0 - JM;
                jxa = jx0 & ~3;
                wave_lds_sync();
                stage_bf<S::JRW, S::JRH>(jreg, sink, J, jxa, jy0, lane);
                wave_lds_sync();
            }
            float aa = npx - ix0, bb = npy - iy0;
            const int w00 = uround((1.f - aa) * (1.f - bb) * (1 << W_BITS));
            const int w01 = uround(aa * (1.f - bb) * (1 << W_BITS));
            const int w10 = uround((1.f - aa) * bb * (1 << W_BITS));
            const int w11 = (1 << W_BITS) - w00 - w01 - w10;
            const unsigned W0 = pack16(w00, w01), W1 = pack16(w10, w11);
            int sad = 0;
            {
                const unsigned* jp = jreg + (iy0 - jy0 + r0) * S::JRW + (ix0 - jxa + sc);
#pragma unroll
                for (int k = 0; k < RPG; k++) {
                    const int jv = sdot2(jp[k * S::JRW], W0, sdot2_r(jp[(k + 1) * S::JRW], W1, rnd_i)) >>
                                   (W_BITS - 5);
                    const unsigned pr = I2[k >> 1];
                    const int iv = (k & 1) ? ((int)pr >> 16) : (int)(short)(pr & 0xFFFFu);
                    const int diff = jv - iv;
                    if (strip && (S::FULL || r0 + k < WH)) sad += diff < 0 ? -diff : diff;
                }
            }
            errv = (float)wave_sum_exact(sad) * 1.f / (float)(32 * WW * WH);
        }
        wave_lds_sync();
    }
    if (lane == 0) {
        next_xy[2 * pt] = nx;
        next_xy[2 * pt + 1] = ny;
        B.status[base + pt] = (uint8_t)st;
        if (B.err) B.err[base + pt] = errv;
        if (B.iters) B.iters[base + pt] = itcount;
    }
    }  // features of this wave
}

// ---------------------------------------------------------------------------
// Helpers of the four-features-per-wave kernel (lk_multi_kernel below).
template <int CTRL>
__device__ __forceinline__ int dpp_row_add(int v) {
    // quad_perm / row_ror read a valid lane for every lane: bound_ctrl lets the
    // compiler fold the move into one v_add_u32_dpp (no zero-initialised old value)
    return v + __builtin_amdgcn_update_dpp(0, v, CTRL, 0xf, 0xf, true);
}
__device__ __forceinline__ int swz16_add(int v) {  // + lane ^ 16 (within 32-lane groups)
    return v + __builtin_amdgcn_ds_swizzle(v, 0x401f);
}
// float of the exact h * 2^16 + l (one rounding: the product is exact), NOT scaled by
// FLT_SCALE -- the callers apply it (A) or fold it into 1 / det (b)
__device__ __forceinline__ float halves_lane_float(int h, int l) { return __builtin_fmaf((float)h, 65536.f, (float)l); }

// OpenCV's rounded bilinear weights (LKTrackerInvoker: iw00 = cvRound((1 - a)(1 - b)
// 2^14), iw01, iw10, iw11 = 2^14 - the others), packed for v_dot2 as (w00 | w01 << 16,
// w10 | w11 << 16). cvRound(p 2^14) for a float product p in [0, 1] is computed as
// p + 768: that sum lies in [768, 1024), where the float grid is 2^-14, so the
// addition rounds p to a multiple of 2^-14 with ties to even -- rint's rounding --
// and the low mantissa bits then hold round(p 2^14) (768.f = 0x44400000 has zero
// low bits). Fast-rate adds in place of rndne + cvt (both half-rate on gfx950).
__device__ __forceinline__ unsigned wbits(float p) { return __float_as_uint(p + 768.f); }
struct BiW {
    unsigned W0, W1;
};
__device__ __forceinline__ BiW bilinear_weights(float a, float b) {
    const float ia = 1.f - a, ib = 1.f - b;
    const unsigned b00 = wbits(ia * ib), b01 = wbits(a * ib), b10 = wbits(ia * b);
    // 2^14 - w00 - w01 - w10 with w = bits - 0x44400000, modulo 2^32 (w11 may be -1)
    const unsigned w11 = (1u << W_BITS) + 3u * 0x44400000u - b00 - b01 - b10;
    return {__builtin_amdgcn_perm(b01, b00, 0x05040100u), __builtin_amdgcn_perm(w11, b10, 0x05040100u)};
}

// NR rows of one strip: I (x32) / Ix / Iy at the strip's pixels packed by row pairs
// (NR / 2 pairs), accumulated into the A sums and into per-lane c1 += I.Ix,
// c2 += I.Iy (sum (J - I) G = sum J G - sum I G exactly -- int32 wrap-around
// arithmetic, the per-lane total is the same bounded value -- so an iteration starts
// its b sums at (-c1, -c2) and needs no J - I subtraction). An odd NR leaves a last
// row: with ODD = false it is closed by a zero row (one more pair, half empty); with
// ODD = true its raw sums are returned (li, lx, ly) for odd_pair_setup, which pairs
// the last rows of two strips.
__device__ __forceinline__ void pair_setup(unsigned I2, unsigned GXm, unsigned GYm, int& a11, int& a12, int& a22,
                                           int& c1, int& c2) {
    a11 = sdot2(GXm, GXm, a11);
    a12 = sdot2(GXm, GYm, a12);
    a22 = sdot2(GYm, GYm, a22);
    c1 = sdot2(I2, GXm, c1);
    c2 = sdot2(I2, GYm, c2);
}
template <int NR, bool ODD>
__device__ __forceinline__ void strip_setup_c(const unsigned* P, const u32x2a4* D, unsigned IW0, unsigned IW1,
                                              unsigned GW0, unsigned GW1, unsigned* GX, unsigned* GY, int& a11,
                                              int& a12, int& a22, int& c1, int& c2, int& li, int& lx, int& ly) {
    constexpr int NP = ODD ? NR / 2 : (NR + 1) / 2;
    const int rnd_i = 1 << (W_BITS - 6), rnd_d = 1 << (W_BITS + kDerShift - 1);
    int iv[NR + 1], gx[NR + 1], gy[NR + 1];
    iv[NR] = gx[NR] = gy[NR] = 0;
#pragma unroll
    for (int j = 0; j < NR; j++) {
        iv[j] = sdot2(P[j], IW0, sdot2_r(P[j + 1], IW1, rnd_i)) >> (W_BITS - 5);
        const unsigned X0 = __builtin_amdgcn_perm(D[j].y, D[j].x, 0x05040100u);
        const unsigned X1 = __builtin_amdgcn_perm(D[j + 1].y, D[j + 1].x, 0x05040100u);
        const unsigned Y0 = __builtin_amdgcn_perm(D[j].y, D[j].x, 0x07060302u);
        const unsigned Y1 = __builtin_amdgcn_perm(D[j + 1].y, D[j + 1].x, 0x07060302u);
        gx[j] = sdot2(X0, GW0, sdot2_r(X1, GW1, rnd_d));  // CV_DESCALE(., W_BITS) in bits 16..31
        gy[j] = sdot2(Y0, GW0, sdot2_r(Y1, GW1, rnd_d));
    }
    static_assert(W_BITS + kDerShift == 16, "derivative sums must carry their descaled value in bits 16..31");
#pragma unroll
    for (int m = 0; m < NP; m++) {
        GX[m] = hi16x2(gx[2 * m], gx[2 * m + 1]);
        GY[m] = hi16x2(gy[2 * m], gy[2 * m + 1]);
        pair_setup(lo16x2(iv[2 * m], iv[2 * m + 1]), GX[m], GY[m], a11, a12, a22, c1, c2);
    }
    if constexpr (ODD) {
        li = iv[NR - 1];
        lx = gx[NR - 1];
        ly = gy[NR - 1];
    }
}
// the last rows of strips k (i0 ..) and k + 1 (i1 ..) as one pair
__device__ __forceinline__ void odd_pair_setup(int i0, int x0, int y0, int i1, int x1, int y1, unsigned& GXm,
                                               unsigned& GYm, int& a11, int& a12, int& a22, int& c1, int& c2) {
    GXm = hi16x2(x0, x1);
    GYm = hi16x2(y0, y1);
    pair_setup(lo16x2(i0, i1), GXm, GYm, a11, a12, a22, c1, c2);
}

// Staging geometry of a JRW x JRH pair region (JRW = 2 mod 4): each lane loads one
// aligned dword of a row (LPR dwords cover the JRW + 1 pixels of a row, RPP rows
// per pass) and writes the four pixel pairs it starts -- entries 4d .. 4d + 3, each
// pixel scaled by 2^kJShift (<= 32640, int16) so that a bilinear J sum carries
// CV_DESCALE(., W_BITS - 5) in its high 16 bits, packed by one permute -- as two
// 8-byte stores (rows are JRW dwords apart: 8- but not 16-byte aligned). The pairs
// take the next lane's dword for their right pixels (ds_bpermute). No store is
// masked and nothing goes to a sink:
//  * a row's last lane (d = LPR - 1) starts only entries JRW - 2, JRW - 1, from its
//    own dword: its second store repeats its first (same address, same data --
//    per-lane permute selectors and address);
//  * lanes past the RPP x LPR slots, and rows past the region in the last pass,
//    repeat a real slot (row RPP - 1, or row JRH - 1): same load, same neighbour
//    (the bpermute source is the real slot's neighbour), same store.
constexpr int kJShift = 7;
static_assert(W_BITS - 5 + kJShift == 16, "J sums must carry their descaled value in bits 16..31");

template <int JRW, int JRH>
struct StageGeom {
    static_assert(JRW % 4 == 2, "rows of 4k + 2 entries: the last lane starts two");
    static constexpr int LPR = (JRW + 2) / 4, RPP = 64 / LPR, NPS = (JRH + RPP - 1) / RPP;
    int lr, d;            // the slot this lane loads and writes (lanes past the slots repeat row RPP - 1)
    int src;              // ds_bpermute byte address of the slot's neighbour
    unsigned selx, sely;  // permute selectors of the second store's pairs (high bytes)
    int hi;               // dword offset of the second store from the first (2, or 0 for the last lane)
    __device__ __forceinline__ explicit StageGeom(int lane) {
        const int l0 = lane / LPR;
        lr = l0 < RPP ? l0 : RPP - 1;
        d = lane - l0 * LPR;
        src = (lr * LPR + d + 1) << 2;
        const bool last = d == LPR - 1;
        selx = last ? 0x010c000cu : 0x030c020cu;  // pixel pairs in the halves' high bytes
        sely = last ? 0x020c010cu : 0x040c030cu;
        hi = last ? 0 : 2;
    }
    __device__ __forceinline__ int row(int q) const {
        const int r = q * RPP + lr;
        return r < JRH ? r : JRH - 1;
    }
    // entries of pass q's row into the region (its row r = row(q))
    __device__ __forceinline__ void write(unsigned* region, int r, unsigned v) const {
        const unsigned nv = (unsigned)__builtin_amdgcn_ds_bpermute(src, (int)v);
        unsigned* p = region + r * JRW + 4 * d;
        uint2 a, b;
        // each pixel permuted into the high byte of its half (x 256), then one logical
        // right shift to x 2^kJShift: a fast-rate shift (v_lshrrev; v_lshlrev issues at
        // the slow rate on gfx950, profiles/r05/a_valu_rates.txt)
        constexpr int R = 8 - kJShift;
        a.x = __builtin_amdgcn_perm(nv, v, 0x010c000cu) >> R;
        a.y = __builtin_amdgcn_perm(nv, v, 0x020c010cu) >> R;
        b.x = __builtin_amdgcn_perm(nv, v, selx) >> R;
        b.y = __builtin_amdgcn_perm(nv, v, sely) >> R;
        *reinterpret_cast<uint2*>(p) = a;
        *reinterpret_cast<uint2*>(p + hi) = b;
    }
};

// The staged region (pixel columns xa .. xa + 4 LPR - 1 read as dwords, rows
// y0 .. y0 + JRH - 1) lies inside the padded level.
template <int JRW, int JRH>
__device__ __forceinline__ bool region_in_pad(const ImgLevel& L, int xa, int y0) {
    return xa >= -kPyrPad && y0 >= -kPyrPad && xa + 4 * StageGeom<JRW, JRH>::LPR <= L.w + kPyrPad &&
           y0 + JRH <= L.h + kPyrPad;
}

// one group's region re-staged at (xa, y0) (inside the padding)
template <int W, int H>
__device__ __forceinline__ void stage_padded(unsigned* dst, const ImgLevel& L, int xa, int y0,
                                             const StageGeom<W, H>& g) {
    using G = StageGeom<W, H>;
    const gu8 base = pad_origin(L.data, L.pitch, kPyrPad, 1);
    const unsigned o0 = (unsigned)(xa + kPyrPad + 4 * g.d) + (unsigned)(y0 + kPyrPad) * (unsigned)L.pitch;
    unsigned v[G::NPS];
#pragma unroll
    for (int q = 0; q < G::NPS; q++) v[q] = ldg_off<unsigned>(base, o0 + (unsigned)g.row(q) * (unsigned)L.pitch);
#pragma unroll
    for (int q = 0; q < G::NPS; q++) g.write(dst, g.row(q), v[q]);
}

// ---------------------------------------------------------------------------
// FPW features per wave (WW x WH windows, WH a multiple of the strip height NR):
// each group of LPF = 64 / FPW lanes owns one feature; the window's WW x WH / NR
// vertical NR-row strips (21 x 21: 63 strips of 7 rows, 21 columns x 3 row groups;
// 11 x 11: 11 strips of 11 rows) are dealt to the group's lanes, lane l taking
// strips l, l + LPF, ... (slots past the last strip carry zero weights). The per-feature work every
// lane repeats (bilinear weights, bounds / convergence tests, the 2x2 solve) and
// the exact group reduction serve FPW features per instruction. Staged next-
// image regions (margin QJM) for all FPW features share the wave's LDS slice.
// Same exact integer sums and float solve as every other LK kernel.
// Staged region of one group: JRW pair entries x JRH rows. Entry e of row r is the
// pixel pair (x0 + e, x0 + e + 1) with x0 = jx0 & ~3 (the staging reads aligned
// dwords), so an estimate inside the +-QJM margin reads entries up to
// 3 + 2 QJM + WW - 1 and its pair partner: JRW = WW + 2 QJM + 3 entries, not rounded
// up to a multiple of 4 (21 x 21: 26 x 24 entries, 2,496 B; rounding up to 28 cost
// 192 B per group and, with the groups' padding, a wave per CU: 4 x 2,752 B held LK
// at 14 waves per CU, 4 x 2,496 B + the sink admits 16).
// JSTRIDE: the groups' regions lie JSTRIDE bytes apart, the smallest dword count >=
// the region with (dwords mod 32) = 16. ds_read_b32 / ds_read2_b32 bank by (dword
// address) mod 32 over each 32-lane half -- two groups, reading the same strip
// pattern at the same offsets of their own regions: at a multiple of 32 dwords
// apart every read of the pair collided (2-way), 16 banks apart they take disjoint
// halves.
template <int QJM, int WW = 21, int WH = 21, int FPW = 4>
struct MultiShape {
    static_assert(FPW == 4, "four 16-lane groups per wave");
    static constexpr int JRW0 = WW + 2 * QJM + 3;                  // entries the margin needs
    static constexpr int JRW = JRW0 + (6 - JRW0 % 4) % 4;          // rounded up to 4k + 2
    static constexpr int JRH = WH + 1 + 2 * QJM;
    static constexpr int JBYTES = JRW * JRH * 4;
    static constexpr int RES = 16;
    static constexpr int JSTRIDE = (JBYTES / 4 + ((RES - JBYTES / 4) % 32 + 32) % 32) * 4;
    static_assert(JSTRIDE >= JBYTES && (JSTRIDE / 4) % 32 == RES && JSTRIDE - JBYTES < 128, "group stride");
    static_assert(JRW % 4 == 2 && JRW >= JRW0 && JRW < JRW0 + 4, "entries 4k + 2");
};

// Exact sums over the LPF lanes of each group (every lane receives its group's
// total), as floats of the exact integers (one rounding): int32 DPP steps while
// the partial sums provably fit (STEPS32), then 16-bit halves.
template <int LPF, int STEPS32>
__device__ __forceinline__ int group_add_step(int v, int step) {
    switch (step) {
        case 0: return dpp_row_add<0xb1>(v);   // quad_perm 1,0,3,2
        case 1: return dpp_row_add<0x4e>(v);   // quad_perm 2,3,0,1
        case 2: return dpp_row_add<0x124>(v);  // row_ror:4
        case 3: return dpp_row_add<0x128>(v);  // row_ror:8
        default: return swz16_add(v);          // lane ^ 16
    }
}
template <int LPF, int STEPS32, int NV>
__device__ __forceinline__ void group_sum_f(int (&v)[NV], float (&f)[NV]) {
    constexpr int STEPS = LPF == 16 ? 4 : 5;
    static_assert(LPF == 16 || LPF == 32, "groups of 16 or 32 lanes");
#pragma unroll
    for (int s = 0; s < STEPS32; s++)
#pragma unroll
        for (int i = 0; i < NV; i++) v[i] = group_add_step<LPF, STEPS32>(v[i], s);
    int h[NV], lo[NV];
#pragma unroll
    for (int i = 0; i < NV; i++) {
        h[i] = v[i] >> 16;
        lo[i] = v[i] & 0xFFFF;
    }
#pragma unroll
    for (int s = STEPS32; s < STEPS; s++)
#pragma unroll
        for (int i = 0; i < NV; i++) {
            h[i] = group_add_step<LPF, STEPS32>(h[i], s);
            lo[i] = group_add_step<LPF, STEPS32>(lo[i], s);
        }
#pragma unroll
    for (int i = 0; i < NV; i++) f[i] = halves_lane_float(h[i], lo[i]);
}
// the same group reduction stopped before the float: every lane receives its group's
// exact total as 16-bit-half sums (h, lo), total = h 2^16 + lo
template <int LPF, int STEPS32>
__device__ __forceinline__ void group_halves(int v, int& h, int& lo) {
    constexpr int STEPS = LPF == 16 ? 4 : 5;
#pragma unroll
    for (int s = 0; s < STEPS32; s++) v = group_add_step<LPF, STEPS32>(v, s);
    h = v >> 16;
    lo = v & 0xFFFF;
#pragma unroll
    for (int s = STEPS32; s < STEPS; s++) {
        h = group_add_step<LPF, STEPS32>(h, s);
        lo = group_add_step<LPF, STEPS32>(lo, s);
    }
}
// exact 64-lane totals of two int32 partials (|v| < 2^31 / 8 per lane) as half sums in
// scalars: three int32 DPP steps (8-lane partials), then the halves (wave_sum_f2's steps)
__device__ __forceinline__ void wave_halves2(int x, int y, int& xh, int& xl, int& yh, int& yl) {
    x = dpp_add<0xb1, 0xf, true>(x);
    y = dpp_add<0xb1, 0xf, true>(y);
    x = dpp_add<0x4e, 0xf, true>(x);
    y = dpp_add<0x4e, 0xf, true>(y);
    x = dpp_add<0x114, 0xf, true>(x);
    y = dpp_add<0x114, 0xf, true>(y);
    int ah = x >> 16, al = x & 0xFFFF, bh = y >> 16, bl = y & 0xFFFF;
    ah = dpp_add<0x118, 0xf, true>(ah);
    al = dpp_add<0x118, 0xf, true>(al);
    bh = dpp_add<0x118, 0xf, true>(bh);
    bl = dpp_add<0x118, 0xf, true>(bl);
    ah = dpp_add<0x142, 0xa, false>(ah);
    al = dpp_add<0x142, 0xa, false>(al);
    bh = dpp_add<0x142, 0xa, false>(bh);
    bl = dpp_add<0x142, 0xa, false>(bl);
    ah = dpp_add<0x143, 0xc, false>(ah);
    al = dpp_add<0x143, 0xc, false>(al);
    bh = dpp_add<0x143, 0xc, false>(bh);
    bl = dpp_add<0x143, 0xc, false>(bl);
    xh = __builtin_amdgcn_readlane(ah, 63);
    xl = __builtin_amdgcn_readlane(al, 63);
    yh = __builtin_amdgcn_readlane(bh, 63);
    yl = __builtin_amdgcn_readlane(bl, 63);
}
__device__ __forceinline__ float rl_f(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

// LOOP (the stereo call): the grid covers LKBatch::grid_hint features per sequence
// (the expected count) and a block whose sequence holds more takes the tiles
// gridDim.x, 2 gridDim.x, ... further on; without it (the temporal call) a block
// owns one tile and blocks past a sequence's count return at once. The stereo
// call's bound is the feature budget (~2,100 per sequence) while the speculative
// count is ~100: sized to the bound, 131k of its 134k waves per launch only read a
// count and exited, dispatched beside LK.
template <int FPW, int QJM, int MINW, int KKS = 2, int WW = 21, int WH = 21, int NR = 7, bool LOOP = false>
__global__ __launch_bounds__(64, MINW) void lk_multi_kernel(LKBatch B, LKDev p) {
    using Q = MultiShape<QJM, WW, WH, FPW>;
    static_assert(WH % NR == 0, "whole strips");
    static_assert(WW + QJM + 3 <= kPyrPad && WW + 1 <= kDerPad, "padding too small for the window");
    constexpr int JRW = Q::JRW, JRH = Q::JRH;
    constexpr int NSTRIP = WW * (WH / NR);
    constexpr int LPF = 64 / FPW;                 // lanes per feature
    constexpr int K = (NSTRIP + LPF - 1) / LPF;   // strips per lane
    // an odd strip height pairs the last rows of strips 2i and 2i + 1 (ODD; K even),
    // otherwise the last row is closed by a zero row
    constexpr bool ODD = NR % 2 == 1 && K % 2 == 0;
    constexpr int NP = ODD ? NR / 2 : (NR + 1) / 2;  // full row pairs per strip
    constexpr int NO = ODD ? K / 2 : 1;              // odd-row pairs per lane
    // int32 partial sums: a lane holds <= NR K products |diff * g| <= 8160 * 4080
    // (A sums: 4080^2); steps while 2^steps * NR K * 8160 * 4080 < 2^31
    constexpr long long kProd = (long long)NR * K * 8160 * 4080;
    constexpr int STEPS32 = 4 * kProd < (1ll << 31) ? 2 : 2 * kProd < (1ll << 31) ? 1 : 0;
    static_assert(kProd < (1ll << 31), "a lane's partial sums must fit int32");
    // the single-group tail (below): the 21 x 21 temporal shape, four strips per lane
    constexpr bool TAIL = !LOOP && FPW == 4 && K == 4 && ODD && NP == 3 && NO == 2;
    // a tail lane's b partial: NP full row pairs + one odd pair, 8160 * 4080 each
    static_assert(!TAIL || 8ll * (2 * NP + 2) * 8160 * 4080 < (1ll << 31), "tail partials: 3 int32 DPP steps");
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int lane = threadIdx.x & 63;
    const int g = lane / LPF, l = lane % LPF;
    // in XCD order the blocks one XCD runs are consecutive features of one sequence
    // (neighbouring windows: shared L2 lines) instead of every 8th block
    const XcdTile tile = p.xcd ? xcd_tile() : XcdTile{(int)blockIdx.x, (int)blockIdx.y, 0};
    const int seq = tile.y;
    const int n = B.counts ? B.counts[seq] : B.n;
    int tx = tile.x;
next_tile:  // (LOOP: the block's next tile, gridDim.x further on)
    const int pt0 = tx * FPW;
    if (pt0 >= n) return;
    const int pt = pt0 + g;
    const bool live = pt < n;
    const int ptc = live ? pt : n - 1;  // an idle group shadows a real feature, writes nothing
    const size_t base = (size_t)seq * B.cap;
    const float* __restrict__ prev_xy = B.prev_xy + 2 * base;
    float* __restrict__ next_xy = B.next_xy + 2 * base;
    const cpyr prev = (cpyr)B.prev + seq;
    const cpyr next = (cpyr)B.next + seq;
    const DerivDesc& dprev = B.dprev[seq];
    unsigned* jregs = reinterpret_cast<unsigned*>(lds);
    const unsigned* jmine = jregs + g * (Q::JSTRIDE / 4);
    const StageGeom<JRW, JRH> sg(lane);

    // the lane's strips: column, first row, LDS offset; slots past NSTRIP are dummies
    int scol[K], srow[K];
    bool sreal[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
        const int sidx = l + LPF * k;
        sreal[k] = sidx < NSTRIP;
        const int sc = sreal[k] ? sidx : 0;
        scol[k] = sc % WW;
        srow[k] = (sc / WW) * NR;
    }
    constexpr float halfWx = (WW - 1) * 0.5f, halfWy = (WH - 1) * 0.5f;
    const int rnd_j = 1 << (W_BITS - 6 + kJShift);

    const float px = prev_xy[2 * ptc], py = prev_xy[2 * ptc + 1];
    float nx = 0.f, ny = 0.f;
    if (p.flags & SVO_LK_USE_INITIAL_FLOW) {
        nx = next_xy[2 * ptc];
        ny = next_xy[2 * ptc + 1];
    }
    int st = live ? 1 : 0;
    float errv = 0.f;
    // iterations per feature, counted from the active-lane ballot: wave-uniform, so
    // scalar registers (a per-lane counter is the first VGPR spilled under MINW = 4)
    int itc[FPW];
#pragma unroll
    for (int f = 0; f < FPW; f++) itc[f] = 0;
    const int max_level = p.max_level;

    for (int level = max_level; level >= 0; level--) {
        const ImgLevel I{prev->lv[level].data, prev->lv[level].w, prev->lv[level].h, prev->lv[level].pitch};
        const ImgLevel J{next->lv[level].data, next->lv[level].w, next->lv[level].h, next->lv[level].pitch};
        const float lscale = __builtin_amdgcn_ldexpf(1.f, -level);
        float prevx = px * lscale, prevy = py * lscale;
        float nextx, nexty;
        if (level == max_level) {
            if (p.flags & SVO_LK_USE_INITIAL_FLOW) {
                nextx = nx * lscale;
                nexty = ny * lscale;
            } else {
                nextx = prevx;
                nexty = prevy;
            }
        } else {
            nextx = nx * 2.f;
            nexty = ny * 2.f;
        }
        nx = nextx;
        ny = nexty;
        prevx -= halfWx;
        prevy -= halfWy;
        const float fpx = __builtin_floorf(prevx), fpy = __builtin_floorf(prevy);
        const int ipx = (int)fpx, ipy = (int)fpy;
        // ipx < -WW || ipx >= I.w || ipy < -WH || ipy >= I.h, one unsigned compare per axis
        const bool inb = (unsigned)(ipx + WW) < (unsigned)(I.w + WW) && (unsigned)(ipy + WH) < (unsigned)(I.h + WH);
        if (!inb && level == 0 && live) {
            st = 0;
            errv = 0.f;
        }
        bool lact = live && inb;
        // a = prevPt.x - iprevPt.x: the float of the floor is the floor (|x| < 2^24)
        const BiW iw = bilinear_weights(prevx - fpx, prevy - fpy);
        const unsigned IW0 = iw.W0, IW1 = iw.W1;

        int jx0 = ufloor(nextx - halfWx) - QJM, jy0 = ufloor(nexty - halfWy) - QJM;
        int jxa = jx0 & ~3;
        int jbase = jy0 * JRW + jxa;  // the region origin as an entry offset (iny * JRW + inx - jbase)
        unsigned GX[K][NP], GY[K][NP], GXO[NO], GYO[NO];
        int li[K], lx[K], ly[K];  // (ODD) the strips' last rows until paired
        int asum[3] = {0, 0, 0};
        int csum[2] = {0, 0};  // sum I.Ix, I.Iy over the lane's strips
        {
            // branch-free reads (padded levels); an inactive group (or one whose
            // region lies beyond the padding: its first bounds test deactivates
            // it) stages and reads at the level origin, results unused
            using SL = StageGeom<JRW, JRH>;
            int xs[FPW], ys[FPW];
#pragma unroll
            for (int f = 0; f < FPW; f++) {
                const int xa = __builtin_amdgcn_readlane(jxa, LPF * f), y0 = __builtin_amdgcn_readlane(jy0, LPF * f);
                const bool ok = __builtin_amdgcn_readlane((int)lact, LPF * f) && region_in_pad<JRW, JRH>(J, xa, y0);
                xs[f] = ok ? xa : 0;
                ys[f] = ok ? y0 : 0;
            }
            unsigned sv[FPW][SL::NPS];
            // wave-uniform row bases (scalar adds) + one per-lane offset for every
            // feature: 4d + (the lane's pass-0 row) * pitch; the last pass's rows are
            // clamped to the region (per lane)
            const gu8 jbase = pad_origin(J.data, J.pitch, kPyrPad, 1) + (size_t)kPyrPad * (J.pitch + 1);
            const unsigned ol = 4u * (unsigned)sg.d + (unsigned)sg.row(0) * (unsigned)J.pitch;
            const unsigned olast = 4u * (unsigned)sg.d + (unsigned)sg.row(SL::NPS - 1) * (unsigned)J.pitch;
#pragma unroll
            for (int f = 0; f < FPW; f++) {
                const gu8 fb = jbase + xs[f] + (ptrdiff_t)ys[f] * J.pitch;
#pragma unroll
                for (int q = 0; q < SL::NPS; q++)
                    sv[f][q] = q + 1 < SL::NPS ? ldg_off<unsigned>(fb + (size_t)q * SL::RPP * J.pitch, ol)
                                               : ldg_off<unsigned>(fb, olast);
            }
            const int dpitch = dprev.pitch[level];
            const gu8 ibase = pad_origin(I.data, I.pitch, kPyrPad, 1);
            const gu8 dbase = pad_origin((const uint8_t*)dprev.data[level], dpitch, kDerPad, 4);
            const int sx = inb ? ipx : 0, sy = inb ? ipy : 0;
            const auto load_strip = [&](int k, unsigned* P, u32x2a4* Dv) {
                // per-lane offsets of the strip's first row; the rows by wave-uniform bases
                const int x = sx + scol[k], y = sy + srow[k];
                const unsigned oi = (unsigned)(x + kPyrPad) + (unsigned)(y + kPyrPad) * (unsigned)I.pitch;
                const unsigned od = 4u * ((unsigned)(x + kDerPad) + (unsigned)(y + kDerPad) * (unsigned)dpitch);
#pragma unroll
                for (int r = 0; r <= NR; r++) {
                    P[r] = __builtin_amdgcn_perm(0u, (unsigned)ldg_off<u16a1>(ibase + (size_t)r * I.pitch, oi),
                                                 0x0c010c00u);
                    Dv[r] = ldg_off<u32x2a4>(dbase + (size_t)r * 4 * dpitch, od);
                }
            };
            const auto write_staging = [&] {
#pragma unroll
                for (int f = 0; f < FPW; f++)
#pragma unroll
                    for (int q = 0; q < SL::NPS; q++) sg.write(jregs + f * (Q::JSTRIDE / 4), sg.row(q), sv[f][q]);
            };
            // strips KKS at a time: loads of a group in flight together
            static_assert(KKS >= 1, "strips loaded per setup group");
#pragma unroll
            for (int k0 = 0; k0 < K; k0 += KKS) {
                constexpr int KK = K >= KKS ? KKS : 1;
                unsigned P[KK][NR + 1];
                u32x2a4 Dv[KK][NR + 1];
#pragma unroll
                for (int kk = 0; kk < KK; kk++) load_strip(k0 + kk, P[kk], Dv[kk]);
                if (k0 == 0) write_staging();
#pragma unroll
                for (int kk = 0; kk < KK; kk++) {
                    const int k = k0 + kk;
                    strip_setup_c<NR, ODD>(P[kk], Dv[kk], IW0, IW1, sreal[k] ? IW0 : 0u, sreal[k] ? IW1 : 0u, GX[k],
                                           GY[k], asum[0], asum[1], asum[2], csum[0], csum[1], li[k], lx[k], ly[k]);
                    if (ODD && (k & 1))
                        odd_pair_setup(li[k - 1], lx[k - 1], ly[k - 1], li[k], lx[k], ly[k], GXO[k / 2], GYO[k / 2],
                                       asum[0], asum[1], asum[2], csum[0], csum[1]);
                }
            }
        }
        wave_lds_sync();
        float A[3];
        group_sum_f<LPF, STEPS32>(asum, A);
        const float A11 = A[0] * FLT_SCALE, A12 = A[1] * FLT_SCALE, A22 = A[2] * FLT_SCALE;

        float D = A11 * A22 - A12 * A12;
        const float minEig =
            (A22 + A11 - sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) / (float)(2 * WW * WH);
        if (lact && p.want_err && (p.flags & SVO_LK_GET_MIN_EIGENVALS)) errv = minEig;
        if (lact && (minEig < p.min_eig || D < FLT_EPSILON)) {
            if (level == 0) st = 0;
            lact = false;
        }
        D = 1.f / D;
        // the b sums arrive unscaled: (A12 b2 s - A22 b1 s) D == (A12 b2 - A22 b1) (s D)
        // exactly for s = FLT_SCALE (a power of two commutes with every rounding here)
        const float Ds = D * FLT_SCALE;

        nextx -= halfWx;
        nexty -= halfWy;
        float pdx = 0.f, pdy = 0.f;
        int tail_j = -1;
        for (int j = 0; j < p.max_count; j++) {
            const unsigned long long act0 = __builtin_amdgcn_ballot_w64(lact);
            if (act0 == 0) break;
            if constexpr (TAIL) {
                // one feature left: its iterations go to all 64 lanes (below)
                const unsigned long long gm = act0 & 0x0001000100010001ull;
                if (p.tail && (gm & (gm - 1)) == 0) {
                    tail_j = j;
                    break;
                }
            }
            const float fnx = __builtin_floorf(nextx), fny = __builtin_floorf(nexty);
            const int inx = (int)fnx, iny = (int)fny;
            if (lact && !((unsigned)(inx + WW) < (unsigned)(J.w + WW) && (unsigned)(iny + WH) < (unsigned)(J.h + WH))) {
                if (level == 0) st = 0;
                lact = false;
            }
            const bool need = lact && ((unsigned)(inx - jx0) > 2u * QJM || (unsigned)(iny - jy0) > 2u * QJM);
            unsigned long long nb = __builtin_amdgcn_ballot_w64(need && l == 0);
            if (nb) {  // (rare: the region's origin moves only inside this branch)
                if (need) {
                    jx0 = inx - QJM;
                    jy0 = iny - QJM;
                    jxa = jx0 & ~3;
                    jbase = jy0 * JRW + jxa;
                }
                wave_lds_sync();
                while (nb) {
                    const int f = (int)(__builtin_ctzll(nb) / LPF);
                    nb &= nb - 1;
                    stage_padded<JRW, JRH>(jregs + f * (Q::JSTRIDE / 4), J,
                                           __builtin_amdgcn_readlane(jxa, LPF * f),
                                           __builtin_amdgcn_readlane(jy0, LPF * f), sg);
                }
                wave_lds_sync();
            }
            {
                const unsigned long long act = __builtin_amdgcn_ballot_w64(lact);
#pragma unroll
                for (int f = 0; f < FPW; f++) itc[f] += (int)((act >> (LPF * f)) & 1ull);
            }
            const BiW w = bilinear_weights(nextx - fnx, nexty - fny);
            const unsigned W0 = w.W0, W1 = w.W1;
            int bsum[2] = {-csum[0], -csum[1]};
            {
                // (iny - jy0) JRW + (inx - jxa) as one 24-bit multiply-add against the
                // region origin's offset; an inactive group reads inside its own region
                // (results unused)
                const int off = lact ? __mul24(iny, JRW) + inx - jbase : 0;
                const unsigned* jb = jmine + off;
                int jlast = 0;  // (ODD) the even strip's last row
#pragma unroll
                for (int k = 0; k < K; k++) {
                    const unsigned* js = jb + srow[k] * JRW + scol[k];
                    unsigned q[NR + 1];
#pragma unroll
                    for (int r = 0; r <= NR; r++) q[r] = js[r * JRW];
                    int jv[NR + 1];
                    jv[NR] = 0;
#pragma unroll
                    for (int r = 0; r < NR; r++)  // J x 2^kJShift: descaled value in bits 16..31
                        jv[r] = sdot2(q[r], W0, sdot2_r(q[r + 1], W1, rnd_j));
#pragma unroll
                    for (int m = 0; m < NP; m++) {
                        const unsigned jj = hi16x2(jv[2 * m], jv[2 * m + 1]);  // J; the I part is in csum
                        bsum[0] = sdot2(jj, GX[k][m], bsum[0]);
                        bsum[1] = sdot2(jj, GY[k][m], bsum[1]);
                    }
                    if constexpr (ODD) {
                        if (k & 1) {
                            const unsigned jj = hi16x2(jlast, jv[NR - 1]);
                            bsum[0] = sdot2(jj, GXO[k / 2], bsum[0]);
                            bsum[1] = sdot2(jj, GYO[k / 2], bsum[1]);
                        } else {
                            jlast = jv[NR - 1];
                        }
                    }
                }
            }
            float fb[2];
            group_sum_f<LPF, STEPS32>(bsum, fb);
            // materialised here, ahead of the lane-divergent update below: sunk into
            // it, the last DPP step splits into v_mov_dpp + a separate add per value
            asm volatile("" : "+v"(fb[0]), "+v"(fb[1]));
            const float fb1 = fb[0], fb2 = fb[1];
            const float dx = (A12 * fb2 - A22 * fb1) * Ds;
            const float dy = (A12 * fb1 - A11 * fb2) * Ds;
            if (lact) {
                nextx += dx;
                nexty += dy;
                nx = nextx + halfWx;
                ny = nexty + halfWy;
                if (converged(dx, dy, p.eps2_lo, p.eps2_hi, p.eps2)) {
                    lact = false;
                } else if (j > 0 && below_001(dx + pdx) && below_001(dy + pdy)) {
                    nx -= dx * 0.5f;
                    ny -= dy * 0.5f;
                    lact = false;
                } else {
                    pdx = dx;
                    pdy = dy;
                }
            }
        }
        if constexpr (TAIL) {
            if (tail_j >= 0) {
                // The single-group tail. One feature (group fs) is still iterating and
                // the wave's other groups are done with this level, so its iterations
                // run on all 64 lanes, one strip per lane instead of four: lane t takes
                // strip (l, k) = ((t >> 1) & 15, 2 (t >> 5) + (t & 1)) of the group's map
                // -- strips 2i and 2i + 1 of a group lane on neighbouring lanes, so the
                // odd-row pair that joins their last rows is one DPP move away. The
                // feature's G pairs move to LDS once (the region of a finished group:
                // it is not read again this level), its state to scalars. The b sums
                // stay exact integers: sum J G over the 64 lanes as 16-bit halves minus
                // the group's sum I G (its csum lanes, halves), rounded to float once
                // -- the same float as the group path, whatever the distribution.
                const int fs = (int)(__builtin_ctzll(__builtin_amdgcn_ballot_w64(lact)) / LPF);
                const int ls = fs * LPF;
                unsigned* const gst = jregs + ((fs + 1) & (FPW - 1)) * (Q::JSTRIDE / 4);
                unsigned* const jstar = jregs + fs * (Q::JSTRIDE / 4);
                if (g == fs) {
#pragma unroll
                    for (int k = 0; k < K; k++) {
                        const int t = ((k >> 1) << 5) | (l << 1) | (k & 1);
                        const unsigned ox = (k & 1) ? GXO[k >> 1] : 0u, oy = (k & 1) ? GYO[k >> 1] : 0u;
                        *reinterpret_cast<uint4*>(gst + 8 * t) = uint4{GX[k][0], GX[k][1], GX[k][2], GY[k][0]};
                        *reinterpret_cast<uint4*>(gst + 8 * t + 4) = uint4{GY[k][1], GY[k][2], ox, oy};
                    }
                }
                int ch0, cl0, ch1, cl1;
                group_halves<LPF, STEPS32>(csum[0], ch0, cl0);
                group_halves<LPF, STEPS32>(csum[1], ch1, cl1);
                ch0 = __builtin_amdgcn_readlane(ch0, ls);
                cl0 = __builtin_amdgcn_readlane(cl0, ls);
                ch1 = __builtin_amdgcn_readlane(ch1, ls);
                cl1 = __builtin_amdgcn_readlane(cl1, ls);
                wave_lds_sync();
                const uint4 ga = *reinterpret_cast<const uint4*>(gst + 8 * lane);
                const uint4 gb = *reinterpret_cast<const uint4*>(gst + 8 * lane + 4);
                const unsigned TX[NP] = {ga.x, ga.y, ga.z}, TY[NP] = {ga.w, gb.x, gb.y};
                const unsigned TXO = gb.z, TYO = gb.w;
                int soff;
                {
                    const int sidx = ((lane >> 1) & (LPF - 1)) + LPF * (((lane >> 5) << 1) | (lane & 1));
                    const int sc = sidx < NSTRIP ? sidx : 0;
                    soff = (sc / WW) * NR * JRW + sc % WW;
                }
                float tnx = rl_f(nextx, ls), tny = rl_f(nexty, ls), tpdx = rl_f(pdx, ls), tpdy = rl_f(pdy, ls);
                float tox = rl_f(nx, ls), toy = rl_f(ny, ls);
                const float tA11 = rl_f(A11, ls), tA12 = rl_f(A12, ls), tA22 = rl_f(A22, ls), tDs = rl_f(Ds, ls);
                int tjx0 = __builtin_amdgcn_readlane(jx0, ls), tjy0 = __builtin_amdgcn_readlane(jy0, ls);
                int tjbase = __builtin_amdgcn_readlane(jbase, ls);
                int tst = __builtin_amdgcn_readlane(st, ls);
                int titc = 0;
                for (int j = tail_j; j < p.max_count; j++) {
                    const float fnx = __builtin_floorf(tnx), fny = __builtin_floorf(tny);
                    const int inx = (int)fnx, iny = (int)fny;
                    if (!((unsigned)(inx + WW) < (unsigned)(J.w + WW) && (unsigned)(iny + WH) < (unsigned)(J.h + WH))) {
                        if (level == 0) tst = 0;
                        break;
                    }
                    if ((unsigned)(inx - tjx0) > 2u * QJM || (unsigned)(iny - tjy0) > 2u * QJM) {
                        tjx0 = inx - QJM;
                        tjy0 = iny - QJM;
                        tjbase = tjy0 * JRW + (tjx0 & ~3);
                        wave_lds_sync();
                        stage_padded<JRW, JRH>(jstar, J, tjx0 & ~3, tjy0, sg);
                        wave_lds_sync();
                    }
                    titc++;
                    const BiW w = bilinear_weights(tnx - fnx, tny - fny);
                    const unsigned* js = jstar + (__mul24(iny, JRW) + inx - tjbase) + soff;
                    unsigned q[NR + 1];
#pragma unroll
                    for (int r = 0; r <= NR; r++) q[r] = js[r * JRW];
                    int jv[NR];
#pragma unroll
                    for (int r = 0; r < NR; r++) jv[r] = sdot2(q[r], w.W0, sdot2_r(q[r + 1], w.W1, rnd_j));
                    int b0 = 0, b1 = 0;
#pragma unroll
                    for (int m = 0; m < NP; m++) {
                        const unsigned jj = hi16x2(jv[2 * m], jv[2 * m + 1]);
                        b0 = sdot2(jj, TX[m], b0);
                        b1 = sdot2(jj, TY[m], b1);
                    }
                    {
                        // the even strip's last row from the neighbouring lane (quad_perm
                        // 1,0,3,2); even lanes hold zero odd-pair G
                        const int jp = __builtin_amdgcn_update_dpp(0, jv[NR - 1], 0xb1, 0xf, 0xf, true);
                        const unsigned jj = hi16x2(jp, jv[NR - 1]);
                        b0 = sdot2(jj, TXO, b0);
                        b1 = sdot2(jj, TYO, b1);
                    }
                    int h0, l0, h1, l1;
                    wave_halves2(b0, b1, h0, l0, h1, l1);
                    const float fb1 = __builtin_fmaf((float)(h0 - ch0), 65536.f, (float)(l0 - cl0));
                    const float fb2 = __builtin_fmaf((float)(h1 - ch1), 65536.f, (float)(l1 - cl1));
                    const float dx = (tA12 * fb2 - tA22 * fb1) * tDs;
                    const float dy = (tA12 * fb1 - tA11 * fb2) * tDs;
                    tnx += dx;
                    tny += dy;
                    tox = tnx + halfWx;
                    toy = tny + halfWy;
                    if (converged(dx, dy, p.eps2_lo, p.eps2_hi, p.eps2)) break;
                    if (j > 0 && below_001(dx + tpdx) && below_001(dy + tpdy)) {
                        tox -= dx * 0.5f;
                        toy -= dy * 0.5f;
                        break;
                    }
                    tpdx = dx;
                    tpdy = dy;
                }
                if (g == fs) {
                    nx = tox;
                    ny = toy;
                    st = tst;
                }
#pragma unroll
                for (int f = 0; f < FPW; f++) itc[f] += f == fs ? titc : 0;
            }
        }
        wave_lds_sync();
    }
    if (l == 0 && live) {
        next_xy[2 * pt] = nx;
        next_xy[2 * pt + 1] = ny;
        B.status[base + pt] = (uint8_t)st;
        if (B.err) B.err[base + pt] = errv;
        if (B.iters) {
            int itcount = itc[0];
#pragma unroll
            for (int f = 1; f < FPW; f++) itcount = g == f ? itc[f] : itcount;
            B.iters[base + pt] = itcount;
        }
    }
    if constexpr (LOOP) {
        tx += gridDim.x;
        goto next_tile;
    }
}

// ---------------------------------------------------------------------------
// OpenCV's float summation order, four features per wave (lk_cvq_kernel): the
// sums of lk_cv_kernel (the same chains, the same 2^24 shortcut, the same
// combination of lanes: oracle/lk.c ACC_SSE) on lk_multi_kernel's lane map and
// staging. lk_cv_kernel runs one feature per wave, so its ordered chains -- ten
// per iteration, fifteen per level -- kept 10-15 of 64 lanes busy; here each
// 16-lane group runs its own feature's chains on its lanes 0-9 / 0-14, four
// features at once.
//  * setup per level: every strip lane samples I (x32), Ix, Iy at its pixels
//    (fixed point, as lk_multi_kernel) and keeps them; Ix | Iy << 16 go to the
//    group's LDS window in the A chains' order; the exact A sums decide the
//    shortcut (A11, A22 <= 2^24: every chain exact);
//  * iteration: the b terms d Ix, d Iy of every pixel go to the group's LDS region
//    in the b chains' order (the A window's place: it is no longer read), the
//    exact |term| total decides the shortcut.
// Per wave: the four groups' next-image regions (MultiShape), their term regions
// (2 win_w win_h ints) and the chain results (16 floats per group).
template <int WW, int WH, int NR>
struct CvqShape {
    using Q = MultiShape<1, WW, WH, 4>;
    static constexpr int NPX = WW * WH;
    static constexpr int SE4 = WW >= 4 ? ((WW - 4) / 4 + 1) * 4 : 0;  // OpenCV's 4-wide column end
    static constexpr int SE8 = WW >= 8 ? ((WW - 8) / 8 + 1) * 8 : 0;  // and the 8-wide b loop's
    static constexpr int M4 = SE4 / 4, B8 = SE8 / 8;
    static constexpr int TSTRIDE = 2 * NPX;  // ints per group's term region
    static constexpr int TERM_OFF = 4 * Q::JSTRIDE;
    static constexpr int CHAIN_OFF = TERM_OFF + 4 * TSTRIDE * 4;
    static constexpr int LDS_BYTES = CHAIN_OFF + 4 * 16 * 4;
    // a pixel's slot in the A chains' order (lane k = x & 3 over x < SE4: row by row,
    // columns in order; then the scalar chain over the rest)
    static __device__ __forceinline__ int a_slot(int y, int x) {
        return x < SE4 ? (x & 3) * WH * M4 + y * M4 + (x >> 2) : 4 * WH * M4 + y * (WW - SE4) + (x - SE4);
    }
    // and in the b chains' (lane t = x & 3 over x < SE8: per row and 8-column block
    // the pair x, x + 4 adjacent; then the scalar chain)
    static __device__ __forceinline__ int b_slot(int y, int x) {
        return x < SE8 ? (x & 3) * WH * 2 * B8 + y * 2 * B8 + 2 * (x >> 3) + ((x >> 2) & 1)
                       : WH * SE8 + y * (WW - SE8) + (x - SE8);
    }
};

// group sum of an int32 whose 16-lane total fits int32 (the shortcuts' operands)
__device__ __forceinline__ int group16_sum(int v) {
    v = dpp_row_add<0xb1>(v);
    v = dpp_row_add<0x4e>(v);
    v = dpp_row_add<0x124>(v);
    return dpp_row_add<0x128>(v);
}

template <int WW, int WH, int NR>
__global__ __launch_bounds__(64) void lk_cvq_kernel(LKBatch B, LKDev p) {
    constexpr int FPW = 4, LPF = 16;
    using C = CvqShape<WW, WH, NR>;
    using Q = typename C::Q;
    static_assert(WH % NR == 0, "whole strips");
    static_assert(WW + 4 <= kPyrPad && WW + 1 <= kDerPad, "padding too small for the window");
    constexpr int JRW = Q::JRW, JRH = Q::JRH, QJM = 1;
    constexpr int NSTRIP = WW * (WH / NR);
    constexpr int K = (NSTRIP + LPF - 1) / LPF;
    constexpr int NPX = C::NPX, SE4 = C::SE4, SE8 = C::SE8, M4 = C::M4, B8 = C::B8;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int lane = threadIdx.x & 63;
    const int g = lane / LPF, l = lane % LPF;
    const XcdTile tile = p.xcd ? xcd_tile() : XcdTile{(int)blockIdx.x, (int)blockIdx.y, 0};
    const int seq = tile.y;
    const int n = B.counts ? B.counts[seq] : B.n;
    const int pt0 = tile.x * FPW;
    if (pt0 >= n) return;
    const int pt = pt0 + g;
    const bool live = pt < n;
    const int ptc = live ? pt : n - 1;  // an idle group shadows a real feature, writes nothing
    const size_t base = (size_t)seq * B.cap;
    const float* __restrict__ prev_xy = B.prev_xy + 2 * base;
    float* __restrict__ next_xy = B.next_xy + 2 * base;
    const cpyr prev = (cpyr)B.prev + seq;
    const cpyr next = (cpyr)B.next + seq;
    const DerivDesc& dprev = B.dprev[seq];
    unsigned* jregs = reinterpret_cast<unsigned*>(lds);
    const unsigned* jmine = jregs + g * (Q::JSTRIDE / 4);
    int* terms = reinterpret_cast<int*>(lds + C::TERM_OFF) + g * C::TSTRIDE;
    float* chains = reinterpret_cast<float*>(lds + C::CHAIN_OFF) + g * 16;
    const StageGeom<JRW, JRH> sg(lane);

    int scol[K], srow[K];
    bool sreal[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
        const int sidx = l + LPF * k;
        sreal[k] = sidx < NSTRIP;
        const int sc = sreal[k] ? sidx : 0;
        scol[k] = sc % WW;
        srow[k] = (sc / WW) * NR;
    }
    // this lane's chains: A (lanes 0-14: quantity l / 5, SIMD lane l % 5 < 4 or the
    // scalar chain), b (lanes 0-9: b1 / b2 the same way)
    const int aq = l / 5, ak = l - 5 * (l / 5);
    const int a_off = ak < 4 ? ak * WH * M4 : 4 * WH * M4;
    const int a_len = l < 15 ? (ak < 4 ? WH * M4 : WH * (WW - SE4)) : 0;
    const int b_off = aq * NPX + (ak < 4 ? ak * WH * 2 * B8 : WH * SE8);
    const int b_len = l < 10 ? (ak < 4 ? WH * B8 : WH * (WW - SE8)) : 0;

    constexpr float halfWx = (WW - 1) * 0.5f, halfWy = (WH - 1) * 0.5f;
    const int rnd_i = 1 << (W_BITS - 6), rnd_d = 1 << (W_BITS + kDerShift - 1);
    const int rnd_j = 1 << (W_BITS - 6 + kJShift);

    const float px = prev_xy[2 * ptc], py = prev_xy[2 * ptc + 1];
    float nx = 0.f, ny = 0.f;
    if (p.flags & SVO_LK_USE_INITIAL_FLOW) {
        nx = next_xy[2 * ptc];
        ny = next_xy[2 * ptc + 1];
    }
    int st = live ? 1 : 0;
    float errv = 0.f;
    int itc[FPW];
#pragma unroll
    for (int f = 0; f < FPW; f++) itc[f] = 0;
    const int max_level = p.max_level;

    for (int level = max_level; level >= 0; level--) {
        const ImgLevel I{prev->lv[level].data, prev->lv[level].w, prev->lv[level].h, prev->lv[level].pitch};
        const ImgLevel J{next->lv[level].data, next->lv[level].w, next->lv[level].h, next->lv[level].pitch};
        const float lscale = __builtin_amdgcn_ldexpf(1.f, -level);
        float prevx = px * lscale, prevy = py * lscale;
        float nextx, nexty;
        if (level == max_level) {
            if (p.flags & SVO_LK_USE_INITIAL_FLOW) {
                nextx = nx * lscale;
                nexty = ny * lscale;
            } else {
                nextx = prevx;
                nexty = prevy;
            }
        } else {
            nextx = nx * 2.f;
            nexty = ny * 2.f;
        }
        nx = nextx;
        ny = nexty;
        prevx -= halfWx;
        prevy -= halfWy;
        const float fpx = __builtin_floorf(prevx), fpy = __builtin_floorf(prevy);
        const int ipx = (int)fpx, ipy = (int)fpy;
        const bool inb = (unsigned)(ipx + WW) < (unsigned)(I.w + WW) && (unsigned)(ipy + WH) < (unsigned)(I.h + WH);
        if (!inb && level == 0 && live) {
            st = 0;
            errv = 0.f;
        }
        bool lact = live && inb;
        const BiW iw = bilinear_weights(prevx - fpx, prevy - fpy);
        const unsigned IW0 = iw.W0, IW1 = iw.W1;

        int jx0 = ufloor(nextx - halfWx) - QJM, jy0 = ufloor(nexty - halfWy) - QJM;
        int jxa = jx0 & ~3;
        int jbase = jy0 * JRW + jxa;
        // per strip pixel: I (x32) and Ix | Iy << 16 (descaled, int16 each)
        int IV[K][NR];
        unsigned IXY[K][NR];
        int a11 = 0, a22 = 0;  // exact partials (the shortcut needs A11 and A22 only)
        {
            using SL = StageGeom<JRW, JRH>;
            int xs[FPW], ys[FPW];
#pragma unroll
            for (int f = 0; f < FPW; f++) {
                const int xa = __builtin_amdgcn_readlane(jxa, LPF * f), y0 = __builtin_amdgcn_readlane(jy0, LPF * f);
                const bool ok = __builtin_amdgcn_readlane((int)lact, LPF * f) && region_in_pad<JRW, JRH>(J, xa, y0);
                xs[f] = ok ? xa : 0;
                ys[f] = ok ? y0 : 0;
            }
            {
                unsigned sv[FPW][SL::NPS];
                const gu8 jb0 = pad_origin(J.data, J.pitch, kPyrPad, 1) + (size_t)kPyrPad * (J.pitch + 1);
                const unsigned ol = 4u * (unsigned)sg.d + (unsigned)sg.row(0) * (unsigned)J.pitch;
                const unsigned olast = 4u * (unsigned)sg.d + (unsigned)sg.row(SL::NPS - 1) * (unsigned)J.pitch;
#pragma unroll
                for (int f = 0; f < FPW; f++) {
                    const gu8 fb = jb0 + xs[f] + (ptrdiff_t)ys[f] * J.pitch;
#pragma unroll
                    for (int q = 0; q < SL::NPS; q++)
                        sv[f][q] = q + 1 < SL::NPS ? ldg_off<unsigned>(fb + (size_t)q * SL::RPP * J.pitch, ol)
                                                   : ldg_off<unsigned>(fb, olast);
                }
#pragma unroll
                for (int f = 0; f < FPW; f++)
#pragma unroll
                    for (int q = 0; q < SL::NPS; q++) sg.write(jregs + f * (Q::JSTRIDE / 4), sg.row(q), sv[f][q]);
            }
            const int dpitch = dprev.pitch[level];
            const gu8 ibase = pad_origin(I.data, I.pitch, kPyrPad, 1);
            const gu8 dbase = pad_origin((const uint8_t*)dprev.data[level], dpitch, kDerPad, 4);
            const int sx = inb ? ipx : 0, sy = inb ? ipy : 0;
#pragma unroll
            for (int k = 0; k < K; k++) {
                unsigned P[NR + 1];
                u32x2a4 Dv[NR + 1];
                const int x = sx + scol[k], y = sy + srow[k];
                const unsigned oi = (unsigned)(x + kPyrPad) + (unsigned)(y + kPyrPad) * (unsigned)I.pitch;
                const unsigned od = 4u * ((unsigned)(x + kDerPad) + (unsigned)(y + kDerPad) * (unsigned)dpitch);
#pragma unroll
                for (int r = 0; r <= NR; r++) {
                    P[r] = __builtin_amdgcn_perm(0u, (unsigned)ldg_off<u16a1>(ibase + (size_t)r * I.pitch, oi),
                                                 0x0c010c00u);
                    Dv[r] = ldg_off<u32x2a4>(dbase + (size_t)r * 4 * dpitch, od);
                }
                const unsigned GW0 = sreal[k] ? IW0 : 0u, GW1 = sreal[k] ? IW1 : 0u;
#pragma unroll
                for (int j = 0; j < NR; j++) {
                    IV[k][j] = sdot2(P[j], IW0, sdot2_r(P[j + 1], IW1, rnd_i)) >> (W_BITS - 5);
                    const unsigned X0 = __builtin_amdgcn_perm(Dv[j].y, Dv[j].x, 0x05040100u);
                    const unsigned X1 = __builtin_amdgcn_perm(Dv[j + 1].y, Dv[j + 1].x, 0x05040100u);
                    const unsigned Y0 = __builtin_amdgcn_perm(Dv[j].y, Dv[j].x, 0x07060302u);
                    const unsigned Y1 = __builtin_amdgcn_perm(Dv[j + 1].y, Dv[j + 1].x, 0x07060302u);
                    const int ix = sdot2(X0, GW0, sdot2_r(X1, GW1, rnd_d)) >> 16;  // CV_DESCALE(., W_BITS)
                    const int iy = sdot2(Y0, GW0, sdot2_r(Y1, GW1, rnd_d)) >> 16;
                    IXY[k][j] = pack16(ix, iy);
                    a11 += ix * ix;
                    a22 += iy * iy;
                    if (sreal[k]) terms[C::a_slot(srow[k] + j, scol[k])] = (int)IXY[k][j];
                }
            }
        }
        wave_lds_sync();
        // the shortcut: every A chain is exact when A11, A22 <= 2^24 (|Ix Iy| <= (Ix^2 +
        // Iy^2) / 2); a lane's partials stay < 2^31 (<= NR K 4080^2), capped so that the
        // group's 16 cannot overflow
        constexpr int kCap = (1 << 24) + 1;
        const int e11 = group16_sum(min(a11, kCap)), e22 = group16_sum(min(a22, kCap));
        const bool a_exact = e11 <= (1 << 24) && e22 <= (1 << 24);
        float sA[3];
        {
            // the exact sums, for the groups the shortcut covers (A12 then too: |A12| <=
            // 2^24); and the ordered chains if any active group needs them
            int e12p = 0;
#pragma unroll
            for (int k = 0; k < K; k++)
#pragma unroll
                for (int j = 0; j < NR; j++) e12p += (int)(short)(IXY[k][j] & 0xffffu) * ((int)IXY[k][j] >> 16);
            const int e12 = group16_sum(a_exact ? e12p : 0);
            sA[0] = (float)e11;
            sA[1] = (float)e12;
            sA[2] = (float)e22;
            if (__builtin_amdgcn_ballot_w64(lact && !a_exact)) {
                float acc = 0.f;
                const int* src = terms + a_off;
#pragma unroll 4
                for (int i = 0; i < a_len; i++) {
                    const int w = src[i];
                    const int ix = (int)(short)(w & 0xffff), iy = w >> 16;
                    acc += (float)(aq == 0 ? ix * ix : aq == 1 ? ix * iy : iy * iy);
                }
                if (l < 15) chains[l] = acc;
                wave_lds_sync();
                if (!a_exact) {
#pragma unroll
                    for (int q = 0; q < 3; q++)
                        sA[q] = chains[5 * q + 4] + ((chains[5 * q] + chains[5 * q + 2]) + (chains[5 * q + 1] + chains[5 * q + 3]));
                }
            }
        }
        wave_lds_sync();  // (the A window's reads finish before the b terms reuse it)
        const float A11 = sA[0] * FLT_SCALE, A12 = sA[1] * FLT_SCALE, A22 = sA[2] * FLT_SCALE;
        float D = A11 * A22 - A12 * A12;
        const float minEig = (A22 + A11 - sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) / (float)(2 * WW * WH);
        if (lact && p.want_err && (p.flags & SVO_LK_GET_MIN_EIGENVALS)) errv = minEig;
        if (lact && (minEig < p.min_eig || D < FLT_EPSILON)) {
            if (level == 0) st = 0;
            lact = false;
        }
        D = 1.f / D;

        nextx -= halfWx;
        nexty -= halfWy;
        float pdx = 0.f, pdy = 0.f;
        for (int j = 0; j < p.max_count; j++) {
            if (__builtin_amdgcn_ballot_w64(lact) == 0) break;
            const float fnx = __builtin_floorf(nextx), fny = __builtin_floorf(nexty);
            const int inx = (int)fnx, iny = (int)fny;
            if (lact && !((unsigned)(inx + WW) < (unsigned)(J.w + WW) && (unsigned)(iny + WH) < (unsigned)(J.h + WH))) {
                if (level == 0) st = 0;
                lact = false;
            }
            const bool need = lact && ((unsigned)(inx - jx0) > 2u * QJM || (unsigned)(iny - jy0) > 2u * QJM);
            unsigned long long nb = __builtin_amdgcn_ballot_w64(need && l == 0);
            if (nb) {
                if (need) {
                    jx0 = inx - QJM;
                    jy0 = iny - QJM;
                    jxa = jx0 & ~3;
                    jbase = jy0 * JRW + jxa;
                }
                wave_lds_sync();
                while (nb) {
                    const int f = (int)(__builtin_ctzll(nb) / LPF);
                    nb &= nb - 1;
                    stage_padded<JRW, JRH>(jregs + f * (Q::JSTRIDE / 4), J, __builtin_amdgcn_readlane(jxa, LPF * f),
                                           __builtin_amdgcn_readlane(jy0, LPF * f), sg);
                }
                wave_lds_sync();
            }
            {
                const unsigned long long act = __builtin_amdgcn_ballot_w64(lact);
#pragma unroll
                for (int f = 0; f < FPW; f++) itc[f] += (int)((act >> (LPF * f)) & 1ull);
            }
            const BiW w = bilinear_weights(nextx - fnx, nexty - fny);
            const unsigned W0 = w.W0, W1 = w.W1;
            int b1 = 0, b2 = 0, babs = 0;
            {
                const int off = lact ? __mul24(iny, JRW) + inx - jbase : 0;
                const unsigned* jb = jmine + off;
#pragma unroll
                for (int k = 0; k < K; k++) {
                    const unsigned* js = jb + srow[k] * JRW + scol[k];
                    unsigned q[NR + 1];
#pragma unroll
                    for (int r = 0; r <= NR; r++) q[r] = js[r * JRW];
#pragma unroll
                    for (int r = 0; r < NR; r++) {
                        const int jv = sdot2(q[r], W0, sdot2_r(q[r + 1], W1, rnd_j)) >> 16;
                        const int d = jv - IV[k][r];
                        const int t1 = d * (int)(short)(IXY[k][r] & 0xffffu), t2 = d * ((int)IXY[k][r] >> 16);
                        b1 += t1;
                        b2 += t2;
                        // |terms| <= 8160 * 4080 < 2^25: capped so the group's 16 lanes cannot overflow
                        babs = min(babs + abs(t1) + abs(t2), kCap);
                        if (sreal[k]) {
                            const int s = C::b_slot(srow[k] + r, scol[k]);
                            terms[s] = t1;
                            terms[NPX + s] = t2;
                        }
                    }
                }
            }
            const bool b_exact = group16_sum(babs) <= (1 << 24);
            float fb1 = (float)group16_sum(b_exact ? b1 : 0), fb2 = (float)group16_sum(b_exact ? b2 : 0);
            if (__builtin_amdgcn_ballot_w64(lact && !b_exact)) {
                wave_lds_sync();
                float acc = 0.f;
                const int* src = terms + b_off;
                if (ak < 4) {
#pragma unroll 6
                    for (int i = 0; i < b_len; i++) acc += (float)(src[2 * i] + src[2 * i + 1]);
                } else {
#pragma unroll 8
                    for (int i = 0; i < b_len; i++) acc += (float)src[i];
                }
                if (l < 10) chains[l] = acc;
                wave_lds_sync();
                if (!b_exact) {
                    fb1 = chains[4] + (((chains[0] + chains[2]) + 0.f) + ((chains[1] + chains[3]) + 0.f));
                    fb2 = chains[9] + (((chains[5] + chains[7]) + 0.f) + ((chains[6] + chains[8]) + 0.f));
                }
            }
            wave_lds_sync();  // (the terms' reads finish before the next iteration's writes)
            fb1 *= FLT_SCALE;
            fb2 *= FLT_SCALE;
            const float dx = (A12 * fb2 - A22 * fb1) * D;
            const float dy = (A12 * fb1 - A11 * fb2) * D;
            if (lact) {
                nextx += dx;
                nexty += dy;
                nx = nextx + halfWx;
                ny = nexty + halfWy;
                if (converged(dx, dy, p.eps2_lo, p.eps2_hi, p.eps2)) {
                    lact = false;
                } else if (j > 0 && below_001(dx + pdx) && below_001(dy + pdy)) {
                    nx -= dx * 0.5f;
                    ny -= dy * 0.5f;
                    lact = false;
                } else {
                    pdx = dx;
                    pdy = dy;
                }
            }
        }
        wave_lds_sync();
    }
    if (l == 0 && live) {
        next_xy[2 * pt] = nx;
        next_xy[2 * pt + 1] = ny;
        B.status[base + pt] = (uint8_t)st;
        if (B.err) B.err[base + pt] = errv;
        if (B.iters) {
            int itcount = itc[0];
#pragma unroll
            for (int f = 1; f < FPW; f++) itcount = g == f ? itc[f] : itcount;
            B.iters[base + pt] = itcount;
        }
    }
}

template <int WW, int WH, int NR>
hipError_t launch_cvq(const LKBatch& b, int nseq, int max_n, const LKDev& d, hipStream_t st) {
    dim3 grid((max_n + 3) / 4, nseq);
    constexpr int lds_bytes = CvqShape<WW, WH, NR>::LDS_BYTES;
    hipLaunchKernelGGL((lk_cvq_kernel<WW, WH, NR>), grid, dim3(64), lds_bytes, st, b, d);
    return hipGetLastError();
}

template <int FPW, int QJM, int MINW = 4, int KKS = 2, int WW = 21, int WH = 21, int NR = 7, bool LOOP = false>
hipError_t launch_multi(const LKBatch& b, int nseq, int max_n, const LKDev& d, hipStream_t st) {
    const int gn = LOOP && b.grid_hint > 0 && b.grid_hint < max_n ? b.grid_hint : max_n;
    dim3 grid((gn + FPW - 1) / FPW, nseq);
    // SVO_LK_LDS_PAD (bytes, temporal call): a larger LDS carve per wave caps LK's waves
    // per CU below the 16 its 9,984 B allow, leaving LDS for the kernels that run beside it
    static const int lds_pad = [] {
        const char* e = std::getenv("SVO_LK_LDS_PAD");
        return e ? std::atoi(e) : 0;
    }();
    const int lds_bytes = FPW * MultiShape<QJM, WW, WH, FPW>::JSTRIDE + (LOOP ? 0 : lds_pad);
    hipLaunchKernelGGL((lk_multi_kernel<FPW, QJM, MINW, KKS, WW, WH, NR, LOOP>), grid, dim3(64), lds_bytes, st, b, d);
    return hipGetLastError();
}

template <int WW, int WH>
hipError_t launch_fast(const LKBatch& b, int nseq, int max_n, const LKDev& d, hipStream_t st) {
    const int gn = b.grid_hint > 0 && b.grid_hint < max_n ? b.grid_hint : max_n;
    dim3 grid((gn + 3) / 4, nseq);
    constexpr int lds_bytes = 4 * Shape<WW, WH>::WAVE_BYTES;
    // occupancy is limited by LDS (7 blocks/CU) and ~70 VGPRs alike; capping the
    // VGPRs lower spills (measured: launch bounds 6/7/8 waves all slower)
    hipLaunchKernelGGL((lk_fast_kernel<WW, WH, 1>), grid, dim3(256), lds_bytes, st, b, d);
    return hipGetLastError();
}

template <int RPG>
hipError_t launch_rpg(const LKBatch& b, int nseq, int max_n, const LKDev& d, hipStream_t st) {
    dim3 grid((max_n + 3) / 4, nseq);
    if (d.groups * RPG == d.win_h)
        hipLaunchKernelGGL((lk_kernel<RPG, true>), grid, dim3(256), 4 * d.lds_wave, st, b, d);
    else
        hipLaunchKernelGGL((lk_kernel<RPG, false>), grid, dim3(256), 4 * d.lds_wave, st, b, d);
    return hipGetLastError();
}

template <int RPG>
hipError_t launch_cv_rpg(const LKBatch& b, int nseq, int max_n, const LKDev& d, hipStream_t st) {
    CvOrder co;
    co.se4 = d.win_w >= 4 ? ((d.win_w - 4) / 4 + 1) * 4 : 0;
    co.se8 = d.win_w >= 8 ? ((d.win_w - 8) / 8 + 1) * 8 : 0;
    co.term_off = (d.lds_wave + 15) & ~15;
    const int lds = co.term_off + 3 * d.win_w * d.win_h * 4;
    dim3 grid(max_n, nseq);
    if (d.groups * RPG == d.win_h)
        hipLaunchKernelGGL((lk_cv_kernel<RPG, true>), grid, dim3(64), lds, st, b, d, co);
    else
        hipLaunchKernelGGL((lk_cv_kernel<RPG, false>), grid, dim3(64), lds, st, b, d, co);
    return hipGetLastError();
}

}  // namespace

void lk_apply_env(LKParams& p) {
    const char* gen = std::getenv("SVO_LK_GENERIC");
    p.generic = gen && gen[0] == '1' ? 1 : 0;
    const char* quad = std::getenv("SVO_LK_QUAD");
    p.quad = quad && quad[0] == '0' ? 0 : 1;
}

bool lk_supported(int win_w, int win_h) {
    if (win_w < 3 || win_h < 3 || win_w + 2 * JM > 64 || win_w + 3 > 64) return false;
    int groups = 64 / win_w;
    int rpg = (win_h + groups - 1) / groups;
    return rpg <= 32 && win_w * win_h <= 2048;
}

hipError_t launch_lk(const LKBatch& b, int nseq, int max_n, const LKParams& lp, hipStream_t st) {
    if (max_n <= 0 || nseq <= 0) return hipSuccess;
    LKDev d;
    d.win_w = lp.win_w;
    d.win_h = lp.win_h;
    d.groups = 64 / lp.win_w;
    int rpg = (lp.win_h + d.groups - 1) / d.groups;
    d.ip_w = lp.win_w;                // prev window: win_w pairs x (win_h + 1) rows
    d.ip_h = lp.win_h + 1;
    d.jr_w = lp.win_w + 2 * JM;       // next region: pair entries per row (win_w + 2JM + 1 pixels)
    d.jr_h = lp.win_h + 1 + 2 * JM;
    d.ip_bytes = (d.ip_w * d.ip_h * 4 + 15) & ~15;
    d.lds_wave = d.ip_bytes + ((d.jr_w * d.jr_h * 4 + 15) & ~15);
    d.max_level = lp.max_level;
    d.max_count = lp.max_count;
    d.eps2 = lp.eps2;
    // |float(dx*dx + dy*dy) / exact - 1| <= 3 * 2^-24: outside eps2 * (1 -+ 2^-20) the
    // float sum decides the double comparison exactly
    d.eps2_lo = (float)(lp.eps2 * (1.0 - 0x1p-20));
    d.eps2_hi = (float)(lp.eps2 * (1.0 + 0x1p-20));
    if ((double)d.eps2_lo > lp.eps2 * (1.0 - 0x1p-20)) d.eps2_lo = nextafterf(d.eps2_lo, 0.f);
    if ((double)d.eps2_hi < lp.eps2 * (1.0 + 0x1p-20)) d.eps2_hi = nextafterf(d.eps2_hi, INFINITY);
    d.flags = lp.flags;
    d.want_err = lp.want_err;
    d.min_eig = lp.min_eig;
    {
        static const bool lk_xcd = [] {
            const char* e = std::getenv("SVO_LK_XCD");
            return !(e && e[0] == '0');
        }();
        d.xcd = lk_xcd ? 1 : 0;
        static const bool lk_tail = [] {
            const char* e = std::getenv("SVO_LK_TAIL");
            return !(e && e[0] == '0');
        }();
        d.tail = lk_tail ? 1 : 0;
    }
    if (lp.cv_order) {
        // OpenCV's float summation order: the reference's two windows four features
        // per wave (lk_cvq_kernel; not the SAD error of flags 0 + err), else one per
        // wave (lk_cv_kernel)
        const bool multi_ok = !(lp.want_err && !(lp.flags & SVO_LK_GET_MIN_EIGENVALS));
        if (!lp.generic && lp.quad && multi_ok) {
            if (lp.win_w == 21 && lp.win_h == 21) return launch_cvq<21, 21, 7>(b, nseq, max_n, d, st);
            if (lp.win_w == 11 && lp.win_h == 11) return launch_cvq<11, 11, 11>(b, nseq, max_n, d, st);
        }
#define SVO_LK_CV_CASE(R) \
    case R: return launch_cv_rpg<R>(b, nseq, max_n, d, st);
        switch (rpg) {
            SVO_LK_CV_CASE(1) SVO_LK_CV_CASE(2) SVO_LK_CV_CASE(3) SVO_LK_CV_CASE(4) SVO_LK_CV_CASE(5)
            SVO_LK_CV_CASE(6) SVO_LK_CV_CASE(7) SVO_LK_CV_CASE(8) SVO_LK_CV_CASE(11) SVO_LK_CV_CASE(16)
            default:
                break;
        }
#undef SVO_LK_CV_CASE
        if (rpg <= 16) return launch_cv_rpg<16>(b, nseq, max_n, d, st);
        return launch_cv_rpg<32>(b, nseq, max_n, d, st);
    }
    if (!lp.generic) {
        // four features per wave: the SAD error (flags 0 + want_err) stays on lk_fast_kernel
        const bool multi_ok = !(lp.want_err && !(lp.flags & SVO_LK_GET_MIN_EIGENVALS));
        if (lp.win_w == 21 && lp.win_h == 21 && multi_ok && lp.quad) {
            // four features per wave, 1-px staging margin (re-staged when the
            // estimate leaves it; measured 2.7 % faster alone than a 2-px margin
            // and than 3 px; two features per wave (lk_dual_kernel, another lane
            // map) measured slower and is gone; 4 waves/SIMD, 8 features per wave
            // and one strip ahead in the setup measured slower: DESIGN.md section 5)
            return launch_multi<4, 1, SVO_LK_MINW, SVO_LK_KKS>(b, nseq, max_n, d, st);
        }
        // the stereo call's 11 x 11 (findLeftFeaturesInRight, no err): four
        // features per wave too, one 11-row strip per lane (11 of 16 lanes). Capped
        // at 80 VGPRs (6 waves per SIMD; a few spills in the per-tile / per-level
        // code, none in the trip loop) so its waves fit beside LK's three per SIMD
        // (141 VGPRs each): +1.7 % frames/s over 91 VGPRs
        // (profiles/r06/e_setprio_stereo_minw_ab.txt)
        if (lp.win_w == 11 && lp.win_h == 11 && multi_ok && lp.quad)
            return launch_multi<4, 1, 6, 1, 11, 11, 11, true>(b, nseq, max_n, d, st);
        if (lp.win_w == 21 && lp.win_h == 21) return launch_fast<21, 21>(b, nseq, max_n, d, st);
        if (lp.win_w == 11 && lp.win_h == 11) return launch_fast<11, 11>(b, nseq, max_n, d, st);
        if (lp.win_w == 15 && lp.win_h == 15) return launch_fast<15, 15>(b, nseq, max_n, d, st);
        if (lp.win_w == 31 && lp.win_h == 31) return launch_fast<31, 31>(b, nseq, max_n, d, st);
    }
#define SVO_LK_CASE(R) \
    case R: return launch_rpg<R>(b, nseq, max_n, d, st);
    switch (rpg) {
        SVO_LK_CASE(1) SVO_LK_CASE(2) SVO_LK_CASE(3) SVO_LK_CASE(4) SVO_LK_CASE(5) SVO_LK_CASE(6)
        SVO_LK_CASE(7) SVO_LK_CASE(8) SVO_LK_CASE(9) SVO_LK_CASE(10) SVO_LK_CASE(11) SVO_LK_CASE(12)
        SVO_LK_CASE(14) SVO_LK_CASE(16)
        default:
            break;
    }
#undef SVO_LK_CASE
    // uncommon strip heights: round up to the next instantiated size
    if (rpg <= 13) return launch_rpg<14>(b, nseq, max_n, d, st);
    if (rpg <= 16) return launch_rpg<16>(b, nseq, max_n, d, st);
    return launch_rpg<32>(b, nseq, max_n, d, st);
}

}  // namespace svo
