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
//  * Per level the wave stages the (win+3)^2 u8 patch of the previous image in
//    LDS (REFLECT_101 outside the image, as OpenCV's padded pyramid), computes
//    the Scharr derivative at the (win+1)^2 bilinear grid points in LDS (zero
//    outside the image, as OpenCV's zero-padded derivative level) -- no
//    derivative image is ever materialised in HBM.
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

#include <cfloat>

namespace svo {

namespace {

constexpr int W_BITS = 14;
constexpr float FLT_SCALE = 1.f / (1 << 20);

__device__ __forceinline__ int descale(int x, int n) { return (x + (1 << (n - 1))) >> n; }

__device__ __forceinline__ int refl101(int p, int len) {
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        p = p < 0 ? -p : 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

__device__ __forceinline__ int ufloor(float v) {  // cvFloor
    int i = (int)v;
    return i - (i > v);
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
    int tile_w, tile_h, grid_w, grid_h;
    int tile_bytes, lds_wave;      // per-wave LDS carve
    int max_level, max_count;
    double eps2;
    int flags, want_err;
    float min_eig;
};

template <int RPG>
__global__ __launch_bounds__(256) void lk_kernel(PyrDesc prev, PyrDesc next,
                                                 const float* __restrict__ prev_xy,
                                                 float* __restrict__ next_xy,
                                                 uint8_t* __restrict__ status,
                                                 float* __restrict__ err, int* __restrict__ iters,
                                                 int n, LKDev p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int pt = blockIdx.x * 4 + wid;
    if (pt >= n) return;
    uint8_t* tile = lds + wid * p.lds_wave;
    int* grid = reinterpret_cast<int*>(tile + p.tile_bytes);

    const int win_w = p.win_w, win_h = p.win_h;
    const int sc = lane % win_w;
    const int sg = lane / win_w;
    const bool strip = sg < p.groups;
    const int r0 = sg * RPG;
    const int tile_rows_per_pass = 64 / p.tile_w;
    const int tl_r = lane / p.tile_w, tl_c = lane - (lane / p.tile_w) * p.tile_w;

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
        int iw00 = uround((1.f - a) * (1.f - b) * (1 << W_BITS));
        int iw01 = uround(a * (1.f - b) * (1 << W_BITS));
        int iw10 = uround((1.f - a) * b * (1 << W_BITS));
        int iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;

        // ---- stage the previous-image patch (rows ipy-1.., cols ipx-1..) ----
        {
            const int ty0 = ipy - 1, tx0 = ipx - 1;
            const bool inside = tx0 >= 0 && ty0 >= 0 && tx0 + p.tile_w <= I.w && ty0 + p.tile_h <= I.h;
            if (tl_r < tile_rows_per_pass) {
                for (int r = tl_r; r < p.tile_h; r += tile_rows_per_pass) {
                    int sy = ty0 + r, sx = tx0 + tl_c;
                    if (!inside) {
                        sy = refl101(sy, I.h);
                        sx = refl101(sx, I.w);
                    }
                    tile[r * p.tile_w + tl_c] = I.data[(size_t)sy * I.pitch + sx];
                }
            }
        }
        wave_lds_sync();
        // ---- Scharr derivative at the (win+1)^2 grid points, zero outside ----
        for (int k = lane; k < p.grid_w * p.grid_h; k += 64) {
            int gr = k / p.grid_w, gc = k - gr * p.grid_w;
            int X = ipx + gc, Y = ipy + gr;
            int v = 0;
            if (X >= 0 && X < I.w && Y >= 0 && Y < I.h) {
                const uint8_t* t0 = tile + gr * p.tile_w + gc;   // row Y-1, col X-1
                const uint8_t* t1 = t0 + p.tile_w;
                const uint8_t* t2 = t1 + p.tile_w;
                int tl = t0[0], tm = t0[1], tr = t0[2];
                int ml = t1[0], mr = t1[2];
                int bl = t2[0], bm = t2[1], br = t2[2];
                int ix = (3 * (tr + br) + 10 * mr) - (3 * (tl + bl) + 10 * ml);
                int iy = 3 * ((br - tr) + (bl - tl)) + 10 * (bm - tm);
                v = (int)(((unsigned)iy << 16) | ((unsigned)ix & 0xFFFFu));
            }
            grid[k] = v;
        }
        wave_lds_sync();

        // ---- per-lane strip: I (x32) and (Ix, Iy) at its window pixels ----
        int ival[RPG], gxy[RPG];
        int a11 = 0, a12 = 0, a22 = 0;
#pragma unroll
        for (int j = 0; j < RPG; j++) {
            ival[j] = 0;
            gxy[j] = 0;
            const int r = r0 + j;
            if (strip && r < win_h) {
                const uint8_t* t = tile + (r + 1) * p.tile_w + (sc + 1);
                ival[j] = descale(t[0] * iw00 + t[1] * iw01 + t[p.tile_w] * iw10 + t[p.tile_w + 1] * iw11,
                                  W_BITS - 5);
                const int* g = grid + r * p.grid_w + sc;
                int g00 = g[0], g01 = g[1], g10 = g[p.grid_w], g11 = g[p.grid_w + 1];
                int ix = descale((int)(short)g00 * iw00 + (int)(short)g01 * iw01 + (int)(short)g10 * iw10 +
                                     (int)(short)g11 * iw11, W_BITS);
                int iy = descale((g00 >> 16) * iw00 + (g01 >> 16) * iw01 + (g10 >> 16) * iw10 +
                                     (g11 >> 16) * iw11, W_BITS);
                gxy[j] = (int)(((unsigned)iy << 16) | ((unsigned)ix & 0xFFFFu));
                a11 += ix * ix;
                a12 += ix * iy;
                a22 += iy * iy;
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
            a = nextx - inx;
            b = nexty - iny;
            int w00 = uround((1.f - a) * (1.f - b) * (1 << W_BITS));
            int w01 = uround(a * (1.f - b) * (1 << W_BITS));
            int w10 = uround((1.f - a) * b * (1 << W_BITS));
            int w11 = (1 << W_BITS) - w00 - w01 - w10;
            int b1 = 0, b2 = 0;
            if (strip) {
                const bool inside = inx >= 0 && iny >= 0 && inx + win_w < J.w && iny + win_h < J.h;
                int c0 = inx + sc, c1 = c0 + 1;
                if (!inside) {
                    c0 = refl101(c0, J.w);
                    c1 = refl101(c1, J.w);
                }
                int jv[RPG + 1][2];
#pragma unroll
                for (int k = 0; k <= RPG; k++) {
                    jv[k][0] = jv[k][1] = 0;
                    if (r0 + k <= win_h) {
                        int y = iny + r0 + k;
                        if (!inside) y = refl101(y, J.h);
                        const uint8_t* row = J.data + (size_t)y * J.pitch;
                        jv[k][0] = row[c0];
                        jv[k][1] = row[c1];
                    }
                }
#pragma unroll
                for (int k = 0; k < RPG; k++) {
                    if (r0 + k < win_h) {
                        int diff = descale(jv[k][0] * w00 + jv[k][1] * w01 + jv[k + 1][0] * w10 +
                                               jv[k + 1][1] * w11, W_BITS - 5) - ival[k];
                        b1 += diff * (int)(short)gxy[k];
                        b2 += diff * (gxy[k] >> 16);
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
            float aa = npx - ix0, bb = npy - iy0;
            int w00 = uround((1.f - aa) * (1.f - bb) * (1 << W_BITS));
            int w01 = uround(aa * (1.f - bb) * (1 << W_BITS));
            int w10 = uround((1.f - aa) * bb * (1 << W_BITS));
            int w11 = (1 << W_BITS) - w00 - w01 - w10;
            int sad = 0;
            if (strip) {
                int c0 = refl101(ix0 + sc, J.w), c1 = refl101(ix0 + sc + 1, J.w);
#pragma unroll
                for (int k = 0; k < RPG; k++) {
                    if (r0 + k < win_h) {
                        const uint8_t* ra = J.data + (size_t)refl101(iy0 + r0 + k, J.h) * J.pitch;
                        const uint8_t* rb = J.data + (size_t)refl101(iy0 + r0 + k + 1, J.h) * J.pitch;
                        int diff = descale(ra[c0] * w00 + ra[c1] * w01 + rb[c0] * w10 + rb[c1] * w11,
                                           W_BITS - 5) - ival[k];
                        sad += diff < 0 ? -diff : diff;
                    }
                }
            }
            // |diff| sums stay < 2^24 for windows <= 2048 px: exact in float
            errv = (float)wave_sum_exact(sad) * 1.f / (float)(32 * win_w * win_h);
        }
    }
    if (lane == 0) {
        next_xy[2 * pt] = nx;
        next_xy[2 * pt + 1] = ny;
        status[pt] = (uint8_t)st;
        if (err) err[pt] = errv;
        if (iters) iters[pt] = itcount;
    }
}

template <int RPG>
hipError_t launch_rpg(const PyrDesc& prev, const PyrDesc& next, const float* prev_xy, float* next_xy,
                      uint8_t* status, float* err, int* iters, int n, const LKDev& d,
                      hipStream_t st) {
    dim3 grid((n + 3) / 4);
    hipLaunchKernelGGL(lk_kernel<RPG>, grid, dim3(256), 4 * d.lds_wave, st, prev, next, prev_xy,
                       next_xy, status, err, iters, n, d);
    return hipGetLastError();
}

}  // namespace

bool lk_supported(int win_w, int win_h) {
    if (win_w < 3 || win_h < 3 || win_w + 3 > 64) return false;
    int groups = 64 / win_w;
    int rpg = (win_h + groups - 1) / groups;
    return rpg <= 32 && win_w * win_h <= 2048;
}

hipError_t launch_lk(const PyrDesc& prev, const PyrDesc& next, const float* prev_xy, float* next_xy,
                     uint8_t* status, float* err, int* iters, int n, const LKParams& lp,
                     hipStream_t st) {
    if (n <= 0) return hipSuccess;
    LKDev d;
    d.win_w = lp.win_w;
    d.win_h = lp.win_h;
    d.groups = 64 / lp.win_w;
    int rpg = (lp.win_h + d.groups - 1) / d.groups;
    d.tile_w = lp.win_w + 3;
    d.tile_h = lp.win_h + 3;
    d.grid_w = lp.win_w + 1;
    d.grid_h = lp.win_h + 1;
    d.tile_bytes = (d.tile_w * d.tile_h + 15) & ~15;
    d.lds_wave = d.tile_bytes + ((d.grid_w * d.grid_h * 4 + 15) & ~15);
    d.max_level = lp.max_level;
    d.max_count = lp.max_count;
    d.eps2 = lp.eps2;
    d.flags = lp.flags;
    d.want_err = lp.want_err;
    d.min_eig = lp.min_eig;
#define SVO_LK_CASE(R) \
    case R: return launch_rpg<R>(prev, next, prev_xy, next_xy, status, err, iters, n, d, st);
    switch (rpg) {
        SVO_LK_CASE(1) SVO_LK_CASE(2) SVO_LK_CASE(3) SVO_LK_CASE(4) SVO_LK_CASE(5) SVO_LK_CASE(6)
        SVO_LK_CASE(7) SVO_LK_CASE(8) SVO_LK_CASE(9) SVO_LK_CASE(10) SVO_LK_CASE(11) SVO_LK_CASE(12)
        SVO_LK_CASE(14) SVO_LK_CASE(16)
        default:
            break;
    }
#undef SVO_LK_CASE
    // uncommon strip heights: round up to the next instantiated size
    if (rpg <= 13) return launch_rpg<14>(prev, next, prev_xy, next_xy, status, err, iters, n, d, st);
    if (rpg <= 16) return launch_rpg<16>(prev, next, prev_xy, next_xy, status, err, iters, n, d, st);
    return launch_rpg<32>(prev, next, prev_xy, next_xy, status, err, iters, n, d, st);
}

}  // namespace svo
