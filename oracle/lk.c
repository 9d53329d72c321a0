/*
 * Oracle (TEST INFRASTRUCTURE ONLY -- see svo_oracle.h; parity unpinned).
 *
 * Restates OpenCV 4.x modules/video/src/lkpyramid.cpp:
 *   SparsePyrLKOpticalFlowImpl::calc  -- criteria clamping, pyramid build, level loop
 *   cv::detail::LKTrackerInvoker::operator() -- per-point fixed-point tracker
 * as called by the reference at R:src/tracking.cpp:101-105 (stereo: 11x11,
 * maxLevel 3, {COUNT+EPS, 30, 1e-3}, flags 0) and :160-165 (temporal: 21x21,
 * maxLevel 3, {COUNT+EPS, 50, 1e-3}, OPTFLOW_LK_GET_MIN_EIGENVALS).
 *
 * The pyramid levels are padded by the window with BORDER_REFLECT_101 and the
 * Scharr derivative levels with BORDER_CONSTANT 0, exactly as OpenCV stores them.
 */
#include "svo_oracle.h"
#include "oracle_internal.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define W_BITS 14
#define W_BITS1 14
#define FLT_SCALE (1.f / (1 << 20))
#define DESCALE(x, n) (((x) + (1 << ((n)-1))) >> (n))

typedef struct {
    int w, h, pw, ph, bx, by; /* level size, padded size, border */
    uint8_t* img;             /* padded u8 image, stride pw */
    int16_t* der;             /* padded (Ix,Iy) int16, stride 2*pw (prev only) */
} level_t;

static void make_padded(level_t* L, const uint8_t* src, int w, int h, int bx, int by)
{
    L->w = w; L->h = h; L->bx = bx; L->by = by;
    L->pw = w + 2 * bx; L->ph = h + 2 * by;
    L->img = (uint8_t*)malloc((size_t)L->pw * L->ph);
    for (int y = 0; y < L->ph; y++) {
        int sy = svo_oracle_reflect101(y - by, h);
        for (int x = 0; x < L->pw; x++)
            L->img[(size_t)y * L->pw + x] = src[(size_t)sy * w + svo_oracle_reflect101(x - bx, w)];
    }
    L->der = NULL;
}

static void make_deriv(level_t* L, const uint8_t* src)
{
    int16_t* d = (int16_t*)malloc(sizeof(int16_t) * 2 * (size_t)L->w * L->h);
    svo_oracle_scharr(src, L->w, L->h, L->w, d);
    L->der = (int16_t*)calloc((size_t)L->pw * L->ph * 2, sizeof(int16_t));
    for (int y = 0; y < L->h; y++)
        memcpy(L->der + ((size_t)(y + L->by) * L->pw + L->bx) * 2, d + (size_t)y * L->w * 2,
               sizeof(int16_t) * 2 * (size_t)L->w);
    free(d);
}

static inline const uint8_t* img_at(const level_t* L, int x, int y)
{
    return L->img + (size_t)(y + L->by) * L->pw + (x + L->bx);
}
static inline const int16_t* der_at(const level_t* L, int x, int y)
{
    return L->der + ((size_t)(y + L->by) * L->pw + (x + L->bx)) * 2;
}

/* one LKTrackerInvoker pass for one point at one level */
static void track_point(const level_t* I, const level_t* J, int ptidx, const float* prevPts,
                        float* nextPts, uint8_t* status, float* err, int winW, int winH,
                        int maxCount, double epsilon, int level, int maxLevel, int flags,
                        float minEigThreshold, int acc, int16_t* IWin, int16_t* dIWin, int* iters)
{
    const float halfWx = (winW - 1) * 0.5f, halfWy = (winH - 1) * 0.5f;
    const float lscale = (float)(1. / (1 << level));
    float prevx = prevPts[2 * ptidx] * lscale, prevy = prevPts[2 * ptidx + 1] * lscale;
    float nextx, nexty;
    if (level == maxLevel) {
        if (flags & SVO_ORACLE_LK_USE_INITIAL_FLOW) {
            nextx = nextPts[2 * ptidx] * lscale;
            nexty = nextPts[2 * ptidx + 1] * lscale;
        } else {
            nextx = prevx;
            nexty = prevy;
        }
    } else {
        nextx = nextPts[2 * ptidx] * 2.f;
        nexty = nextPts[2 * ptidx + 1] * 2.f;
    }
    nextPts[2 * ptidx] = nextx;
    nextPts[2 * ptidx + 1] = nexty;

    prevx -= halfWx;
    prevy -= halfWy;
    int ipx = ora_floor_f(prevx), ipy = ora_floor_f(prevy);
    if (ipx < -winW || ipx >= I->w || ipy < -winH || ipy >= I->h) {
        if (level == 0) {
            status[ptidx] = 0;
            if (err) err[ptidx] = 0;
        }
        return;
    }

    float a = prevx - ipx, b = prevy - ipy;
    int iw00 = ora_round_f((1.f - a) * (1.f - b) * (1 << W_BITS));
    int iw01 = ora_round_f(a * (1.f - b) * (1 << W_BITS));
    int iw10 = ora_round_f((1.f - a) * b * (1 << W_BITS));
    int iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;

    /* ---- patch extraction + covariance ---- */
    int64_t eA11 = 0, eA12 = 0, eA22 = 0;   /* EXACT */
    float sA11 = 0, sA12 = 0, sA22 = 0;     /* SCALAR / SSE tail */
    float qA11[4] = {0, 0, 0, 0}, qA12[4] = {0, 0, 0, 0}, qA22[4] = {0, 0, 0, 0};
    const int simd_end4 = (acc == SVO_ORACLE_ACC_SSE) ? ((winW >= 4) ? ((winW - 4) / 4 + 1) * 4 : 0) : 0;
    for (int y = 0; y < winH; y++) {
        const uint8_t* s0 = img_at(I, ipx, ipy + y);
        const uint8_t* s1 = img_at(I, ipx, ipy + y + 1);
        const int16_t* d0 = der_at(I, ipx, ipy + y);
        const int16_t* d1 = der_at(I, ipx, ipy + y + 1);
        for (int x = 0; x < winW; x++) {
            int ival = DESCALE(s0[x] * iw00 + s0[x + 1] * iw01 + s1[x] * iw10 + s1[x + 1] * iw11, W_BITS1 - 5);
            int ixval = DESCALE(d0[2 * x] * iw00 + d0[2 * x + 2] * iw01 + d1[2 * x] * iw10 + d1[2 * x + 2] * iw11, W_BITS1);
            int iyval = DESCALE(d0[2 * x + 1] * iw00 + d0[2 * x + 3] * iw01 + d1[2 * x + 1] * iw10 + d1[2 * x + 3] * iw11, W_BITS1);
            IWin[y * winW + x] = (int16_t)ival;
            dIWin[2 * (y * winW + x)] = (int16_t)ixval;
            dIWin[2 * (y * winW + x) + 1] = (int16_t)iyval;
            if (acc == SVO_ORACLE_ACC_EXACT) {
                eA11 += (int64_t)ixval * ixval;
                eA12 += (int64_t)ixval * iyval;
                eA22 += (int64_t)iyval * iyval;
            } else if (acc == SVO_ORACLE_ACC_SSE && x < simd_end4) {
                int k = x & 3;
                float fx = (float)ixval, fy = (float)iyval;
                /* v_muladd without FMA: mul then add (order in source: A22, A12, A11) */
                qA22[k] = fy * fy + qA22[k];
                qA12[k] = fx * fy + qA12[k];
                qA11[k] = fx * fx + qA11[k];
            } else {
                sA11 += (float)(ixval * ixval);
                sA12 += (float)(ixval * iyval);
                sA22 += (float)(iyval * iyval);
            }
        }
    }
    float A11, A12, A22;
    if (acc == SVO_ORACLE_ACC_EXACT) {
        A11 = (float)eA11 * FLT_SCALE;
        A12 = (float)eA12 * FLT_SCALE;
        A22 = (float)eA22 * FLT_SCALE;
    } else {
        if (acc == SVO_ORACLE_ACC_SSE) {
            sA11 += (qA11[0] + qA11[2]) + (qA11[1] + qA11[3]);
            sA12 += (qA12[0] + qA12[2]) + (qA12[1] + qA12[3]);
            sA22 += (qA22[0] + qA22[2]) + (qA22[1] + qA22[3]);
        }
        A11 = sA11 * FLT_SCALE;
        A12 = sA12 * FLT_SCALE;
        A22 = sA22 * FLT_SCALE;
    }

    float D = A11 * A22 - A12 * A12;
    float minEig = (A22 + A11 - sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) /
                   (float)(2 * winW * winH);
    if (err && (flags & SVO_ORACLE_LK_GET_MIN_EIGENVALS) != 0) err[ptidx] = minEig;
    if (minEig < minEigThreshold || D < FLT_EPSILON) {
        if (level == 0) status[ptidx] = 0;
        return;
    }
    D = 1.f / D;

    nextx -= halfWx;
    nexty -= halfWy;
    float pdx = 0.f, pdy = 0.f;
    const int simd_end8 = (acc == SVO_ORACLE_ACC_SSE) ? ((winW >= 8) ? ((winW - 8) / 8 + 1) * 8 : 0) : 0;
    for (int j = 0; j < maxCount; j++) {
        int inx = ora_floor_f(nextx), iny = ora_floor_f(nexty);
        if (inx < -winW || inx >= J->w || iny < -winH || iny >= J->h) {
            if (level == 0) status[ptidx] = 0;
            break;
        }
        if (iters) iters[ptidx]++;
        a = nextx - inx;
        b = nexty - iny;
        iw00 = ora_round_f((1.f - a) * (1.f - b) * (1 << W_BITS));
        iw01 = ora_round_f(a * (1.f - b) * (1 << W_BITS));
        iw10 = ora_round_f((1.f - a) * b * (1 << W_BITS));
        iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;
        int64_t eb1 = 0, eb2 = 0;
        float sb1 = 0, sb2 = 0;
        float qb0[4] = {0, 0, 0, 0}, qb1[4] = {0, 0, 0, 0};
        for (int y = 0; y < winH; y++) {
            const uint8_t* j0 = img_at(J, inx, iny + y);
            const uint8_t* j1 = img_at(J, inx, iny + y + 1);
            const int16_t* Ip = IWin + y * winW;
            const int16_t* dIp = dIWin + 2 * y * winW;
            int x = 0;
            if (acc == SVO_ORACLE_ACC_SSE) {
                for (; x < simd_end8; x += 8) {
                    int d[8];
                    for (int t = 0; t < 8; t++)
                        d[t] = DESCALE(j0[x + t] * iw00 + j0[x + t + 1] * iw01 + j1[x + t] * iw10 +
                                           j1[x + t + 1] * iw11, W_BITS1 - 5) - Ip[x + t];
                    const int16_t* g = dIp + 2 * x;
                    /* v_dotprod pairs (exact int32) -> v_cvt_f32 -> lane add */
                    qb0[0] += (float)(d[0] * g[0] + d[4] * g[8]);
                    qb0[1] += (float)(d[0] * g[1] + d[4] * g[9]);
                    qb0[2] += (float)(d[1] * g[2] + d[5] * g[10]);
                    qb0[3] += (float)(d[1] * g[3] + d[5] * g[11]);
                    qb1[0] += (float)(d[2] * g[4] + d[6] * g[12]);
                    qb1[1] += (float)(d[2] * g[5] + d[6] * g[13]);
                    qb1[2] += (float)(d[3] * g[6] + d[7] * g[14]);
                    qb1[3] += (float)(d[3] * g[7] + d[7] * g[15]);
                }
            }
            for (; x < winW; x++) {
                int diff = DESCALE(j0[x] * iw00 + j0[x + 1] * iw01 + j1[x] * iw10 + j1[x + 1] * iw11,
                                   W_BITS1 - 5) - Ip[x];
                if (acc == SVO_ORACLE_ACC_EXACT) {
                    eb1 += (int64_t)diff * dIp[2 * x];
                    eb2 += (int64_t)diff * dIp[2 * x + 1];
                } else {
                    sb1 += (float)(diff * dIp[2 * x]);
                    sb2 += (float)(diff * dIp[2 * x + 1]);
                }
            }
        }
        float b1, b2;
        if (acc == SVO_ORACLE_ACC_EXACT) {
            b1 = (float)eb1 * FLT_SCALE;
            b2 = (float)eb2 * FLT_SCALE;
        } else {
            if (acc == SVO_ORACLE_ACC_SSE) {
                float s0 = qb0[0] + qb1[0], s1 = qb0[1] + qb1[1];
                float s2 = qb0[2] + qb1[2], s3 = qb0[3] + qb1[3];
                sb1 += (s0 + 0.f) + (s2 + 0.f);
                sb2 += (s1 + 0.f) + (s3 + 0.f);
            }
            b1 = sb1 * FLT_SCALE;
            b2 = sb2 * FLT_SCALE;
        }
        float dx = (float)((A12 * b2 - A22 * b1) * D);
        float dy = (float)((A12 * b1 - A11 * b2) * D);
        nextx += dx;
        nexty += dy;
        nextPts[2 * ptidx] = nextx + halfWx;
        nextPts[2 * ptidx + 1] = nexty + halfWy;
        if ((double)dx * dx + (double)dy * dy <= epsilon) break;
        if (j > 0 && fabs((double)fabsf(dx + pdx)) < 0.01 && fabs((double)fabsf(dy + pdy)) < 0.01) {
            nextPts[2 * ptidx] -= dx * 0.5f;
            nextPts[2 * ptidx + 1] -= dy * 0.5f;
            break;
        }
        pdx = dx;
        pdy = dy;
    }

    if (status[ptidx] && err && level == 0 && (flags & SVO_ORACLE_LK_GET_MIN_EIGENVALS) == 0) {
        float npx = nextPts[2 * ptidx] - halfWx, npy = nextPts[2 * ptidx + 1] - halfWy;
        int ix = ora_floor_f(npx), iy = ora_floor_f(npy);
        if (ix < -winW || ix >= J->w || iy < -winH || iy >= J->h) {
            status[ptidx] = 0;
            return;
        }
        float aa = npx - ix, bb = npy - iy;
        iw00 = ora_round_f((1.f - aa) * (1.f - bb) * (1 << W_BITS));
        iw01 = ora_round_f(aa * (1.f - bb) * (1 << W_BITS));
        iw10 = ora_round_f((1.f - aa) * bb * (1 << W_BITS));
        iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;
        float errval = 0.f;
        for (int y = 0; y < winH; y++) {
            const uint8_t* j0 = img_at(J, ix, iy + y);
            const uint8_t* j1 = img_at(J, ix, iy + y + 1);
            const int16_t* Ip = IWin + y * winW;
            for (int x = 0; x < winW; x++) {
                int diff = DESCALE(j0[x] * iw00 + j0[x + 1] * iw01 + j1[x] * iw10 + j1[x + 1] * iw11,
                                   W_BITS1 - 5) - Ip[x];
                errval += fabsf((float)diff);
            }
        }
        err[ptidx] = errval * 1.f / (float)(32 * winW * winH);
    }
}

int svo_oracle_lk(const uint8_t* prev, const uint8_t* next, int w, int h, int stride,
                  const float* prev_xy, float* next_xy, uint8_t* status, float* err,
                  int npts, int win_w, int win_h, int max_level,
                  int crit_type, int max_count, double epsilon,
                  int flags, double min_eig_threshold, int acc_mode, int* iters_out)
{
    if (max_level < 0 || win_w <= 2 || win_h <= 2 || max_level > 30) return -1;
    if (npts <= 0) return max_level;
    /* SparsePyrLKOpticalFlowImpl::calc criteria clamping */
    if ((crit_type & SVO_ORACLE_TERM_COUNT) == 0) max_count = 30;
    else max_count = max_count < 0 ? 0 : max_count > 100 ? 100 : max_count;
    if ((crit_type & SVO_ORACLE_TERM_EPS) == 0) epsilon = 0.01;
    else epsilon = epsilon < 0. ? 0. : epsilon > 10. ? 10. : epsilon;
    epsilon *= epsilon;
    /* SVO_ORACLE_LEVEL_ITERS: iters_out holds (max_level + 1) x npts counts, one row per level */
    const int per_level = (acc_mode & SVO_ORACLE_LEVEL_ITERS) != 0;
    acc_mode &= ~SVO_ORACLE_LEVEL_ITERS;

    for (int i = 0; i < npts; i++) status[i] = 1;

    int lw[32], lh[32];
    int ml = svo_oracle_pyramid_levels(w, h, win_w, win_h, max_level, lw, lh);
    if (iters_out) memset(iters_out, 0, sizeof(int) * (size_t)npts * (per_level ? (size_t)(max_level + 1) : 1));
    size_t total = 0;
    for (int l = 0; l <= ml; l++) total += (size_t)lw[l] * lh[l];
    uint8_t* pp = (uint8_t*)malloc(total);
    uint8_t* np = (uint8_t*)malloc(total);
    svo_oracle_build_pyramid(prev, w, h, stride, win_w, win_h, ml, pp);
    svo_oracle_build_pyramid(next, w, h, stride, win_w, win_h, ml, np);

    size_t off = total;
    for (int level = ml; level >= 0; level--) {
        off -= (size_t)lw[level] * lh[level];
        level_t I, J;
        make_padded(&I, pp + off, lw[level], lh[level], win_w, win_h);
        make_padded(&J, np + off, lw[level], lh[level], win_w, win_h);
        make_deriv(&I, pp + off);
        /* cv::parallel_for_ over points (LKTrackerInvoker): points are independent */
#pragma omp parallel
        {
            int16_t* IWin = (int16_t*)malloc(sizeof(int16_t) * (size_t)win_w * win_h);
            int16_t* dIWin = (int16_t*)malloc(sizeof(int16_t) * 2 * (size_t)win_w * win_h);
#pragma omp for schedule(dynamic, 64)
            for (int i = 0; i < npts; i++)
                track_point(&I, &J, i, prev_xy, next_xy, status, err, win_w, win_h, max_count, epsilon,
                            level, ml, flags, (float)min_eig_threshold, acc_mode, IWin, dIWin,
                            iters_out && per_level ? iters_out + (size_t)level * npts : iters_out);
            free(IWin);
            free(dIWin);
        }
        free(I.img); free(I.der); free(J.img);
    }
    free(pp); free(np);
    return ml;
}

/* Host threads of the LK point loop (OpenMP; OpenCV's parallel_for_). */
#include <omp.h>
void svo_oracle_set_threads(int n)
{
    omp_set_num_threads(n > 0 ? n : 1);
}
