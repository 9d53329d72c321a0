/*
 * Oracle (TEST INFRASTRUCTURE ONLY -- see svo_oracle.h; parity unpinned).
 * Restates OpenCV 4.x modules/imgproc/src/pyramids.cpp (pyrDown_, 8U, REFLECT_101)
 * and modules/video/src/lkpyramid.cpp (buildOpticalFlowPyramid, calcSharrDeriv),
 * as reached from the reference's cv::calcOpticalFlowPyrLK calls at
 * R:src/tracking.cpp:101-105 and :160-165.
 */
#include "svo_oracle.h"
#include "oracle_internal.h"

#include <stdlib.h>
#include <string.h>

/* core/src/copy.cpp borderInterpolate, BORDER_REFLECT_101 */
int svo_oracle_reflect101(int p, int len)
{
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        if (p < 0) p = -p - 1 + 1;
        else p = len - 1 - (p - len) - 1;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

/* pyrDown_<FixPtCast<uchar,8>>: separable 1-4-6-4-1, exact integer sums, so
 * the row/column order of OpenCV's two passes does not matter. */
void svo_oracle_pyr_down(const uint8_t* src, int w, int h, int sstride,
                         uint8_t* dst, int dstride)
{
    static const int k[5] = {1, 4, 6, 4, 1};
    int dw = (w + 1) / 2, dh = (h + 1) / 2;
    int* rowbuf = (int*)malloc(sizeof(int) * 5 * (size_t)dw);
    for (int dy = 0; dy < dh; dy++) {
        /* horizontal pass on the 5 source rows this output row needs */
        for (int r = 0; r < 5; r++) {
            const uint8_t* s = src + (size_t)svo_oracle_reflect101(2 * dy + r - 2, h) * sstride;
            int* o = rowbuf + (size_t)r * dw;
            for (int dx = 0; dx < dw; dx++) {
                int acc = 0;
                for (int j = 0; j < 5; j++) acc += k[j] * s[svo_oracle_reflect101(2 * dx + j - 2, w)];
                o[dx] = acc;
            }
        }
        uint8_t* d = dst + (size_t)dy * dstride;
        for (int dx = 0; dx < dw; dx++) {
            int acc = 0;
            for (int r = 0; r < 5; r++) acc += k[r] * rowbuf[(size_t)r * dw + dx];
            int v = (acc + 128) >> 8;
            d[dx] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
        }
    }
    free(rowbuf);
}

/* buildOpticalFlowPyramid: level l+1 = pyrDown(level l); stop early once the
 * next size would be <= the window (returns the level reached). */
int svo_oracle_pyramid_levels(int w, int h, int win_w, int win_h, int max_level,
                              int* lw, int* lh)
{
    int sw = w, sh = h;
    for (int level = 0; level <= max_level; level++) {
        lw[level] = sw;
        lh[level] = sh;
        sw = (sw + 1) / 2;
        sh = (sh + 1) / 2;
        if (sw <= win_w || sh <= win_h) return level;
    }
    return max_level;
}

int svo_oracle_build_pyramid(const uint8_t* img, int w, int h, int stride,
                             int win_w, int win_h, int max_level, uint8_t* out)
{
    int lw[32], lh[32];
    if (max_level < 0 || max_level > 30) return -1;
    int ml = svo_oracle_pyramid_levels(w, h, win_w, win_h, max_level, lw, lh);
    uint8_t* cur = out;
    for (int y = 0; y < h; y++) memcpy(cur + (size_t)y * w, img + (size_t)y * stride, (size_t)w);
    for (int l = 1; l <= ml; l++) {
        uint8_t* nxt = cur + (size_t)lw[l - 1] * lh[l - 1];
        svo_oracle_pyr_down(cur, lw[l - 1], lh[l - 1], lw[l - 1], nxt, lw[l]);
        cur = nxt;
    }
    return ml;
}

/* lkpyramid.cpp calcSharrDeriv: vertical [3 10 3]/[-1 0 1] with row reflect-101,
 * horizontal with column reflect-101, int16 interleaved (Ix, Iy). */
void svo_oracle_scharr(const uint8_t* src, int w, int h, int stride, int16_t* dst)
{
    int* t0 = (int*)malloc(sizeof(int) * (size_t)(w + 2));
    int* t1 = (int*)malloc(sizeof(int) * (size_t)(w + 2));
    for (int y = 0; y < h; y++) {
        const uint8_t* s0 = src + (size_t)(y > 0 ? y - 1 : (h > 1 ? 1 : 0)) * stride;
        const uint8_t* s1 = src + (size_t)y * stride;
        const uint8_t* s2 = src + (size_t)(y < h - 1 ? y + 1 : (h > 1 ? h - 2 : 0)) * stride;
        for (int x = 0; x < w; x++) {
            t0[x + 1] = (int16_t)((s0[x] + s2[x]) * 3 + s1[x] * 10);
            t1[x + 1] = (int16_t)(s2[x] - s0[x]);
        }
        int x0 = w > 1 ? 1 : 0, x1 = w > 1 ? w - 2 : 0;
        t0[0] = t0[x0 + 1]; t0[w + 1] = t0[x1 + 1];
        t1[0] = t1[x0 + 1]; t1[w + 1] = t1[x1 + 1];
        int16_t* d = dst + (size_t)y * w * 2;
        for (int x = 0; x < w; x++) {
            d[2 * x] = (int16_t)(t0[x + 2] - t0[x]);
            d[2 * x + 1] = (int16_t)((t1[x + 2] + t1[x]) * 3 + t1[x + 1] * 10);
        }
    }
    free(t0);
    free(t1);
}
