/*
 * Oracle (TEST INFRASTRUCTURE ONLY -- see svo_oracle.h; parity unpinned).
 *
 * Restates OpenCV 4.x modules/features2d/src/fast.cpp (FAST_t<16>, makeOffsets),
 * fast_score.cpp (cornerScore<16>) and keypoint.cpp (KeyPointsFilter::
 * runByPixelsMask), reached from cv::FastFeatureDetector::detect at
 * R:src/tracking.cpp:82 (created at :54-57 with threshold / nonmaxSuppression
 * from R:include/config_reader.h:35-38), plus the mask rectangles drawn at
 * R:src/tracking.cpp:76-79 (imgproc/src/drawing.cpp rectangle, FILLED).
 */
#include "svo_oracle.h"
#include "oracle_internal.h"

#include <stdlib.h>
#include <string.h>

static const int offsets16[16][2] = {
    {0, 3}, {1, 3}, {2, 2}, {3, 1}, {3, 0}, {3, -1}, {2, -2}, {1, -3},
    {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

static void make_offsets(int pixel[25], int stride)
{
    int k;
    for (k = 0; k < 16; k++) pixel[k] = offsets16[k][0] + offsets16[k][1] * stride;
    for (; k < 25; k++) pixel[k] = pixel[k - 16];
}

static int imin(int a, int b) { return a < b ? a : b; }
static int imax(int a, int b) { return a > b ? a : b; }

/* cornerScore<16> */
static int corner_score16(const uint8_t* ptr, const int pixel[25], int threshold)
{
    const int K = 8, N = K * 3 + 1;
    int k, v = ptr[0];
    short d[25];
    for (k = 0; k < N; k++) d[k] = (short)(v - ptr[pixel[k]]);
    int a0 = threshold;
    for (k = 0; k < 16; k += 2) {
        int a = imin(d[k + 1], d[k + 2]);
        a = imin(a, d[k + 3]);
        if (a <= a0) continue;
        a = imin(a, d[k + 4]);
        a = imin(a, d[k + 5]);
        a = imin(a, d[k + 6]);
        a = imin(a, d[k + 7]);
        a = imin(a, d[k + 8]);
        a0 = imax(a0, imin(a, d[k]));
        a0 = imax(a0, imin(a, d[k + 9]));
    }
    int b0 = -a0;
    for (k = 0; k < 16; k += 2) {
        int b = imax(d[k + 1], d[k + 2]);
        b = imax(b, d[k + 3]);
        b = imax(b, d[k + 4]);
        b = imax(b, d[k + 5]);
        if (b >= b0) continue;
        b = imax(b, d[k + 6]);
        b = imax(b, d[k + 7]);
        b = imax(b, d[k + 8]);
        b0 = imin(b0, imax(b, d[k]));
        b0 = imin(b0, imax(b, d[k + 9]));
    }
    return -b0 - 1;
}

/* The FAST-9 segment test of FAST_t<16> for one pixel: returns 1 if corner. */
static int is_corner16(const uint8_t* ptr, const int pixel[25], int threshold, const uint8_t* tab0)
{
    const int K = 8, N = 25;
    int v = ptr[0];
    const uint8_t* tab = tab0 - v + 255;
    int d = tab[ptr[pixel[0]]] | tab[ptr[pixel[8]]];
    if (d == 0) return 0;
    d &= tab[ptr[pixel[2]]] | tab[ptr[pixel[10]]];
    d &= tab[ptr[pixel[4]]] | tab[ptr[pixel[12]]];
    d &= tab[ptr[pixel[6]]] | tab[ptr[pixel[14]]];
    if (d == 0) return 0;
    d &= tab[ptr[pixel[1]]] | tab[ptr[pixel[9]]];
    d &= tab[ptr[pixel[3]]] | tab[ptr[pixel[11]]];
    d &= tab[ptr[pixel[5]]] | tab[ptr[pixel[13]]];
    d &= tab[ptr[pixel[7]]] | tab[ptr[pixel[15]]];
    if (d & 1) {
        int vt = v - threshold, count = 0;
        for (int k = 0; k < N; k++) {
            int x = ptr[pixel[k]];
            if (x < vt) {
                if (++count > K) return 1;
            } else
                count = 0;
        }
    }
    if (d & 2) {
        int vt = v + threshold, count = 0;
        for (int k = 0; k < N; k++) {
            int x = ptr[pixel[k]];
            if (x > vt) {
                if (++count > K) return 1;
            } else
                count = 0;
        }
    }
    return 0;
}

static void make_tab(uint8_t tab[512], int threshold)
{
    for (int i = -255; i <= 255; i++)
        tab[i + 255] = (uint8_t)(i < -threshold ? 1 : i > threshold ? 2 : 0);
}

void svo_oracle_fast_score(const uint8_t* img, int w, int h, int stride, int threshold,
                           uint8_t* score, uint8_t* corner)
{
    int pixel[25];
    uint8_t tab[512];
    threshold = threshold < 0 ? 0 : threshold > 255 ? 255 : threshold;
    make_offsets(pixel, stride);
    make_tab(tab, threshold);
    memset(score, 0, (size_t)w * h);
    memset(corner, 0, (size_t)w * h);
    for (int i = 3; i < h - 3; i++)
        for (int j = 3; j < w - 3; j++) {
            const uint8_t* ptr = img + (size_t)i * stride + j;
            if (is_corner16(ptr, pixel, threshold, tab)) {
                corner[(size_t)i * w + j] = 1;
                score[(size_t)i * w + j] = (uint8_t)corner_score16(ptr, pixel, threshold);
            }
        }
}

/* FAST_t<16>: three rolling score rows, a corner in row i-1 is emitted after
 * row i is scored; NMS is a strict '>' against all 8 neighbours (non-corners
 * and rows outside 3..h-4 score 0). Then runByPixelsMask (stable). */
int svo_oracle_fast(const uint8_t* img, int w, int h, int stride, int threshold,
                    int nonmax, const uint8_t* mask, float* kp_xyr, int cap)
{
    int pixel[25];
    uint8_t tab[512];
    threshold = threshold < 0 ? 0 : threshold > 255 ? 255 : threshold;
    make_offsets(pixel, stride);
    make_tab(tab, threshold);
    if (w <= 0 || h <= 0) return 0;

    uint8_t* buf[3];
    int* cpbuf[3];
    uint8_t* bufmem = (uint8_t*)calloc((size_t)w * 3, 1);
    int* cpmem = (int*)calloc(((size_t)w + 1) * 3, sizeof(int));
    for (int k = 0; k < 3; k++) {
        buf[k] = bufmem + (size_t)k * w;
        cpbuf[k] = cpmem + (size_t)k * (w + 1) + 1;
    }
    int nkp = 0;
    for (int i = 3; i < h - 2; i++) {
        uint8_t* curr = buf[(i - 3) % 3];
        int* cornerpos = cpbuf[(i - 3) % 3];
        memset(curr, 0, (size_t)w);
        int ncorners = 0;
        if (i < h - 3) {
            for (int j = 3; j < w - 3; j++) {
                const uint8_t* ptr = img + (size_t)i * stride + j;
                if (is_corner16(ptr, pixel, threshold, tab)) {
                    cornerpos[ncorners++] = j;
                    if (nonmax) curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                }
            }
        }
        cornerpos[-1] = ncorners;
        if (i == 3) continue;
        const uint8_t* prev = buf[(i - 4 + 3) % 3];
        const uint8_t* pprev = buf[(i - 5 + 3) % 3];
        cornerpos = cpbuf[(i - 4 + 3) % 3];
        ncorners = cornerpos[-1];
        for (int k = 0; k < ncorners; k++) {
            int j = cornerpos[k];
            int score = prev[j];
            if (!nonmax || (score > prev[j + 1] && score > prev[j - 1] && score > pprev[j - 1] &&
                            score > pprev[j] && score > pprev[j + 1] && score > curr[j - 1] &&
                            score > curr[j] && score > curr[j + 1])) {
                float x = (float)j, y = (float)(i - 1);
                if (mask && mask[(size_t)(int)(y + 0.5f) * w + (int)(x + 0.5f)] == 0) continue;
                if (nkp < cap) {
                    kp_xyr[3 * nkp] = x;
                    kp_xyr[3 * nkp + 1] = y;
                    kp_xyr[3 * nkp + 2] = (float)score;
                }
                nkp++;
            }
        }
    }
    free(bufmem);
    free(cpmem);
    return nkp;
}

/* cv::rectangle(mask, pos-(half,half), pos+(half,half), 0, FILLED): the float
 * corners are converted Point2f -> Point with cvRound (saturate_cast<int>), the
 * filled rectangle covers both corners inclusively, clipped to the image. */
void svo_oracle_mask_boxes(int w, int h, const float* pts_xy, int n, float half, uint8_t* mask)
{
    memset(mask, 255, (size_t)w * h);
    for (int i = 0; i < n; i++) {
        float px = pts_xy[2 * i], py = pts_xy[2 * i + 1];
        int x0 = ora_round_f(px - half), y0 = ora_round_f(py - half);
        int x1 = ora_round_f(px + half), y1 = ora_round_f(py + half);
        if (x0 > x1) { int t = x0; x0 = x1; x1 = t; }
        if (y0 > y1) { int t = y0; y0 = y1; y1 = t; }
        if (x0 < 0) x0 = 0;
        if (y0 < 0) y0 = 0;
        if (x1 > w - 1) x1 = w - 1;
        if (y1 > h - 1) y1 = h - 1;
        for (int y = y0; y <= y1; y++)
            for (int x = x0; x <= x1; x++) mask[(size_t)y * w + x] = 0;
    }
}
