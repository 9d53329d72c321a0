// ORB detection kernels: the reference's shipped default
// detector is cv::ORB (use_orb: 1, R:configs/config.yaml:20-27, created at
// R:src/tracking.cpp:33-50, used through detect() at :82 -- keypoints only, no
// descriptors). Two kernels of the path live here; FAST per level reuses
// fast.hip and the per-level selection runs on the host (orb.cpp).
//
//  * orb_resize_kernel: one pyramid level of ORB's scale pyramid, cv::resize(
//    prev, cur, sz, 0, 0, INTER_LINEAR_EXACT) (imgproc resize.cpp
//    resize_bitExact / interpolationLinear / hlineResizeCn / vlineResize) --
//    exact integer arithmetic on 8-bit fixed-point coefficients the host
//    computes per row/column: h = c0 p0 + c1 p1 (8 fractional bits), out =
//    (c0y h0 + c1y h1 + 2^15) >> 16. Taps that fall outside the source use
//    the edge pixel with weight 256 (OpenCV's dst_min/dst_max clamping). The
//    mask pyramid goes through the same resize and then
//    threshold(254, THRESH_TOZERO), i.e. 255 stays 255, anything else is 0.
//  * orb_harris_kernel: HarrisResponses(img, layerinfo, pts, 7, 0.04f) of
//    features2d orb.cpp for every FAST keypoint of every level (the response
//    of a point does not depend on which other points survive, so scoring the
//    superset keeps the GPU off the host's selection loop).
//
// Both are small byte-gather kernels; the level images are L2-resident.
#include "common.hpp"
#include "orb.hpp"

namespace svo {

// Packed coefficient pair: c0 | c1 << 16 (each in 0..256).
__device__ __forceinline__ void orb_resize_px(const uint8_t* __restrict__ src, int spitch,
                                              const uint8_t* __restrict__ smask, int sw, uint8_t* __restrict__ dst,
                                              int dpitch, uint8_t* __restrict__ dmask, int dw, int x, int y,
                                              const int* __restrict__ xofs, const uint32_t* __restrict__ xc,
                                              const int* __restrict__ yofs, const uint32_t* __restrict__ yc) {
    const int x0 = xofs[x], y0 = yofs[y];
    const uint32_t cx = xc[x], cy = yc[y];
    const uint32_t cx0 = cx & 0xFFFF, cx1 = cx >> 16, cy0 = cy & 0xFFFF, cy1 = cy >> 16;
    // a zero weight may name a tap one past the edge: clamp the address, not the value
    const int x1 = cx1 ? x0 + 1 : x0;
    const uint8_t* r0 = src + (size_t)y0 * spitch;
    const uint8_t* r1 = cy1 ? r0 + spitch : r0;
    const uint32_t h0 = r0[x0] * cx0 + r0[x1] * cx1;
    const uint32_t h1 = r1[x0] * cx0 + r1[x1] * cx1;
    dst[(size_t)y * dpitch + x] = (uint8_t)((h0 * cy0 + h1 * cy1 + 32768u) >> 16);
    if (dmask) {
        const uint8_t* m0 = smask + (size_t)y0 * sw;
        const uint8_t* m1 = cy1 ? m0 + sw : m0;
        const uint32_t g0 = m0[x0] * cx0 + m0[x1] * cx1;
        const uint32_t g1 = m1[x0] * cx0 + m1[x1] * cx1;
        const uint32_t v = (g0 * cy0 + g1 * cy1 + 32768u) >> 16;
        dmask[(size_t)y * dw + x] = v > 254u ? 255 : 0;
    }
}

__global__ void __launch_bounds__(256) orb_resize_kernel(const uint8_t* __restrict__ src, int spitch,
                                                         const uint8_t* __restrict__ smask, int sw,
                                                         uint8_t* __restrict__ dst, int dpitch,
                                                         uint8_t* __restrict__ dmask, int dw, int dh,
                                                         const int* __restrict__ xofs,
                                                         const uint32_t* __restrict__ xc,
                                                         const int* __restrict__ yofs,
                                                         const uint32_t* __restrict__ yc) {
    const int x = blockIdx.x * 64 + threadIdx.x;
    const int y = blockIdx.y * 4 + threadIdx.y;
    if (x >= dw || y >= dh) return;
    orb_resize_px(src, spitch, smask, sw, dst, dpitch, dmask, dw, x, y, xofs, xc, yofs, yc);
}

// the same for one level of every sequence (blockIdx.z)
__global__ void __launch_bounds__(256) orb_resize_batched_kernel(const PyrDesc* __restrict__ src,
                                                                 const PyrDesc* __restrict__ dst,
                                                                 const uint8_t* __restrict__ smask,
                                                                 size_t smask_stride, int sw,
                                                                 uint8_t* __restrict__ dmask, size_t dmask_stride,
                                                                 int dw, int dh, const int* __restrict__ xofs,
                                                                 const uint32_t* __restrict__ xc,
                                                                 const int* __restrict__ yofs,
                                                                 const uint32_t* __restrict__ yc) {
    const int x = blockIdx.x * 64 + threadIdx.x;
    const int y = blockIdx.y * 4 + threadIdx.y;
    if (x >= dw || y >= dh) return;
    const size_t s = blockIdx.z;
    const ImgLevel S = src[s].lv[0], D = dst[s].lv[0];
    orb_resize_px(S.data, S.pitch, dmask ? smask + s * smask_stride : nullptr, sw, const_cast<uint8_t*>(D.data),
                  D.pitch, dmask ? dmask + s * dmask_stride : nullptr, dw, x, y, xofs, xc, yofs, yc);
}

hipError_t launch_orb_resize(const uint8_t* src, int spitch, const uint8_t* smask, int sw, uint8_t* dst, int dpitch,
                             uint8_t* dmask, int dw, int dh, const int* xofs, const uint32_t* xc, const int* yofs,
                             const uint32_t* yc, hipStream_t st) {
    if (dw <= 0 || dh <= 0) return hipSuccess;
    dim3 grid((dw + 63) / 64, (dh + 3) / 4);
    hipLaunchKernelGGL(orb_resize_kernel, grid, dim3(64, 4), 0, st, src, spitch, smask, sw, dst, dpitch, dmask, dw,
                       dh, xofs, xc, yofs, yc);
    return hipGetLastError();
}

// HarrisResponses (orb.cpp: block 7, k 0.04) at integer point (x0, y0) of level L.
// Points closer than 4 px to the level's edge (never kept by ORB's border filter,
// which is >= edgeThreshold) get response 0 instead of a read.
__device__ float orb_harris_at(const ImgLevel& L, const svo_keypoint& k) {
    // cvRound of integer-valued coordinates
    const int x0 = (int)k.x, y0 = (int)k.y;
    float r = 0.f;
    constexpr int B = 7, R = B / 2;
    if (x0 - R - 1 >= 0 && y0 - R - 1 >= 0 && x0 + R + 1 < L.w && y0 + R + 1 < L.h) {
        const int step = L.pitch;
        const uint8_t* p0 = L.data + (size_t)(y0 - R) * step + (x0 - R);
        int a = 0, b = 0, c = 0;
        for (int yy = 0; yy < B; yy++) {
            const uint8_t* q = p0 + yy * step;
            for (int xx = 0; xx < B; xx++) {
                const uint8_t* p = q + xx;
                const int Ix = (p[1] - p[-1]) * 2 + (p[-step + 1] - p[-step - 1]) + (p[step + 1] - p[step - 1]);
                const int Iy = (p[step] - p[-step]) * 2 + (p[step - 1] - p[-step - 1]) + (p[step + 1] - p[-step + 1]);
                a += Ix * Ix;
                b += Iy * Iy;
                c += Ix * Iy;
            }
        }
        // float expression of orb.cpp HarrisResponses, evaluated op by op
        const float scale = 1.f / ((1 << 2) * B * 255.f);
        const float s2 = scale * scale;
        const float scale_sq_sq = s2 * scale * scale;
        const float fa = (float)a, fb = (float)b, fc = (float)c;
        const float k004 = 0.04f;
        const float t0 = fa * fb;
        const float t1 = fc * fc;
        const float sab = fa + fb;
        const float t2 = k004 * sab;
        const float t3 = t2 * sab;
        r = ((t0 - t1) - t3) * scale_sq_sq;
    }
    return r;
}

// Per level l: image lv[l] of `levels`, keypoints kps + l*cap (n[l] of them).
__global__ void __launch_bounds__(256) orb_harris_kernel(PyrDesc levels, const svo_keypoint* __restrict__ kps,
                                                         const int* __restrict__ n, int cap,
                                                         float* __restrict__ resp) {
    const int l = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int nl = n[l] < cap ? n[l] : cap;
    if (i >= nl) return;
    resp[(size_t)l * cap + i] = orb_harris_at(levels.lv[l], kps[(size_t)l * cap + i]);
}

// every sequence (blockIdx.z): level l of sequence s is levels[l * nseq + s].lv[0]
__global__ void __launch_bounds__(256) orb_harris_batched_kernel(const PyrDesc* __restrict__ levels, int nseq,
                                                                 const svo_keypoint* __restrict__ kps,
                                                                 const int* __restrict__ n, int cap,
                                                                 float* __restrict__ resp) {
    const size_t ls = (size_t)blockIdx.y * nseq + blockIdx.z;
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int nl = n[ls] < cap ? n[ls] : cap;
    if (i >= nl) return;
    resp[ls * cap + i] = orb_harris_at(levels[ls].lv[0], kps[ls * cap + i]);
}

hipError_t launch_orb_harris(const PyrDesc& levels, int nlevels, const svo_keypoint* kps, const int* n, int cap,
                             int max_n, float* resp, hipStream_t st) {
    if (max_n <= 0 || nlevels <= 0) return hipSuccess;
    dim3 grid((max_n + 255) / 256, nlevels);
    hipLaunchKernelGGL(orb_harris_kernel, grid, dim3(256), 0, st, levels, kps, n, cap, resp);
    return hipGetLastError();
}

hipError_t launch_orb_harris_batched(const PyrDesc* levels, int nlevels, int nseq, const svo_keypoint* kps,
                                     const int* n, int cap, int max_n, float* resp, hipStream_t st) {
    if (max_n <= 0 || nlevels <= 0 || nseq <= 0) return hipSuccess;
    dim3 grid((max_n + 255) / 256, nlevels, nseq);
    hipLaunchKernelGGL(orb_harris_batched_kernel, grid, dim3(256), 0, st, levels, nseq, kps, n, cap, resp);
    return hipGetLastError();
}

hipError_t launch_orb_resize_batched(const PyrDesc* src, const PyrDesc* dst, const uint8_t* smask,
                                     size_t smask_stride, int sw, uint8_t* dmask, size_t dmask_stride, int dw, int dh,
                                     int nseq, const int* xofs, const uint32_t* xc, const int* yofs,
                                     const uint32_t* yc, hipStream_t st) {
    if (dw <= 0 || dh <= 0 || nseq <= 0) return hipSuccess;
    dim3 grid((dw + 63) / 64, (dh + 3) / 4, nseq);
    hipLaunchKernelGGL(orb_resize_batched_kernel, grid, dim3(64, 4), 0, st, src, dst, smask, smask_stride, sw, dmask,
                       dmask_stride, dw, dh, xofs, xc, yofs, yc);
    return hipGetLastError();
}

}  // namespace svo
