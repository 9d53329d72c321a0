// Batched two-view DLT triangulation (§8f-1): cv::triangulatePoints(P1, P2,
// pts1, pts2, points4D) + cv::convertPointsFromHomogeneous, as called by
// Tracking::triangulateNewMapPoints (R:src/tracking.cpp:125-131).
//
// Per point (one thread): A (4x4, double) has rows x*P[2]-P[0], y*P[2]-P[1]
// for each view (OpenCV triangulate.cpp); the homogeneous point is A's right
// singular vector of the smallest singular value, found here by a one-sided
// Jacobi SVD held entirely in registers (fixed 4x4, fully unrolled). The vector
// is normalised to unit length with w >= 0 (OpenCV's sign is its SVD's; it
// cancels in the division), rounded to float like points4D (CV_32F), and
// divided by w in float (convertPointsFromHomogeneous).
// Work per point: ~1.5k DP flops; bytes: 16 in + 28 out.
#include "common.hpp"
#include "dlt.hpp"

namespace svo {

namespace {

__global__ __launch_bounds__(256) void triangulate_kernel(const float* __restrict__ P, const float* __restrict__ p1,
                                                          const float* __restrict__ p2, int n,
                                                          float* __restrict__ xyzw, float* __restrict__ xyz) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float h[4], Pv[24];
#pragma unroll
    for (int k = 0; k < 24; k++) Pv[k] = P[k];
    dlt_point(Pv, p1[2 * i], p1[2 * i + 1], p2[2 * i], p2[2 * i + 1], h);
    if (xyzw) {
#pragma unroll
        for (int k = 0; k < 4; k++) xyzw[4 * i + k] = h[k];
    }
    if (xyz) {
        float x[3];
        dlt_euclidean(h, x);
        xyz[3 * i] = x[0];
        xyz[3 * i + 1] = x[1];
        xyz[3 * i + 2] = x[2];
    }
}

}  // namespace

hipError_t launch_triangulate(const float* d_P, const float* d_p1, const float* d_p2, int n, float* d_xyzw,
                              float* d_xyz, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(triangulate_kernel, dim3((n + 255) / 256), dim3(256), 0, st, d_P, d_p1, d_p2, n, d_xyzw,
                       d_xyz);
    return hipGetLastError();
}

}  // namespace svo
