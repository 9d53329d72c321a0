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

namespace svo {

namespace {

__device__ __forceinline__ void jrot(double (&W)[4][4], double (&V)[4][4], int p, int q, bool& rotated) {
    double al = 0, be = 0, ga = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        al += W[k][p] * W[k][p];
        be += W[k][q] * W[k][q];
        ga += W[k][p] * W[k][q];
    }
    if (ga == 0 || fabs(ga) <= 1e-15 * sqrt(al * be)) return;
    rotated = true;
    const double z = (be - al) / (2 * ga);
    const double t = (z >= 0 ? 1.0 : -1.0) / (fabs(z) + sqrt(1 + z * z));
    const double c = 1 / sqrt(1 + t * t), s = c * t;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const double x = W[k][p], y = W[k][q];
        W[k][p] = c * x - s * y;
        W[k][q] = s * x + c * y;
        const double vx = V[k][p], vy = V[k][q];
        V[k][p] = c * vx - s * vy;
        V[k][q] = s * vx + c * vy;
    }
}

__global__ __launch_bounds__(256) void triangulate_kernel(const float* __restrict__ P, const float* __restrict__ p1,
                                                          const float* __restrict__ p2, int n,
                                                          float* __restrict__ xyzw, float* __restrict__ xyz) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double W[4][4], V[4][4];
    const float x1 = p1[2 * i], y1 = p1[2 * i + 1], x2 = p2[2 * i], y2 = p2[2 * i + 1];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        W[0][k] = (double)x1 * P[8 + k] - P[k];
        W[1][k] = (double)y1 * P[8 + k] - P[4 + k];
        W[2][k] = (double)x2 * P[20 + k] - P[12 + k];
        W[3][k] = (double)y2 * P[20 + k] - P[16 + k];
#pragma unroll
        for (int j = 0; j < 4; j++) V[k][j] = k == j;
    }
    for (int sweep = 0; sweep < 30; sweep++) {
        bool rotated = false;
        jrot(W, V, 0, 1, rotated);
        jrot(W, V, 0, 2, rotated);
        jrot(W, V, 0, 3, rotated);
        jrot(W, V, 1, 2, rotated);
        jrot(W, V, 1, 3, rotated);
        jrot(W, V, 2, 3, rotated);
        if (!rotated) break;
    }
    // column of W with the smallest norm -> that column of V
    double best = 0;
    int bj = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const double s = W[0][j] * W[0][j] + W[1][j] * W[1][j] + W[2][j] * W[2][j] + W[3][j] * W[3][j];
        if (j == 0 || s < best) {
            best = s;
            bj = j;
        }
    }
    double v[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        // select by unrolled compare (keeps V in registers)
        double e = V[k][0];
        if (bj == 1) e = V[k][1];
        if (bj == 2) e = V[k][2];
        if (bj == 3) e = V[k][3];
        v[k] = e;
    }
    const double nrm = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3]);
    const double sg = v[3] < 0 ? -1.0 : 1.0;
    float h[4];
#pragma unroll
    for (int k = 0; k < 4; k++) h[k] = (float)(sg * v[k] / nrm);
    if (xyzw) {
#pragma unroll
        for (int k = 0; k < 4; k++) xyzw[4 * i + k] = h[k];
    }
    if (xyz) {
        const float sc = h[3] != 0.f ? 1.f / h[3] : 1.f;
        xyz[3 * i] = h[0] * sc;
        xyz[3 * i + 1] = h[1] * sc;
        xyz[3 * i + 2] = h[2] * sc;
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
