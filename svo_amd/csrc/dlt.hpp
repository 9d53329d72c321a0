// Per-point two-view DLT (cv::triangulatePoints, calib3d/src/triangulate.cpp) as a
// device function: shared by triangulate_kernel (svo_triangulate_points) and the
// batched front end's keyframe append (fe_kernels.hip). P = {P1[12], P2[12]}
// row-major 3x4 floats; h = the homogeneous point (unit length, w >= 0) rounded
// to float like points4D (CV_32F). A (4x4, double) has rows x*P[2]-P[0],
// y*P[2]-P[1] per view; the homogeneous point is A's right singular vector of the
// smallest singular value, found by a one-sided Jacobi SVD held in registers.
#pragma once

#include <hip/hip_runtime.h>

namespace svo {

__device__ __forceinline__ void dlt_jrot(double (&W)[4][4], double (&V)[4][4], int p, int q, bool& rotated) {
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

__device__ __forceinline__ void dlt_point(const float* __restrict__ P, float x1, float y1, float x2, float y2,
                                          float (&h)[4]) {
    double W[4][4], V[4][4];
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
        dlt_jrot(W, V, 0, 1, rotated);
        dlt_jrot(W, V, 0, 2, rotated);
        dlt_jrot(W, V, 0, 3, rotated);
        dlt_jrot(W, V, 1, 2, rotated);
        dlt_jrot(W, V, 1, 3, rotated);
        dlt_jrot(W, V, 2, 3, rotated);
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
#pragma unroll
    for (int k = 0; k < 4; k++) h[k] = (float)(sg * v[k] / nrm);
}

// convertPointsFromHomogeneous (calib3d/src/fundam.cpp): float divide by w, 1 if w == 0
__device__ __forceinline__ void dlt_euclidean(const float (&h)[4], float (&x)[3]) {
    const float sc = h[3] != 0.f ? 1.f / h[3] : 1.f;
    x[0] = h[0] * sc;
    x[1] = h[1] * sc;
    x[2] = h[2] * sc;
}

}  // namespace svo
