// Per-point two-view DLT (cv::triangulatePoints, calib3d/src/triangulate.cpp) as a
// device function: shared by triangulate_kernel (svo_triangulate_points) and the
// batched front end's keyframe append (fe_kernels.hip). P = {P1[12], P2[12]}
// row-major 3x4 floats; h = the homogeneous point (unit length, w >= 0) rounded
// to float like points4D (CV_32F). A (4x4, double) has rows x*P[2]-P[0],
// y*P[2]-P[1] per view; the homogeneous point is A's right singular vector of the
// smallest singular value (below: the matching eigenvector of A^T A).
#pragma once

#include <hip/hip_runtime.h>

namespace svo {

// Symmetric 4x4 held as its 10 upper entries (constant indices: registers)
constexpr int dlt_ix(int i, int j) { return i <= j ? i * 4 - i * (i - 1) / 2 + (j - i) : j * 4 - j * (j - 1) / 2 + (i - j); }

// 1 / sqrt(x) and 1 / x for x > 0 of the rotation formulas: the hardware estimates
// refined by two Newton steps each (full double accuracy; no scaling or fix-up
// paths -- the operands are sums of squares of well-scaled entries, and a zero
// operand only arises for a skipped pair, whose result is discarded)
__device__ __forceinline__ double dlt_rsq(double x) {
    double y = __builtin_amdgcn_rsq(x);
    y = y * (1.5 - 0.5 * x * y * y);
    return y * (1.5 - 0.5 * x * y * y);
}
__device__ __forceinline__ double dlt_rcp(double x) {
    double y = __builtin_amdgcn_rcp(x);
    y = y * (2.0 - x * y);
    return y * (2.0 - x * y);
}

// One Jacobi rotation (p, q) of the symmetric M, accumulated into V's columns
// (M' = J^T M J zeroes M_pq: M_pp -= t M_pq, M_qq += t M_pq, t = tan of the angle
// as the smaller root of t^2 + 2 theta t - 1 = 0, theta = (M_qq - M_pp) / 2 M_pq,
// i.e. t = sign(d) 2 M_pq / (|d| + sqrt(d^2 + 4 M_pq^2)), d = M_qq - M_pp; c = 1 /
// sqrt(1 + t^2)). Branch-free: a pair below the threshold gets t = 0, c = 1, s = 0,
// which leaves every entry exactly as it was (a branch per rotation made the
// compiler copy M and V at every join).
template <int P, int Q>
__device__ __forceinline__ void dlt_jrot(double (&M)[10], double (&V)[4][4]) {
    const double apq = M[dlt_ix(P, Q)], app = M[dlt_ix(P, P)], aqq = M[dlt_ix(Q, Q)];
    const bool skip = apq * apq <= 1e-30 * (app * aqq);  // (also apq == 0)
    const double d = aqq - app;
    const double x = d * d + 4.0 * apq * apq;
    const double t0 = (d >= 0 ? 2.0 * apq : -2.0 * apq) * dlt_rcp(fabs(d) + x * dlt_rsq(x));
    const double t = skip ? 0.0 : t0;
    const double c = dlt_rsq(1.0 + t * t), s = t * c;
    M[dlt_ix(P, P)] = app - t * apq;
    M[dlt_ix(Q, Q)] = aqq + t * apq;
    M[dlt_ix(P, Q)] = skip ? apq : 0.0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        if (k != P && k != Q) {
            const double mp = M[dlt_ix(k, P)], mq = M[dlt_ix(k, Q)];
            M[dlt_ix(k, P)] = c * mp - s * mq;
            M[dlt_ix(k, Q)] = s * mp + c * mq;
        }
        const double vp = V[k][P], vq = V[k][Q];
        V[k][P] = c * vp - s * vq;
        V[k][Q] = s * vp + c * vq;
    }
}

// The homogeneous point is the eigenvector of A^T A (4 x 4, symmetric) of the
// smallest eigenvalue -- A's right singular vector of its smallest singular value,
// which OpenCV's SVD returns -- by cyclic Jacobi on the 10 distinct entries: 26
// doubles in registers (the one-sided SVD of A held A V and V, 32 doubles, and spilled
// V to scratch for the final column pick), so a wave of it fits beside three LK waves
// per SIMD. Sensitivity: eps * (lambda_max / eigen-gap), far below the 1e-5 bar.
__device__ __forceinline__ void dlt_point(const float (&P)[24], float x1, float y1, float x2, float y2,
                                          float (&h)[4]) {
    double M[10], V[4][4];
    {
        double A[4][4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            A[0][k] = (double)x1 * P[8 + k] - P[k];
            A[1][k] = (double)y1 * P[8 + k] - P[4 + k];
            A[2][k] = (double)x2 * P[20 + k] - P[12 + k];
            A[3][k] = (double)y2 * P[20 + k] - P[16 + k];
        }
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int j = i; j < 4; j++)
                M[dlt_ix(i, j)] = A[0][i] * A[0][j] + A[1][i] * A[1][j] + A[2][i] * A[2][j] + A[3][i] * A[3][j];
    }
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
        for (int j = 0; j < 4; j++) V[k][j] = k == j;
    // five cyclic sweeps, unrolled and unconditional: a rolled loop with a
    // data-dependent exit kept two copies of M and V across its back edge (98-157
    // VGPRs); straight-line, the kernel fits 80 with no scratch. Five is a margin
    // over the 3-4 sweeps the DLT systems converge in (an emulation over 200k
    // KITTI-geometry stereo points, depths 1-300 m: 4 sweeps already within 3.4e-9
    // of an SVD; converged rotations are exact no-ops)
#pragma unroll
    for (int sweep = 0; sweep < 5; sweep++) {
        dlt_jrot<0, 1>(M, V);
        dlt_jrot<0, 2>(M, V);
        dlt_jrot<0, 3>(M, V);
        dlt_jrot<1, 2>(M, V);
        dlt_jrot<1, 3>(M, V);
        dlt_jrot<2, 3>(M, V);
    }
    // the column of V of the smallest eigenvalue, picked by selects (no indexing)
    double best = M[dlt_ix(0, 0)];
    double v[4] = {V[0][0], V[1][0], V[2][0], V[3][0]};
#pragma unroll
    for (int j = 1; j < 4; j++) {
        const bool lt = M[dlt_ix(j, j)] < best;
        best = lt ? M[dlt_ix(j, j)] : best;
#pragma unroll
        for (int k = 0; k < 4; k++) v[k] = lt ? V[k][j] : v[k];
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
