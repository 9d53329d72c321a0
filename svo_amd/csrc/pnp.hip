// Batched PnP reprojection residual + inlier scoring for gfx950.
//
// Replaces the inner loop of cv::solvePnPRansac at R:src/tracking.cpp:191-196:
// PnPRansacCallback::computeError (calib3d/src/solvepnp.cpp) -> projectPoints
// (calibration.cpp; K from the reference's Matx33f, zero distortion, double
// arithmetic, CV_32F output) and RANSACPointSetRegistrator::findInliers
// (ptsetreg.cpp; err = normL2Sqr<float>(ipt - ppt) <= (float)(thr*thr)).
// One thread per (hypothesis, point); the double expression order is the
// projectPoints order (x = R0 X + R1 Y + R2 Z + t0, z -> 1/z, x *= z, u = x fx + cx)
// and the build uses -ffp-contract=off, so every residual is bit-exact.
// Outputs: optional f32 residuals, inlier bitmask (32 points per word, one
// ballot per wave), per-hypothesis inlier counts (integer atomics: exact).
#include "common.hpp"

namespace svo {

namespace {

__global__ __launch_bounds__(256) void pnp_residual_kernel(PnpBatch B, double fx, double fy, double cx,
                                                           double cy, float thresh2) {
    const int seq = blockIdx.z;
    const int h = blockIdx.y;
    const int n = B.counts ? B.counts[seq] : B.n;
    if ((int)blockIdx.x * 256 >= n) return;
    const int i = blockIdx.x * 256 + threadIdx.x;
    const float* __restrict__ obj = B.obj + 3 * (size_t)seq * B.cap;
    const float* __restrict__ img = B.img + 2 * (size_t)seq * B.cap;
    const double* R = B.hyp + 12 * ((size_t)seq * B.m + h);  // uniform -> scalar loads
    bool inl = false;
    if (i < n) {
        const double X = obj[3 * i], Y = obj[3 * i + 1], Z = obj[3 * i + 2];
        double x = R[0] * X + R[1] * Y + R[2] * Z + R[9];
        double y = R[3] * X + R[4] * Y + R[5] * Z + R[10];
        double z = R[6] * X + R[7] * Y + R[8] * Z + R[11];
        z = z ? 1. / z : 1;
        x *= z;
        y *= z;
        const float u = (float)(x * fx + cx), v = (float)(y * fy + cy);
        const float dx = img[2 * i] - u, dy = img[2 * i + 1] - v;
        float s = 0.f;
        s += dx * dx;
        s += dy * dy;
        if (B.err) B.err[((size_t)seq * B.m + h) * B.cap + i] = s;
        inl = s <= thresh2;
    }
    const unsigned long long bal = __ballot(inl);
    const int lane = threadIdx.x & 63;
    const int words = (n + 31) >> 5;
    const int w0 = (blockIdx.x * 256 + (threadIdx.x & ~63)) >> 5;
    if (B.bits) {
        uint32_t* bits = B.bits + ((size_t)seq * B.m + h) * B.words_cap;
        if (lane == 0 && w0 < words) bits[w0] = (uint32_t)bal;
        if (lane == 1 && w0 + 1 < words) bits[w0 + 1] = (uint32_t)(bal >> 32);
    }
    if (B.cnt && lane == 0 && bal) atomicAdd(&B.cnt[(size_t)seq * B.m + h], __popcll(bal));
}

}  // namespace

hipError_t launch_pnp_residuals(const PnpBatch& b, int nseq, int max_n, double fx, double fy, double cx,
                                double cy, float thresh2, hipStream_t st) {
    if (max_n <= 0 || b.m <= 0 || nseq <= 0) return hipSuccess;
    if (b.cnt) {
        hipError_t e = hipMemsetAsync(b.cnt, 0, sizeof(int) * (size_t)b.m * nseq, st);
        if (e != hipSuccess) return e;
    }
    dim3 grid((max_n + 255) / 256, b.m, nseq);
    hipLaunchKernelGGL(pnp_residual_kernel, grid, dim3(256), 0, st, b, fx, fy, cx, cy, thresh2);
    return hipGetLastError();
}

}  // namespace svo
