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

// projectPoints + normL2Sqr<float> of point i under hypothesis R (the double
// expression order of calibration.cpp, -ffp-contract=off): the squared residual
__device__ __forceinline__ float pnp_residual2(const double* R, const float* __restrict__ obj,
                                               const float* __restrict__ img, int i, double fx, double fy, double cx,
                                               double cy) {
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
    return s;
}

__global__ __launch_bounds__(256) void pnp_residual_kernel(PnpBatch B, double fx, double fy, double cx,
                                                           double cy, float thresh2) {
    const int seq = blockIdx.z;
    const int h = blockIdx.y;
    const int n = B.counts ? B.counts[seq] : B.n;
    if ((int)blockIdx.x * 256 >= n) return;
    const int i = blockIdx.x * 256 + threadIdx.x;
    const float* __restrict__ obj = B.obj + 3 * (size_t)seq * B.cap;
    const float* __restrict__ img = B.img + 2 * (size_t)seq * B.cap;
    const int ms = B.mstride ? B.mstride : B.m;
    const double* R = B.hyp + 12 * ((size_t)seq * ms + h);  // uniform -> scalar loads
    bool inl = false;
    if (i < n) {
        const float s = pnp_residual2(R, obj, img, i, fx, fy, cx, cy);
        if (B.err) B.err[((size_t)seq * ms + h) * B.cap + i] = s;
        inl = s <= thresh2;
    }
    const unsigned long long bal = __ballot(inl);
    const int lane = threadIdx.x & 63;
    const int words = (n + 31) >> 5;
    const int w0 = (blockIdx.x * 256 + (threadIdx.x & ~63)) >> 5;
    if (B.bits) {
        uint32_t* bits = B.bits + ((size_t)seq * ms + h) * B.words_cap;
        if (lane == 0 && w0 < words) bits[w0] = (uint32_t)bal;
        if (lane == 1 && w0 + 1 < words) bits[w0 + 1] = (uint32_t)(bal >> 32);
    }
    if (B.cnt && lane == 0 && bal) atomicAdd(&B.cnt[(size_t)seq * ms + h], __popcll(bal));
}

// One block per (hypothesis, sequence) over all of the sequence's points: the same
// inlier test, bits written word by word as pnp_residual_kernel does, and the
// inlier count reduced inside the block and written ONCE per hypothesis (B.cnt,
// which may live in host-coherent memory: the host reads m counts per sequence
// instead of summing per-wave counts out of uncached memory, as round 1 did). 256 threads: the
// blocks must find room on CUs a running LK occupies (a 1024-thread block
// waits for a whole CU to drain: measured 290 us against ~25 us)
constexpr int kScoreBlock = 256;
__global__ __launch_bounds__(kScoreBlock) void pnp_score_kernel(PnpBatch B, double fx, double fy, double cx, double cy,
                                                                float thresh2) {
    const int seq = blockIdx.y, h = blockIdx.x;
    const int n = B.counts ? B.counts[seq] : B.n;
    const float* __restrict__ obj = B.obj + 3 * (size_t)seq * B.cap;
    const float* __restrict__ img = B.img + 2 * (size_t)seq * B.cap;
    const int ms = B.mstride ? B.mstride : B.m;
    const double* R = B.hyp + 12 * ((size_t)seq * ms + h);
    uint32_t* bits = B.bits ? B.bits + ((size_t)seq * ms + h) * B.words_cap : nullptr;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int words = (n + 31) >> 5;
    int cnt = 0;
    for (int base = 0; base < n; base += kScoreBlock) {
        const int i = base + threadIdx.x;
        const bool inl = i < n && pnp_residual2(R, obj, img, i, fx, fy, cx, cy) <= thresh2;
        const unsigned long long bal = __ballot(inl);
        const int w0 = (base + (threadIdx.x & ~63)) >> 5;
        if (bits) {
            if (lane == 0 && w0 < words) bits[w0] = (uint32_t)bal;
            if (lane == 1 && w0 + 1 < words) bits[w0 + 1] = (uint32_t)(bal >> 32);
        }
        cnt += __popcll(bal);
    }
    __shared__ int part[kScoreBlock / 64];
    if (lane == 0) part[wv] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
        for (int q = 0; q < kScoreBlock / 64; q++) tot += part[q];
        B.cnt[(size_t)seq * ms + h] = tot;
    }
}

}  // namespace

hipError_t launch_pnp_score(const PnpBatch& b, int nseq, double fx, double fy, double cx, double cy, float thresh2,
                            hipStream_t st) {
    if (b.m <= 0 || nseq <= 0 || !b.cnt) return b.cnt ? hipSuccess : hipErrorInvalidValue;
    hipLaunchKernelGGL(pnp_score_kernel, dim3(b.m, nseq), dim3(kScoreBlock), 0, st, b, fx, fy, cx, cy, thresh2);
    return hipGetLastError();
}

hipError_t launch_pnp_residuals(const PnpBatch& b, int nseq, int max_n, double fx, double fy, double cx,
                                double cy, float thresh2, hipStream_t st) {
    if (max_n <= 0 || b.m <= 0 || nseq <= 0) return hipSuccess;
    if (b.cnt) {
        const int ms = b.mstride ? b.mstride : b.m;
        hipError_t e = hipMemsetAsync(b.cnt, 0, sizeof(int) * (size_t)ms * nseq, st);
        if (e != hipSuccess) return e;
    }
    dim3 grid((max_n + 255) / 256, b.m, nseq);
    hipLaunchKernelGGL(pnp_residual_kernel, grid, dim3(256), 0, st, b, fx, fy, cx, cy, thresh2);
    return hipGetLastError();
}

}  // namespace svo

namespace svo {

namespace {

// Sufficient statistics of the SQPnP cost over each sequence's RANSAC inliers
// (pose.cpp sqpnp_sums, same per-point arithmetic): one block per sequence,
// kStats per-thread partial sums, reduced in a fixed order (wave shuffles, then
// the 4 waves in order) so the result is deterministic.
constexpr int kStats = 40;  // pose.hpp kSqpnpStats
__global__ __launch_bounds__(256) void suffstats_kernel(const float* __restrict__ obj, const float* __restrict__ img,
                                                        const int* __restrict__ counts, int cap,
                                                        const uint32_t* __restrict__ bits, int words_cap, double ifx,
                                                        double ify, double cx, double cy, double* __restrict__ out) {
    const int s = blockIdx.x;
    const int n = counts[s];
    const float* o = obj + 3 * (size_t)s * cap;
    const float* im = img + 2 * (size_t)s * cap;
    const uint32_t* b = bits + (size_t)s * words_cap;
    double acc[kStats];
#pragma unroll
    for (int k = 0; k < kStats; k++) acc[k] = 0;
    for (int i = threadIdx.x; i < n; i += 256) {
        if (!((b[i >> 5] >> (i & 31)) & 1u)) continue;
        const double x = ((double)im[2 * i] - cx) * ifx, y = ((double)im[2 * i + 1] - cy) * ify;
        const double sq = x * x + y * y;
        const double p[3] = {(double)o[3 * i], (double)o[3 * i + 1], (double)o[3 * i + 2]};
        const double pp[6] = {p[0] * p[0], p[0] * p[1], p[0] * p[2], p[1] * p[1], p[1] * p[2], p[2] * p[2]};
        const double c[4] = {1.0, x, y, sq};
        acc[0] += 1.0;
        acc[1] += x;
        acc[2] += y;
        acc[3] += sq;
#pragma unroll
        for (int u = 0; u < 4; u++) {
#pragma unroll
            for (int j = 0; j < 3; j++) acc[4 + 3 * u + j] += c[u] * p[j];
#pragma unroll
            for (int v = 0; v < 6; v++) acc[16 + 6 * u + v] += c[u] * pp[v];
        }
    }
    __shared__ double part[4][kStats];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < kStats; k++) {
        double v = acc[k];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
        if (lane == 0) part[wv][k] = v;
    }
    __syncthreads();
    if (threadIdx.x < kStats) {
        const int k = threadIdx.x;
        out[kStats * (size_t)s + k] = ((part[0][k] + part[1][k]) + part[2][k]) + part[3][k];
    }
}

}  // namespace

hipError_t launch_suffstats(const float* obj, const float* img, const int* counts, int cap, const uint32_t* bits,
                            int words_cap, int nseq, const double K[9], double* out, hipStream_t st) {
    if (nseq <= 0) return hipSuccess;
    hipLaunchKernelGGL(suffstats_kernel, dim3(nseq), dim3(256), 0, st, obj, img, counts, cap, bits, words_cap,
                       1. / K[0], 1. / K[4], K[2], K[5], out);
    return hipGetLastError();
}

}  // namespace svo
