// SQPnP's sufficient statistics of one sequence's RANSAC inliers (pose.hpp
// kSqpnpStats: 40 doubles) computed by one 256-thread workgroup: the normalised
// image point (x, y), x^2 + y^2 and the products with the map point and its
// quadratic terms, accumulated per thread over i = tid, tid + 256, ... and reduced
// in a fixed order (wave shuffles, then ((w0 + w1) + w2) + w3) -- the same sums
// wherever it runs: suffstats_kernel (pnp.hip) or the keyframe's outlier
// compaction (fe_kernels.hip tail_body), which reads the same points and bits.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace svo {

constexpr int kSuffStats = 40;     // pose.hpp kSqpnpStats
constexpr int kSuffThreads = 256;  // the reduction order is that of 4 waves

// part: __shared__ double[kSuffThreads / 64][kSuffStats]; out: kSuffStats doubles
__device__ __forceinline__ void suffstats_block(const float* __restrict__ o, const float* __restrict__ im, int n,
                                                const uint32_t* __restrict__ b, double ifx, double ify, double cx,
                                                double cy, double (*part)[kSuffStats], double* __restrict__ out) {
    double acc[kSuffStats];
#pragma unroll
    for (int k = 0; k < kSuffStats; k++) acc[k] = 0;
    for (int i = threadIdx.x; i < n; i += kSuffThreads) {
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
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < kSuffStats; k++) {
        double v = acc[k];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
        if (lane == 0) part[wv][k] = v;
    }
    __syncthreads();
    if (threadIdx.x < kSuffStats) {
        const int k = threadIdx.x;
        out[k] = ((part[0][k] + part[1][k]) + part[2][k]) + part[3][k];
    }
}

}  // namespace svo
