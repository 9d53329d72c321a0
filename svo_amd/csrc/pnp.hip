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
#include "sqpnp.hpp"

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

// solvePnP(SQPNP) on a sequence's RANSAC inliers (SqpnpFitIn mode 1) and the
// Frame::pose() of every outcome (R:src/tracking.cpp:191-214). Lane 0 assembles the
// cost and Omega's eigen-decomposition; lanes 0..17 run the SQP from the 18 starts
// (the 9 eigenvectors, each +- sqrt(3) e) -- every start a search could ask for,
// each independent of the others; lane 0 then replays the search (sq_select) with
// those results, which takes the same steps as the host's on-demand runs.
__global__ __launch_bounds__(64) void sqpnp_fit_kernel(const double* __restrict__ stats,
                                                       const SqpnpFitIn* __restrict__ in,
                                                       const float* __restrict__ obj, const int* __restrict__ counts,
                                                       int cap, const uint32_t* __restrict__ bits, int words_cap,
                                                       double* __restrict__ pose6, double* __restrict__ pose12) {
    const int s = blockIdx.x, lane = threadIdx.x;
    __shared__ sq::SqpnpCost c;
    __shared__ double ev[9], evec[81], rs[18][9];
    __shared__ int nn_s;
    const SqpnpFitIn fin = in[s];
    if (fin.mode == 1) {
        if (lane == 0) {
            sq::sqpnp_assemble(stats + 40 * (size_t)s, c);
            int nn = -1;
            if (c.ok) {
                double Oc[81];
                for (int k = 0; k < 81; k++) Oc[k] = c.Om[k];
                la::sym_eig_ql(Oc, 9, ev, evec);
                nn = sq::sq_null_count(ev);
            }
            nn_s = nn;
        }
        __syncthreads();
        if (nn_s >= 0 && lane < 18) sq::sq_start(c, evec, lane, rs[lane]);
        __syncthreads();
    }
    if (lane != 0) return;
    double rvec[3] = {0, 0, 0}, tvec[3] = {0, 0, 0};
    if (fin.mode == 2) {
        for (int k = 0; k < 3; k++) {
            rvec[k] = fin.rv[k];
            tvec[k] = fin.t[k];
        }
    } else if (fin.mode == 1) {
        bool found = false;
        double R[9], t[3];
        if (nn_s >= 0) {
            const int n = counts[s];
            const float* o = obj + 3 * (size_t)s * cap;
            const uint32_t* b = bits + (size_t)s * words_cap;
            int n_in = 0;
            for (int w = 0; w < (n + 31) / 32; w++) n_in += __popc(b[w] & (w == n / 32 ? (1u << (n & 31)) - 1u : ~0u));
            sq::sq_select(
                c, ev, evec, nn_s, n_in,
                [&](int j, double* r) {
                    for (int k = 0; k < 9; k++) r[k] = rs[j][k];
                },
                [&](const double* r, const double* tt) {
                    int pos = 0;
                    for (int i = 0; i < n; i++) {
                        if (!((b[i >> 5] >> (i & 31)) & 1u)) continue;
                        const double p[3] = {(double)o[3 * i], (double)o[3 * i + 1], (double)o[3 * i + 2]};
                        pos += dot3(r + 6, p) + tt[2] > 0;
                    }
                    return pos;
                },
                R, t, &found);
        }
        if (found) {
            la::cv::rodrigues_inv(R, rvec);
            for (int k = 0; k < 3; k++) tvec[k] = t[k];
        } else {  // solvePnP(SQPNP) asserted or found nothing: the RANSAC model (as the host)
            la::cv::rodrigues_inv(fin.R, rvec);
            for (int k = 0; k < 3; k++) tvec[k] = fin.t[k];
        }
    }
    double* P6 = pose6 + 6 * (size_t)s;
    for (int k = 0; k < 3; k++) {
        P6[k] = rvec[k];
        P6[3 + k] = tvec[k];
    }
    // Frame::pose(): the inverse of [R(rvec) | tvec] (svo::SE3d::inverse order)
    double Rm[9];
    la::rodrigues(rvec, Rm);
    double* T = pose12 + 12 * (size_t)s;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) T[3 * i + j] = Rm[3 * j + i];
    for (int i = 0; i < 3; i++) T[9 + i] = -(T[3 * i] * tvec[0] + T[3 * i + 1] * tvec[1] + T[3 * i + 2] * tvec[2]);
}

hipError_t launch_sqpnp_fit(const double* stats, const SqpnpFitIn* in, const float* obj, const int* counts, int cap,
                            const uint32_t* bits, int words_cap, int nseq, double* pose6, double* pose12,
                            hipStream_t st) {
    if (nseq <= 0) return hipSuccess;
    hipLaunchKernelGGL(sqpnp_fit_kernel, dim3(nseq), dim3(64), 0, st, stats, in, obj, counts, cap, bits, words_cap,
                       pose6, pose12);
    return hipGetLastError();
}

hipError_t launch_suffstats(const float* obj, const float* img, const int* counts, int cap, const uint32_t* bits,
                            int words_cap, int nseq, const double K[9], double* out, hipStream_t st) {
    if (nseq <= 0) return hipSuccess;
    hipLaunchKernelGGL(suffstats_kernel, dim3(nseq), dim3(256), 0, st, obj, img, counts, cap, bits, words_cap,
                       1. / K[0], 1. / K[4], K[2], K[5], out);
    return hipGetLastError();
}

}  // namespace svo
