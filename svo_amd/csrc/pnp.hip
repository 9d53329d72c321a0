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
#include "suffstats.hpp"
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
// suffstats.hpp (the keyframe's compaction computes the same in the step).
__global__ __launch_bounds__(kSuffThreads) void suffstats_kernel(const float* __restrict__ obj,
                                                                 const float* __restrict__ img,
                                                                 const int* __restrict__ counts, int cap,
                                                                 const uint32_t* __restrict__ bits, int words_cap,
                                                                 double ifx, double ify, double cx, double cy,
                                                                 double* __restrict__ out) {
    __shared__ double part[kSuffThreads / 64][kSuffStats];
    const int s = blockIdx.x;
    suffstats_block(obj + 3 * (size_t)s * cap, img + 2 * (size_t)s * cap, counts[s], bits + (size_t)s * words_cap,
                    ifx, ify, cx, cy, part, out + kSuffStats * (size_t)s);
}

}  // namespace

namespace {

// broadcast of lane `src`'s double (src uniform)
__device__ __forceinline__ double bcast(double v, int src) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), src);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), src);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// sq::sqp_step with the 15 x 16 KKT system one row per lane (lanes 0..14, the row
// in registers): the same elements, the same pivot (the first largest |a| below
// the diagonal, found by the serial scan), the same eliminations and the same
// back-substitution order as the scalar routine, so delta is bit-identical.
// Every lane returns delta. Jw: this wave's LDS rows of J (6 x 9).
__device__ void sqp_step_wave(const double* Om, const double* r, double* delta, double* Jw) {
    constexpr int N = 15;
    const int lane = threadIdx.x & 63;
    const double* r1 = r;
    const double* r2 = r + 3;
    const double* r3 = r + 6;
    if (lane < 54) {  // J[c][j] = 0 except the row-norm / row-dot entries
        const int c = lane / 9, j = lane % 9, k = j % 3, blk = j / 3;
        double v = 0;
        if (c == 0 && blk == 0) v = 2 * r1[k];
        if (c == 1 && blk == 1) v = 2 * r2[k];
        if (c == 2 && blk == 2) v = 2 * r3[k];
        if (c == 3) v = blk == 0 ? r2[k] : blk == 1 ? r1[k] : 0.0;
        if (c == 4) v = blk == 1 ? r3[k] : blk == 2 ? r2[k] : 0.0;
        if (c == 5) v = blk == 0 ? r3[k] : blk == 2 ? r1[k] : 0.0;
        Jw[lane] = v;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const double h[6] = {dot3(r1, r1) - 1, dot3(r2, r2) - 1, dot3(r3, r3) - 1, dot3(r1, r2), dot3(r2, r3),
                         dot3(r1, r3)};
    double a[N + 1];
    for (int j = 0; j <= N; j++) a[j] = 0;
    if (lane < 9) {
        double g = 0;
        for (int j = 0; j < 9; j++) {
            a[j] = 2 * Om[9 * lane + j];
            g += Om[9 * lane + j] * r[j];
        }
        a[N] = -2 * g;
        for (int c = 0; c < 6; c++) a[9 + c] = Jw[9 * c + lane];
    } else if (lane < N) {
        const int c = lane - 9;
        for (int j = 0; j < 9; j++) a[j] = Jw[9 * c + j];
        double hc = h[0];
        for (int q = 1; q < 6; q++)
            if (c == q) hc = h[q];
        a[N] = -hc;
    }
#pragma unroll
    for (int col = 0; col < N; col++) {
        // the scalar loop's pivot: first strict maximum of |a[i][col]|, i >= col
        int piv = col;
        double best = fabs(bcast(a[col], col));
#pragma unroll
        for (int i = col + 1; i < N; i++) {
            const double v = fabs(bcast(a[col], i));
            if (v > best) {
                best = v;
                piv = i;
            }
        }
        double prow[N + 1];  // row col after the swap
        if (piv != col) {
#pragma unroll
            for (int j = 0; j <= N; j++) {
                const double cj = bcast(a[j], col), pj = bcast(a[j], piv);
                if (lane == col) a[j] = pj;
                if (lane == piv) a[j] = cj;
                prow[j] = pj;
            }
        } else {
#pragma unroll
            for (int j = 0; j <= N; j++) prow[j] = bcast(a[j], col);
        }
        const double d = prow[col];
        if (d == 0) continue;
        if (lane > col && lane < N) {
            const double f = a[col] / d;
            if (f != 0)
#pragma unroll
                for (int j = col; j <= N; j++) a[j] -= f * prow[j];
        }
    }
    double x[N];
#pragma unroll
    for (int i = N - 1; i >= 0; i--) {
        double xi = 0;
        if (lane == i) {
            double v = a[N];
#pragma unroll
            for (int j = i + 1; j < N; j++) v -= a[j] * x[j];
            xi = a[i] != 0 ? v / a[i] : 0.0;
        }
        x[i] = bcast(xi, i);
    }
    for (int k = 0; k < 9; k++) delta[k] = x[k];
}

// sq::sq_start with sqp_run's steps taken by sqp_step_wave (every lane holds r)
__device__ void sq_start_wave(const sq::SqpnpCost& c, const double* evec, int j, double* rhat, double* Jw) {
    const double* ev = evec + 9 * (j >> 1);
    double m[9], r[9], delta[9];
    for (int k = 0; k < 9; k++) m[k] = (j & 1) ? -(1.7320508075688772 * ev[k]) : 1.7320508075688772 * ev[k];
    la::nearest_rotation(m, r);
    double dsq = 1.7976931348623157e308;
    int step = 0;
    while (dsq > 1e-10 && step++ < 15) {
        sqp_step_wave(c.Om, r, delta, Jw);
        dsq = 0;
        for (int k = 0; k < 9; k++) {
            r[k] += delta[k];
            dsq += delta[k] * delta[k];
        }
    }
    double d = r[0] * (r[4] * r[8] - r[5] * r[7]) - r[1] * (r[3] * r[8] - r[5] * r[6]) + r[2] * (r[3] * r[7] - r[4] * r[6]);
    if (d < 0) {
        for (int k = 0; k < 9; k++) r[k] = -r[k];
        d = -d;
    }
    if (d > 1.001)
        la::nearest_rotation(r, rhat);
    else
        for (int k = 0; k < 9; k++) rhat[k] = r[k];
}

// the device fit's per-sequence state between its three kernels
struct SqFitWork {
    sq::SqpnpCost c;
    double ev[9], evec[81], rs[18][9];
    int nn, pad;
};

}  // namespace

size_t sqpnp_fit_work_bytes(int nseq) { return sizeof(SqFitWork) * (size_t)nseq; }

namespace {

// 1. the cost from the statistics and Omega's eigen-decomposition (lane 0; the
//    tred2 / tql2 workspace in LDS), one wave per sequence
__global__ __launch_bounds__(64) void sqpnp_eig_kernel(const double* __restrict__ stats,
                                                       const SqpnpFitIn* __restrict__ in, SqFitWork* __restrict__ work) {
    const int s = blockIdx.x;
    __shared__ double ws[81 + 9 + 9];
    __shared__ sq::SqpnpCost c;
    __shared__ double ev[9], evec[81];
    if (threadIdx.x != 0 || in[s].mode != 1) return;
    SqFitWork& w = work[s];
    sq::sqpnp_assemble(stats + 40 * (size_t)s, c);
    int nn = -1;
    if (c.ok) {
        la::sym_eig_ql_ws(c.Om, 9, ev, evec, ws, ws + 81, ws + 90);
        nn = sq::sq_null_count(ev);
    }
    w.c = c;
    for (int k = 0; k < 9; k++) w.ev[k] = ev[k];
    for (int k = 0; k < 81; k++) w.evec[k] = evec[k];
    w.nn = nn;
}

// 2. the SQP runs from starts 2w and 2w + 1 (+- sqrt(3) times eigenvector w), one
//    wave per (eigenvector, sequence) -- every start a search could ask for, each
//    independent of the others; the 15 x 16 KKT systems one row per lane
__global__ __launch_bounds__(64) void sqpnp_sqp_kernel(const SqpnpFitIn* __restrict__ in,
                                                       SqFitWork* __restrict__ work) {
    const int w = blockIdx.x, s = blockIdx.y, lane = threadIdx.x;
    if (in[s].mode != 1) return;
    SqFitWork& wk = work[s];
    if (wk.nn < 0) return;
    __shared__ sq::SqpnpCost c;
    __shared__ double evec[81], Jw[54];
    for (int k = lane; k < 81; k += 64) {
        c.Om[k] = wk.c.Om[k];
        evec[k] = wk.evec[k];
    }
    __syncthreads();
    for (int j = 2 * w; j < 2 * w + 2; j++) {
        double r[9];
        sq_start_wave(c, evec, j, r, Jw);
        if (lane == 0)
            for (int k = 0; k < 9; k++) wk.rs[j][k] = r[k];
    }
}

// 3. the solution search (sq_select, replayed with the runs above: the same steps
//    as the host's on-demand runs; every lane runs it, the positive-depth counts
//    spread over the lanes) and Frame::pose() of every outcome
__global__ __launch_bounds__(64) void sqpnp_select_kernel(const SqpnpFitIn* __restrict__ in,
                                                          const SqFitWork* __restrict__ work,
                                                          const float* __restrict__ obj,
                                                          const int* __restrict__ counts, int cap,
                                                          const uint32_t* __restrict__ bits, int words_cap,
                                                          double* __restrict__ pose6, double* __restrict__ pose12) {
    const int s = blockIdx.x, lane = threadIdx.x;
    __shared__ sq::SqpnpCost c;
    __shared__ double ev[9], evec[81], rs[18][9];
    // the inliers' object points, compacted, for the positive-depth majority test
    // (a search calls it for every candidate whose point mean is behind the camera)
    constexpr int kLdsPts = 2048;
    __shared__ float lp[3 * kLdsPts];
    const SqpnpFitIn fin = in[s];
    const SqFitWork& wk = work[s];
    int nn = -1;
    if (fin.mode == 1) {
        nn = wk.nn;
        for (int k = lane; k < 81; k += 64) {
            c.Om[k] = wk.c.Om[k];
            evec[k] = wk.evec[k];
        }
        for (int k = lane; k < 27; k += 64) c.P[k] = wk.c.P[k];
        for (int k = lane; k < 3; k += 64) c.mean[k] = wk.c.mean[k];
        for (int k = lane; k < 9; k += 64) ev[k] = wk.ev[k];
        for (int k = lane; k < 18 * 9; k += 64) rs[k / 9][k % 9] = wk.rs[k / 9][k % 9];
        if (lane == 0) c.ok = wk.c.ok;
    }
    __syncthreads();
    double rvec[3] = {0, 0, 0}, tvec[3] = {0, 0, 0};
    if (fin.mode == 2) {
        for (int k = 0; k < 3; k++) {
            rvec[k] = fin.rv[k];
            tvec[k] = fin.t[k];
        }
    } else if (fin.mode == 1) {
        bool found = false;
        double R[9], t[3];
        if (nn >= 0) {
            const int n = counts[s];
            const float* o = obj + 3 * (size_t)s * cap;
            const uint32_t* b = bits + (size_t)s * words_cap;
            int n_in = 0;
            for (int w = lane; w < (n + 31) / 32; w += 64)
                n_in += __popc(b[w] & (w == n / 32 ? (1u << (n & 31)) - 1u : ~0u));
            for (int off = 32; off > 0; off >>= 1) n_in += __shfl_xor(n_in, off);
            const bool staged = n_in <= kLdsPts;
            if (staged) {  // ballot compaction, every lane converged (n is uniform)
                int base = 0;
                for (int i0 = 0; i0 < n; i0 += 64) {
                    const int i = i0 + lane;
                    const bool inl = i < n && ((b[i >> 5] >> (i & 31)) & 1u);
                    const unsigned long long m = __ballot(inl);
                    if (inl) {
                        const int k = base + __popcll(m & ((1ull << lane) - 1ull));
                        lp[3 * k] = o[3 * i];
                        lp[3 * k + 1] = o[3 * i + 1];
                        lp[3 * k + 2] = o[3 * i + 2];
                    }
                    base += __popcll(m);
                }
                __syncthreads();
            }
            sq::sq_select(
                c, ev, evec, nn, n_in,
                [&](int j, double* r) {
                    for (int k = 0; k < 9; k++) r[k] = rs[j][k];
                },
                [&](const double* r, const double* tt) {
                    int pos = 0;
                    if (staged) {
                        for (int k = lane; k < n_in; k += 64) {
                            const double p[3] = {(double)lp[3 * k], (double)lp[3 * k + 1], (double)lp[3 * k + 2]};
                            pos += dot3(r + 6, p) + tt[2] > 0;
                        }
                    } else {
                        for (int i = lane; i < n; i += 64) {
                            if (!((b[i >> 5] >> (i & 31)) & 1u)) continue;
                            const double p[3] = {(double)o[3 * i], (double)o[3 * i + 1], (double)o[3 * i + 2]};
                            pos += dot3(r + 6, p) + tt[2] > 0;
                        }
                    }
                    for (int off = 32; off > 0; off >>= 1) pos += __shfl_xor(pos, off);
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
    if (lane != 0) return;
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

}  // namespace

hipError_t launch_sqpnp_fit(const double* stats, const SqpnpFitIn* in, const float* obj, const int* counts, int cap,
                            const uint32_t* bits, int words_cap, int nseq, double* pose6, double* pose12, void* work,
                            hipStream_t st) {
    if (nseq <= 0) return hipSuccess;
    SqFitWork* wk = (SqFitWork*)work;
    hipLaunchKernelGGL(sqpnp_eig_kernel, dim3(nseq), dim3(64), 0, st, stats, in, wk);
    hipLaunchKernelGGL(sqpnp_sqp_kernel, dim3(9, nseq), dim3(64), 0, st, in, wk);
    hipLaunchKernelGGL(sqpnp_select_kernel, dim3(nseq), dim3(64), 0, st, in, wk, obj, counts, cap, bits, words_cap,
                       pose6, pose12);
    return hipGetLastError();
}

hipError_t launch_suffstats(const float* obj, const float* img, const int* counts, int cap, const uint32_t* bits,
                            int words_cap, int nseq, const double K[9], double* out, hipStream_t st) {
    if (nseq <= 0) return hipSuccess;
    hipLaunchKernelGGL(suffstats_kernel, dim3(nseq), dim3(kSuffThreads), 0, st, obj, img, counts, cap, bits, words_cap,
                       1. / K[0], 1. / K[4], K[2], K[5], out);
    return hipGetLastError();
}

}  // namespace svo
