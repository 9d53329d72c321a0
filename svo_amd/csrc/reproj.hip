// Batched pinhole reprojection residuals, SE(3) Jacobians and per-problem
// normal equations (§8 a11: the north star's "ceres reprojection cost"; the
// reference links Ceres but never calls it, SURVEY §0.2, so this is pinned by
// finite differences only). Feeds the host pose solver in refine.cpp.
//
// Problem b: pose T = [R|t] (world -> camera, 12 doubles, R row-major), points
// X_i (double xyz), observations u_i (float xy), K (fx, fy, cx, cy):
//   P = R X + t,  r = (fx Px/Pz + cx - u, fy Py/Pz + cy - v)
//   J = dr/dxi for the left perturbation T <- exp(xi^) T, xi = (rho, phi):
//       dP/dxi = [I | -[P]x]
// Robust weight (Huber, delta > 0): w = 1 if |r| <= delta else delta/|r|;
// H = sum w J^T J (21, upper triangle row-major), g = sum w J^T r (6),
// cost = sum rho(|r|) (rho = |r|^2/2 or Huber). Points with Pz <= 0 add nothing.
// Reduction: per block in a fixed order (wave shuffles, then LDS), partial sums
// per (problem, block), then a second pass summing blocks in index order, so
// every run gives the same bits.
#include "common.hpp"

namespace svo {

namespace {

constexpr int kNE = 28;  // 21 H + 6 g + 1 cost

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__global__ __launch_bounds__(256) void reproj_kernel(const double* __restrict__ obj, const float* __restrict__ img,
                                                     const int* __restrict__ counts, int cap,
                                                     const double* __restrict__ poses, double fx, double fy,
                                                     double cx, double cy, double delta, double* __restrict__ res,
                                                     double* __restrict__ jac, double* __restrict__ partial) {
    const int b = blockIdx.y;
    const int n = counts ? counts[b] : cap;
    const int i = blockIdx.x * 256 + threadIdx.x;
    const double* T = poses + 12 * (size_t)b;
    double e[kNE];
#pragma unroll
    for (int k = 0; k < kNE; k++) e[k] = 0;
    if (i < n) {
        const double* X = obj + 3 * ((size_t)b * cap + i);
        const float* u = img + 2 * ((size_t)b * cap + i);
        const double px = T[0] * X[0] + T[1] * X[1] + T[2] * X[2] + T[9];
        const double py = T[3] * X[0] + T[4] * X[1] + T[5] * X[2] + T[10];
        const double pz = T[6] * X[0] + T[7] * X[1] + T[8] * X[2] + T[11];
        double r0 = 0, r1 = 0, J[12];
#pragma unroll
        for (int k = 0; k < 12; k++) J[k] = 0;
        if (pz > 0) {
            const double iz = 1.0 / pz, x = px * iz, y = py * iz;
            r0 = fx * x + cx - (double)u[0];
            r1 = fy * y + cy - (double)u[1];
            J[0] = fx * iz;
            J[1] = 0;
            J[2] = -fx * x * iz;
            J[3] = -fx * x * y;
            J[4] = fx * (1 + x * x);
            J[5] = -fx * y;
            J[6] = 0;
            J[7] = fy * iz;
            J[8] = -fy * y * iz;
            J[9] = -fy * (1 + y * y);
            J[10] = fy * x * y;
            J[11] = fy * x;
            const double nr = sqrt(r0 * r0 + r1 * r1);
            const double w = (delta > 0 && nr > delta) ? delta / nr : 1.0;
            int k = 0;
#pragma unroll
            for (int a = 0; a < 6; a++)
#pragma unroll
                for (int c = a; c < 6; c++) e[k++] = w * (J[a] * J[c] + J[6 + a] * J[6 + c]);
#pragma unroll
            for (int a = 0; a < 6; a++) e[21 + a] = w * (J[a] * r0 + J[6 + a] * r1);
            e[27] = (delta > 0 && nr > delta) ? delta * (nr - 0.5 * delta) : 0.5 * (r0 * r0 + r1 * r1);
        }
        if (res) {
            res[2 * ((size_t)b * cap + i)] = r0;
            res[2 * ((size_t)b * cap + i) + 1] = r1;
        }
        if (jac)
#pragma unroll
            for (int k = 0; k < 12; k++) jac[12 * ((size_t)b * cap + i) + k] = J[k];
    }
    if (!partial) return;
    __shared__ double S[4][kNE];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < kNE; k++) {
        const double s = wave_sum(e[k]);
        if (lane == 0) S[wv][k] = s;
    }
    __syncthreads();
    if (threadIdx.x < kNE) {
        const int k = threadIdx.x;
        partial[((size_t)b * gridDim.x + blockIdx.x) * kNE + k] = ((S[0][k] + S[1][k]) + S[2][k]) + S[3][k];
    }
}

__global__ void reproj_reduce_kernel(const double* __restrict__ partial, int nblk, int nprob, double* __restrict__ out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nprob * kNE) return;
    const int b = t / kNE, k = t - b * kNE;
    double s = 0;
    for (int j = 0; j < nblk; j++) s += partial[((size_t)b * nblk + j) * kNE + k];
    out[t] = s;
}

}  // namespace

size_t reproj_partial_doubles(int n_problems, int max_n) {
    return (size_t)n_problems * ((max_n + 255) / 256) * kNE;
}

hipError_t launch_reproj(const double* d_obj, const float* d_img, const int* d_counts, int n_problems, int cap,
                         int max_n, const double* d_poses, const double K[9], double delta, double* d_res,
                         double* d_jac, double* d_partial, double* d_normal, hipStream_t st) {
    if (n_problems <= 0 || max_n <= 0) {
        if (d_normal && n_problems > 0)
            return hipMemsetAsync(d_normal, 0, sizeof(double) * kNE * (size_t)n_problems, st);
        return hipSuccess;
    }
    const int nblk = (max_n + 255) / 256;
    hipLaunchKernelGGL(reproj_kernel, dim3(nblk, n_problems), dim3(256), 0, st, d_obj, d_img, d_counts, cap, d_poses,
                       K[0], K[4], K[2], K[5], delta, d_res, d_jac, d_normal ? d_partial : nullptr);
    if (d_normal) {
        const int tot = n_problems * kNE;
        hipLaunchKernelGGL(reproj_reduce_kernel, dim3((tot + 255) / 256), dim3(256), 0, st, d_partial, nblk,
                           n_problems, d_normal);
    }
    return hipGetLastError();
}

}  // namespace svo
