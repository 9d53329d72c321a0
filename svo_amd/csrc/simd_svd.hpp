// la::cv::jacobi_svd<M, N, false> (OpenCV's JacobiSVDImpl_, linalg.hpp) of L
// independent matrices at once, one matrix per SIMD lane (host only). Every lane
// runs exactly the scalar algorithm's operations in the scalar order -- the
// sequential dot products stay sequential per lane, a pair a lane skips leaves
// its rows untouched (blend, not a unit rotation), a lane whose sweep rotated
// nothing stops rotating -- so each lane's result is bit-identical to the
// scalar routine's (tests/test_epnp_cpu.py compares the EPnP solver built on it
// with the oracle's scalar restatement). What changes is the instruction count:
// the 12 x 12 M^T M SVD is ~80 % of an EPnP solve and serial within one matrix,
// so the minimal solver batches hypotheses across lanes instead.
#pragma once

#include <cmath>
#include <cstring>

#include "linalg.hpp"

// every function below is compiled for AVX2 (the 4-lane double vectors in one
// register); callers check simd_svd_ok() first and fall back to the scalar
// routine, whose results are the same bits
#pragma clang attribute push(__attribute__((target("avx2"))), apply_to = function)

namespace svo {
namespace la {
namespace cv {

template <int L>
using vd = double __attribute__((ext_vector_type(L)));
template <int L>
using vm = long __attribute__((ext_vector_type(L)));

template <int L>
__attribute__((always_inline)) inline vd<L> vsel(vm<L> m, vd<L> a, vd<L> b) {  // m lane true (all ones): a
    return m ? a : b;
}
template <int L>
__attribute__((always_inline)) inline vd<L> vsqrt(vd<L> x) {
    return __builtin_elementwise_sqrt(x);
}
template <int L>
__attribute__((always_inline)) inline vd<L> vabs(vd<L> x) {
    return __builtin_elementwise_abs(x);
}
template <int L>
__attribute__((always_inline)) inline bool vany(vm<L> m) {
    for (int l = 0; l < L; l++)
        if (m[l]) return true;
    return false;
}

// the tail of jacobi_svd for one lane group, after the sweeps: singular values
// and the normalisation of every row (vector; a row's scale
// is its own norm wherever the sort moves it), then per lane the selection
// sort's permutation (the scalar routine's swaps replayed on indices)
template <int M, int N, int L>
inline void lanes_tail(vd<L>* At, vd<L>* Wout) {
    const double minval = 2.2250738585072014e-308;
    vd<L> w[N], sc[N];
    bool zero = false;
    for (int i = 0; i < N; i++) {
        vd<L> sd = 0;
        for (int k = 0; k < M; k++) sd += At[i * M + k] * At[i * M + k];
        w[i] = vsqrt(sd);
        const vm<L> big = w[i] > minval;
        zero |= vany(~big);
        sc[i] = vsel(big, 1 / w[i], vd<L>(0));
    }
    if (zero) {  // a zero singular value: the scalar routine's random-vector path, per lane
        for (int l = 0; l < L; l++) {
            double Al[N * M], Wl[N];
            for (int i = 0; i < N * M; i++) Al[i] = At[i][l];
            jacobi_tail<M, N, false>(Al, Wl, nullptr);
            for (int i = 0; i < N * M; i++) At[i][l] = Al[i];
            for (int i = 0; i < N; i++) Wout[i][l] = Wl[i];
        }
        return;
    }
    for (int i = 0; i < N; i++)
        for (int k = 0; k < M; k++) At[i * M + k] *= sc[i];
    vd<L> out[N * M];
    for (int l = 0; l < L; l++) {
        int perm[N];
        double wl[N];
        for (int i = 0; i < N; i++) {
            perm[i] = i;
            wl[i] = w[i][l];
        }
        for (int i = 0; i < N - 1; i++) {
            int j = i;
            for (int k = i + 1; k < N; k++)
                if (wl[j] < wl[k]) j = k;
            if (i != j) {
                const double tw = wl[i];
                wl[i] = wl[j];
                wl[j] = tw;
                const int tp = perm[i];
                perm[i] = perm[j];
                perm[j] = tp;
            }
        }
        for (int i = 0; i < N; i++) {
            Wout[i][l] = wl[i];
            for (int k = 0; k < M; k++) out[i * M + k][l] = At[perm[i] * M + k][l];
        }
    }
    for (int i = 0; i < N * M; i++) At[i] = out[i];
}

// At[g][i * M + k]: element (i, k) of every lane's At (N rows of M) in each of G
// lane groups (the groups' chains interleave: a pair's dot product, rotation
// coefficients and rotation form one serial chain per matrix, ~150 cycles of
// latency, so one group of lanes alone would leave the core mostly idle); W:
// the lanes' singular values (descending) on return, At the normalised left
// vectors.
template <int M, int N, int L, int G>
inline void jacobi_svd_lanes(vd<L> (*At)[N * M], vd<L> (*Wout)[N]) {
    const double eps = 2.220446049250313e-16 * 10;
    constexpr int max_iter = M > 30 ? M : 30;
    vd<L> W[G][N];
    vm<L> live[G];
    for (int g = 0; g < G; g++) {
        live[g] = vm<L>(-1);
        for (int i = 0; i < N; i++) {
            vd<L> sd = 0;
            for (int k = 0; k < M; k++) sd += At[g][i * M + k] * At[g][i * M + k];
            W[g][i] = sd;
        }
    }
    for (int iter = 0; iter < max_iter; iter++) {
        vm<L> changed[G];
        for (int g = 0; g < G; g++) changed[g] = vm<L>(0);
        for (int i = 0; i < N - 1; i++)
            for (int j = i + 1; j < N; j++) {
                vd<L> p[G];
                vm<L> rot[G];
                bool anyrot = false;
                for (int g = 0; g < G; g++) {
                    const vd<L>* Ai = At[g] + i * M;
                    const vd<L>* Aj = At[g] + j * M;
                    p[g] = 0;
                    for (int k = 0; k < M; k++) p[g] += Ai[k] * Aj[k];
                    rot[g] = live[g] & ~(vabs(p[g]) <= eps * vsqrt(W[g][i] * W[g][j]));
                    anyrot |= vany(rot[g]);
                }
                if (!anyrot) continue;
                for (int g = 0; g < G; g++) {
                    vd<L>* Ai = At[g] + i * M;
                    vd<L>* Aj = At[g] + j * M;
                    const vd<L> pp = p[g] * 2;
                    const vd<L> beta = W[g][i] - W[g][j];
                    // hypot_cv(p, beta)
                    const vd<L> ha = vabs(pp), hb = vabs(beta);
                    const vd<L> rb = hb / ha, ra = ha / hb;
                    const vd<L> g1 = ha * vsqrt(1 + rb * rb), g2 = hb * vsqrt(1 + ra * ra);
                    const vd<L> gamma = vsel(ha > hb, g1, vsel(hb > 0, g2, vd<L>(0)));
                    // the beta < 0 and beta >= 0 coefficient forms
                    const vd<L> delta = (gamma - beta) * 0.5;
                    const vd<L> s_n = vsqrt(delta / gamma);
                    const vd<L> c_n = pp / (gamma * s_n * 2);
                    const vd<L> c_p = vsqrt((gamma + beta) / (gamma * 2));
                    const vd<L> s_p = pp / (gamma * c_p * 2);
                    const vm<L> neg = beta < 0;
                    const vd<L> c = vsel(neg, c_n, c_p), s = vsel(neg, s_n, s_p);
                    const vm<L> r = rot[g];
                    vd<L> na = 0, nb = 0;
                    for (int k = 0; k < M; k++) {
                        const vd<L> t0 = c * Ai[k] + s * Aj[k];
                        const vd<L> t1 = -s * Ai[k] + c * Aj[k];
                        Ai[k] = vsel(r, t0, Ai[k]);
                        Aj[k] = vsel(r, t1, Aj[k]);
                        na += t0 * t0;
                        nb += t1 * t1;
                    }
                    W[g][i] = vsel(r, na, W[g][i]);
                    W[g][j] = vsel(r, nb, W[g][j]);
                    changed[g] |= r;
                }
            }
        bool any = false;
        for (int g = 0; g < G; g++) {
            live[g] &= changed[g];
            any |= vany(live[g]);
        }
        if (!any) break;
    }
    for (int g = 0; g < G; g++) lanes_tail<M, N, L>(At[g], Wout[g]);
}

// svd_ut<N> of L square matrices (A[q]: row-major N x N): ut[q] rows = left
// singular vectors, w[q] descending; bit-identical to L calls of svd_ut<N>.
// A[q], q < L * G (q = g * L + l).
template <int N, int L, int G>
inline void svd_ut_lanes(const double* const* A, double* const* w, double* const* ut) {
    vd<L> At[G][N * N], W[G][N];
    for (int g = 0; g < G; g++)
        for (int i = 0; i < N; i++)
            for (int k = 0; k < N; k++)
                for (int l = 0; l < L; l++) At[g][i * N + k][l] = A[g * L + l][k * N + i];
    jacobi_svd_lanes<N, N, L, G>(At, W);
    for (int g = 0; g < G; g++)
        for (int l = 0; l < L; l++) {
            for (int i = 0; i < N; i++) w[g * L + l][i] = W[g][i][l];
            for (int i = 0; i < N * N; i++) ut[g * L + l][i] = At[g][i][l];
        }
}

}  // namespace cv
}  // namespace la
}  // namespace svo

#pragma clang attribute pop

namespace svo {
namespace la {
namespace cv {
inline bool simd_svd_ok() {
    static const bool ok = __builtin_cpu_supports("avx2");
    return ok;
}
}  // namespace cv
}  // namespace la
}  // namespace svo
