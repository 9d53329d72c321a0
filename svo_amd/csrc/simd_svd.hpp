// la::cv::jacobi_svd<M, N, WANT_V> (OpenCV's JacobiSVDImpl_, linalg.hpp) of L
// independent matrices at once, one matrix per SIMD lane (host only). Every lane
// runs exactly the scalar algorithm's operations in the scalar order -- the
// sequential dot products stay sequential per lane, a pair a lane skips leaves
// its rows untouched (blend, not a unit rotation), a lane whose sweep rotated
// nothing stops rotating -- so each lane's result is bit-identical to the
// scalar routine's (tests/test_epnp_cpu.py compares the EPnP solver built on it,
// epnp_lanes.hpp, with the oracle's scalar restatement).
//
// The templates sit in an anonymous namespace: each translation unit that
// includes this header is built for one instruction set (epnp_avx2.cpp with
// -mavx2, epnp_avx512.cpp with -mavx512f) and keeps its own instantiations, so
// the linker never folds an AVX-512 body into the AVX2 path.
#pragma once

#include <cmath>
#include <cstring>

#include "linalg.hpp"

namespace svo {
namespace la {
namespace cv {
namespace {

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
// and the normalisation of every row (vector; a row's scale is its own norm
// wherever the sort moves it), then per lane the selection sort's permutation
// (the scalar routine's swaps replayed on indices) applied to At and Vt. A zero
// singular value in any lane: the scalar tail (its random-vector path) per lane.
template <int M, int N, int L, bool WANT_V>
inline void lanes_tail(vd<L>* At, vd<L>* Wout, vd<L>* Vt) {
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
    if (zero) {
        for (int l = 0; l < L; l++) {
            double Al[N * M], Wl[N], Vl[WANT_V ? N * N : 1];
            for (int i = 0; i < N * M; i++) Al[i] = At[i][l];
            if (WANT_V)
                for (int i = 0; i < N * N; i++) Vl[i] = Vt[i][l];
            jacobi_tail<M, N, WANT_V>(Al, Wl, WANT_V ? Vl : nullptr);
            for (int i = 0; i < N * M; i++) At[i][l] = Al[i];
            if (WANT_V)
                for (int i = 0; i < N * N; i++) Vt[i][l] = Vl[i];
            for (int i = 0; i < N; i++) Wout[i][l] = Wl[i];
        }
        return;
    }
    for (int i = 0; i < N; i++)
        for (int k = 0; k < M; k++) At[i * M + k] *= sc[i];
    vd<L> out[N * M];
    vd<L> vout[WANT_V ? N * N : 1];
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
            if (WANT_V)
                for (int k = 0; k < N; k++) vout[i * N + k][l] = Vt[perm[i] * N + k][l];
        }
    }
    for (int i = 0; i < N * M; i++) At[i] = out[i];
    if (WANT_V)
        for (int i = 0; i < N * N; i++) Vt[i] = vout[i];
}

// At[g][i * M + k]: element (i, k) of every lane's At (N rows of M) in each of G
// lane groups (the groups' chains interleave: a pair's dot product, rotation
// coefficients and rotation form one serial chain per matrix, so one group of
// lanes alone leaves part of the core idle); W: the lanes' singular values
// (descending) on return, At the normalised left vectors, Vt (WANT_V; N x N per
// group) the right vectors as rows.
template <int M, int N, int L, int G, bool WANT_V>
inline void jacobi_svd_lanes(vd<L> (*At)[N * M], vd<L> (*Wout)[N], vd<L> (*Vt)[N * N]) {
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
            if (WANT_V) {
                for (int k = 0; k < N; k++) Vt[g][i * N + k] = 0;
                Vt[g][i * N + i] = 1;
            }
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
                    // hypot_cv(p, beta): each lane the division and square root of
                    // its own branch (the larger magnitude over the smaller one's
                    // ratio), so the lanes issue one of each instead of both forms
                    const vd<L> ha = vabs(pp), hb = vabs(beta);
                    const vm<L> agt = ha > hb;
                    const vd<L> big = vsel(agt, ha, hb), sml = vsel(agt, hb, ha);
                    const vd<L> rr = sml / big;
                    const vd<L> gamma = vsel(agt | (hb > 0), big * vsqrt(1 + rr * rr), vd<L>(0));
                    // the beta < 0 and beta >= 0 coefficient forms, one per lane:
                    //   beta < 0:  s = sqrt(((gamma - beta) * 0.5) / gamma), c = pp / (gamma * s * 2)
                    //   beta >= 0: c = sqrt((gamma + beta) / (gamma * 2)),   s = pp / (gamma * c * 2)
                    const vm<L> neg = beta < 0;
                    const vd<L> num = vsel(neg, (gamma - beta) * 0.5, gamma + beta);
                    const vd<L> den = vsel(neg, gamma, gamma * 2);
                    const vd<L> first = vsqrt(num / den);
                    const vd<L> second = pp / (gamma * first * 2);
                    const vd<L> c = vsel(neg, second, first), s = vsel(neg, first, second);
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
                    if (WANT_V) {
                        vd<L>* Vi = Vt[g] + i * N;
                        vd<L>* Vj = Vt[g] + j * N;
                        for (int k = 0; k < N; k++) {
                            const vd<L> t0 = c * Vi[k] + s * Vj[k];
                            const vd<L> t1 = -s * Vi[k] + c * Vj[k];
                            Vi[k] = vsel(r, t0, Vi[k]);
                            Vj[k] = vsel(r, t1, Vj[k]);
                        }
                    }
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
    for (int g = 0; g < G; g++) lanes_tail<M, N, L, WANT_V>(At[g], Wout[g], WANT_V ? Vt[g] : nullptr);
}

// svd_ut<N> of L * G square matrices (A[q]: row-major N x N, q = g * L + l):
// ut[q] rows = left singular vectors, w[q] descending; bit-identical to svd_ut<N>
template <int N, int L, int G>
inline void svd_ut_lanes(const double* const* A, double* const* w, double* const* ut) {
    vd<L> At[G][N * N], W[G][N];
    for (int g = 0; g < G; g++)
        for (int i = 0; i < N; i++)
            for (int k = 0; k < N; k++)
                for (int l = 0; l < L; l++) At[g][i * N + k][l] = A[g * L + l][k * N + i];
    jacobi_svd_lanes<N, N, L, G, false>(At, W, nullptr);
    for (int g = 0; g < G; g++)
        for (int l = 0; l < L; l++) {
            for (int i = 0; i < N; i++) w[g * L + l][i] = W[g][i][l];
            for (int i = 0; i < N * N; i++) ut[g * L + l][i] = At[g][i][l];
        }
}

}  // namespace
}  // namespace cv
}  // namespace la
}  // namespace svo
