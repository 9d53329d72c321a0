// EPnP minimal solver, one wave (64 lanes) per hypothesis, for gfx950: the same
// arithmetic as the host solver (epnp.hpp, linalg.hpp), operation for operation,
// so the poses are bit-identical (-ffp-contract=off), with the work split where
// it parallelises without reassociating any sum:
//   * M^T M: lane e owns entries e, e + 64, e + 128 (sum over the 5 points in order);
//   * the 12 x 12 eigenproblem (linalg.hpp sym_eig_ql_t<12>, EISPACK tred2 / tql2):
//     the working matrix, d and e live in LDS; every reduction the host does in a
//     fixed order stays a serial loop of one lane-uniform chain, and what the host
//     updates element by element from values fixed before the loop (the rank-2
//     updates, the back-transformation rows, the QL rotations' row pairs) is
//     spread over lanes;
//   * make_L: lane e < 60 forms one entry;
//   * the rest (3 x 3 Jacobi eigen / SVDs, the 6 x {3,4,5} Householder QR solves,
//     Gauss-Newton, Procrustes, Rodrigues) runs lane-uniform in registers
//     (compile-time sizes, fully unrolled).
// Reference call: cv::solvePnPRansac's minimal solver (SOLVEPNP_EPNP on 5 points),
// R:src/tracking.cpp:191-196.
#pragma once

#include "linalg.hpp"

// phase time stamps for tools/epnp_wave_probe.hip (no-op in the library)
#ifndef WEP_STAMP
#define WEP_STAMP(k)
#endif

namespace svo {
namespace wep {

constexpr int kN = 12;

// per-wave LDS workspace
struct Work {
    double W[kN * kN];  // M^T M, then V^T (tred2 / tql2)
    double d[kN], e[kN];
    double Vt[4 * kN];  // eigenvectors of the 4 smallest eigenvalues: rows 8..11 of the sorted Vt
    double L[60];
    int ord[kN];
};

// one-wave blocks: the barrier is a no-op in hardware; it orders the LDS traffic
// (compiler and memory) between lane-parallel writes and lane-uniform reads
__device__ __forceinline__ void wsync() { __syncthreads(); }

template <int N>
__device__ __forceinline__ double sel(const double (&a)[N], int i) {
    double r = a[0];
#pragma unroll
    for (int k = 1; k < N; k++) r = i == k ? a[k] : r;
    return r;
}

// insertion sort of indices, descending by key, ties kept in order (the host's
// `while (j >= 0 && key[order[j]] < key[v])` loop), with compile-time slots
template <int N>
__device__ __forceinline__ void sort_desc(const double (&key)[N], int (&order)[N]) {
#pragma unroll
    for (int i = 0; i < N; i++) order[i] = i;
#pragma unroll
    for (int i = 1; i < N; i++) {
        const int v = i;  // order[i] == i here: slots right of i are untouched
        const double kv = key[i];
        bool moving = true;
#pragma unroll
        for (int jj = i - 1; jj >= 0; jj--) {
            if (moving) {
                if (sel(key, order[jj]) < kv) {
                    order[jj + 1] = order[jj];
                } else {
                    order[jj + 1] = v;
                    moving = false;
                }
            }
        }
        if (moving) order[0] = v;
    }
}

// la::sym_eig for n = 3 (cyclic Jacobi), registers
__device__ __forceinline__ void sym_eig3(double (&A)[9], double (&w)[3], double (&V)[9]) {
    constexpr int n = 3;
    double Q[9];
#pragma unroll
    for (int i = 0; i < 9; i++) Q[i] = 0;
#pragma unroll
    for (int i = 0; i < n; i++) Q[i * n + i] = 1;
    for (int sweep = 0; sweep < 60; sweep++) {
        double off = 0, tot = 0;
#pragma unroll
        for (int p = 0; p < n; p++)
#pragma unroll
            for (int q = 0; q < n; q++) {
                double v = A[p * n + q] * A[p * n + q];
                tot += v;
                if (p != q) off += v;
            }
        if (off == 0 || off <= 1e-32 * tot) break;
#pragma unroll
        for (int p = 0; p < n - 1; p++)
#pragma unroll
            for (int q = p + 1; q < n; q++) {
                const double apq = A[p * n + q];
                if (apq == 0) continue;
                const double theta = (A[q * n + q] - A[p * n + p]) / (2 * apq);
                const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1));
                const double c = 1 / sqrt(t * t + 1), s = t * c;
#pragma unroll
                for (int k = 0; k < n; k++) {
                    const double a = A[k * n + p], b = A[k * n + q];
                    A[k * n + p] = c * a - s * b;
                    A[k * n + q] = s * a + c * b;
                }
#pragma unroll
                for (int k = 0; k < n; k++) {
                    const double a = A[p * n + k], b = A[q * n + k];
                    A[p * n + k] = c * a - s * b;
                    A[q * n + k] = s * a + c * b;
                }
#pragma unroll
                for (int k = 0; k < n; k++) {
                    const double a = Q[k * n + p], b = Q[k * n + q];
                    Q[k * n + p] = c * a - s * b;
                    Q[k * n + q] = s * a + c * b;
                }
            }
    }
    double dg[3] = {A[0], A[4], A[8]};
    int order[3];
    sort_desc<3>(dg, order);
#pragma unroll
    for (int i = 0; i < n; i++) {
        w[i] = sel(dg, order[i]);
#pragma unroll
        for (int k = 0; k < n; k++) {
            const double qk[3] = {Q[k * n + 0], Q[k * n + 1], Q[k * n + 2]};
            V[i * n + k] = sel(qk, order[i]);
        }
    }
}

// la::svd for a 3 x 3 matrix (one-sided Jacobi), registers
__device__ __forceinline__ void svd3(const double (&a)[9], double (&s)[3], double (&U)[9], double (&Vt)[9]) {
    constexpr int m = 3, n = 3;
    double W[9], V[9];
#pragma unroll
    for (int i = 0; i < 9; i++) W[i] = a[i];
#pragma unroll
    for (int i = 0; i < 9; i++) V[i] = 0;
#pragma unroll
    for (int i = 0; i < n; i++) V[i * n + i] = 1;
    for (int sweep = 0; sweep < 60; sweep++) {
        bool rotated = false;
#pragma unroll
        for (int p = 0; p < n - 1; p++)
#pragma unroll
            for (int q = p + 1; q < n; q++) {
                double al = 0, be = 0, ga = 0;
#pragma unroll
                for (int k = 0; k < m; k++) {
                    al += W[k * n + p] * W[k * n + p];
                    be += W[k * n + q] * W[k * n + q];
                    ga += W[k * n + p] * W[k * n + q];
                }
                if (ga == 0 || fabs(ga) <= 1e-15 * sqrt(al * be)) continue;
                rotated = true;
                const double z = (be - al) / (2 * ga);
                const double t = (z >= 0 ? 1.0 : -1.0) / (fabs(z) + sqrt(1 + z * z));
                const double c = 1 / sqrt(1 + t * t), sn = c * t;
#pragma unroll
                for (int k = 0; k < m; k++) {
                    const double x = W[k * n + p], y = W[k * n + q];
                    W[k * n + p] = c * x - sn * y;
                    W[k * n + q] = sn * x + c * y;
                }
#pragma unroll
                for (int k = 0; k < n; k++) {
                    const double x = V[k * n + p], y = V[k * n + q];
                    V[k * n + p] = c * x - sn * y;
                    V[k * n + q] = sn * x + c * y;
                }
            }
        if (!rotated) break;
    }
    double nrm[3];
#pragma unroll
    for (int j = 0; j < n; j++) {
        double acc = 0;
#pragma unroll
        for (int k = 0; k < m; k++) acc += W[k * n + j] * W[k * n + j];
        nrm[j] = sqrt(acc);
    }
    int order[3];
    sort_desc<3>(nrm, order);
#pragma unroll
    for (int i = 0; i < n; i++) {
        const int c = order[i];
        const double nc = sel(nrm, c);
        s[i] = nc;
#pragma unroll
        for (int k = 0; k < n; k++) {
            const double vk[3] = {V[k * n + 0], V[k * n + 1], V[k * n + 2]};
            Vt[i * n + k] = sel(vk, c);
        }
#pragma unroll
        for (int k = 0; k < m; k++) {
            const double wk[3] = {W[k * n + 0], W[k * n + 1], W[k * n + 2]};
            U[k * n + i] = nc > 0 ? sel(wk, c) / nc : 0;
        }
    }
}

__device__ __forceinline__ void pinv3(const double (&A)[9], double (&Ai)[9]) {
    double s[3], U[9], Vt[9];
    svd3(A, s, U, Vt);
    const double tol = s[0] * 3 * 2.220446049250313e-16;
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) {
            double acc = 0;
#pragma unroll
            for (int k = 0; k < 3; k++)
                if (s[k] > tol) acc += Vt[k * 3 + i] * U[j * 3 + k] / s[k];
            Ai[i * 3 + j] = acc;
        }
}

__device__ __forceinline__ double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

// EPnP::qr_solve with compile-time sizes (nr = 6)
template <int NC>
__device__ __forceinline__ void qr_solve(double (&A)[6 * NC], double (&b)[6], double (&X)[NC]) {
    constexpr int nr = 6, nc = NC;
    double A1[NC], A2[NC];
    bool zero = false;
#pragma unroll
    for (int k = 0; k < nc; k++) {
        if (zero) continue;
        double eta = 0;
#pragma unroll
        for (int i = k; i < nr; i++) eta = fmax(eta, fabs(A[i * nc + k]));
        if (eta == 0) {
            zero = true;
            continue;
        }
        double sum2 = 0.0;
        const double ie = 1. / eta;
#pragma unroll
        for (int i = k; i < nr; i++) {
            A[i * nc + k] *= ie;
            sum2 += A[i * nc + k] * A[i * nc + k];
        }
        double sigma = sqrt(sum2);
        if (A[k * nc + k] < 0) sigma = -sigma;
        A[k * nc + k] += sigma;
        A1[k] = sigma * A[k * nc + k];
        A2[k] = -eta * sigma;
#pragma unroll
        for (int j = k + 1; j < nc; j++) {
            double s = 0;
#pragma unroll
            for (int i = k; i < nr; i++) s += A[i * nc + k] * A[i * nc + j];
            const double tau = s / A1[k];
#pragma unroll
            for (int i = k; i < nr; i++) A[i * nc + j] -= tau * A[i * nc + k];
        }
    }
    if (zero) {
#pragma unroll
        for (int j = 0; j < nc; j++) X[j] = 0;
        return;
    }
#pragma unroll
    for (int j = 0; j < nc; j++) {
        double tau = 0;
#pragma unroll
        for (int i = j; i < nr; i++) tau += A[i * nc + j] * b[i];
        tau /= A1[j];
#pragma unroll
        for (int i = j; i < nr; i++) b[i] -= tau * A[i * nc + j];
    }
    X[nc - 1] = b[nc - 1] / A2[nc - 1];
#pragma unroll
    for (int i = nc - 2; i >= 0; i--) {
        double s = 0;
#pragma unroll
        for (int j = i + 1; j < nc; j++) s += A[i * nc + j] * X[j];
        X[i] = (b[i] - s) / A2[i];
    }
}

// EPnP::betas_approx (which = 1, 2, 3) from L (LDS) and rho
template <int WHICH>
__device__ __forceinline__ void betas_approx(const double* L, const double (&rho)[6], double (&b)[4]) {
    if constexpr (WHICH == 1) {
        constexpr int cols1[4] = {0, 1, 3, 6};
        double A[24], bq[6], x[4];
#pragma unroll
        for (int i = 0; i < 6; i++) {
#pragma unroll
            for (int k = 0; k < 4; k++) A[4 * i + k] = L[10 * i + cols1[k]];
            bq[i] = rho[i];
        }
        qr_solve<4>(A, bq, x);
        const double sg = x[0] < 0 ? -1.0 : 1.0;
        b[0] = sqrt(sg * x[0]);
        b[1] = sg * x[1] / b[0];
        b[2] = sg * x[2] / b[0];
        b[3] = sg * x[3] / b[0];
    } else {
        constexpr int nc = WHICH == 2 ? 3 : 5;
        double A[6 * nc], bq[6], x[nc];
#pragma unroll
        for (int i = 0; i < 6; i++) {
#pragma unroll
            for (int k = 0; k < nc; k++) A[nc * i + k] = L[10 * i + k];
            bq[i] = rho[i];
        }
        qr_solve<nc>(A, bq, x);
        if (x[0] < 0) {
            b[0] = sqrt(-x[0]);
            b[1] = (x[2] < 0) ? sqrt(-x[2]) : 0.0;
        } else {
            b[0] = sqrt(x[0]);
            b[1] = (x[2] > 0) ? sqrt(x[2]) : 0.0;
        }
        if (x[1] < 0) b[0] = -b[0];
        if constexpr (WHICH == 3)
            b[2] = x[3] / b[0];
        else
            b[2] = 0.0;
        b[3] = 0.0;
    }
}

__device__ __forceinline__ void gauss_newton(const double* L, const double (&rho)[6], double (&be)[4]) {
    for (int it = 0; it < 5; it++) {
        double A[24], b[6], x[4];
#pragma unroll
        for (int i = 0; i < 6; i++) {
            const double* r = L + 10 * i;
            A[4 * i + 0] = 2 * r[0] * be[0] + r[1] * be[1] + r[3] * be[2] + r[6] * be[3];
            A[4 * i + 1] = r[1] * be[0] + 2 * r[2] * be[1] + r[4] * be[2] + r[7] * be[3];
            A[4 * i + 2] = r[3] * be[0] + r[4] * be[1] + 2 * r[5] * be[2] + r[8] * be[3];
            A[4 * i + 3] = r[6] * be[0] + r[7] * be[1] + r[8] * be[2] + 2 * r[9] * be[3];
            b[i] = rho[i] - (r[0] * be[0] * be[0] + r[1] * be[0] * be[1] + r[2] * be[1] * be[1] + r[3] * be[0] * be[2] +
                             r[4] * be[1] * be[2] + r[5] * be[2] * be[2] + r[6] * be[0] * be[3] + r[7] * be[1] * be[3] +
                             r[8] * be[2] * be[3] + r[9] * be[3] * be[3]);
        }
        qr_solve<4>(A, b, x);
#pragma unroll
        for (int i = 0; i < 4; i++) be[i] += x[i];
    }
}

// The cooperative 12 x 12 eigen-decomposition (sym_eig_ql_t<12>) of S.W (symmetric,
// stored as its own transpose); leaves the rows of Vt for the 4 smallest
// eigenvalues (sorted rows 8..11) in S.Vt. Every lane runs this.
__device__ inline void eig12(Work& S, int lane) {
    constexpr int n = kN;
    double* W = S.W;
    double* d = S.d;
    double* e = S.e;
    // tred2
    WEP_STAMP(1);
    if (lane < n) d[lane] = W[lane * n + n - 1];
    wsync();
    for (int i = n - 1; i > 0; i--) {
        double scale = 0, h = 0;
        for (int k = 0; k < i; k++) scale += fabs(d[k]);
        if (scale == 0) {
            const double ei = d[i - 1];
            if (lane < i) {
                const int j = lane;
                const double dj = W[j * n + i - 1];
                W[j * n + i] = 0;
                W[i * n + j] = 0;
                d[j] = dj;
            }
            wsync();
            if (lane == 0) e[i] = ei;
        } else {
            if (lane < i) d[lane] = d[lane] / scale;
            wsync();
            for (int k = 0; k < i; k++) h += d[k] * d[k];
            double f = d[i - 1];
            double g = sqrt(h);
            if (f > 0) g = -g;
            const double ei = scale * g;
            h = h - f * g;
            wsync();
            if (lane == 0) {
                e[i] = ei;
                d[i - 1] = f - g;
            }
            wsync();
            // W[i][j] = d[j]; e[k] = sum_{j<k} W[j][k] d[j] + W[k][k] d[k] + sum_{k'>k} W[k][k'] d[k']
            double acc = 0;
            if (lane < i) {
                const int k = lane;
                for (int j = 0; j < k; j++) acc += W[j * n + k] * d[j];
                acc = acc + W[k * n + k] * d[k];
                for (int k2 = k + 1; k2 <= i - 1; k2++) acc += W[k * n + k2] * d[k2];
            }
            wsync();
            if (lane < i) {
                W[i * n + lane] = d[lane];
                e[lane] = acc / h;  // e[j] /= h
            }
            wsync();
            f = 0;
            for (int j = 0; j < i; j++) f += e[j] * d[j];
            const double hh = f / (h + h);
            wsync();
            if (lane < i) e[lane] -= hh * d[lane];
            wsync();
            // W[j][k] -= d[j] e[k] + e[j] d[k] for j <= k <= i-1 (old d throughout)
            for (int t = lane; t < i * i; t += 64) {
                const int j = t / i, k = t - j * i;
                if (k >= j) W[j * n + k] -= (d[j] * e[k] + e[j] * d[k]);
            }
            wsync();
            if (lane < i) {
                const int j = lane;
                const double dj = W[j * n + i - 1];
                W[j * n + i] = 0;
                d[j] = dj;
            }
            wsync();
        }
        if (lane == 0) d[i] = h;
        wsync();
    }
    WEP_STAMP(2);
    for (int i = 0; i < n - 1; i++) {
        if (lane == 0) {
            W[i * n + n - 1] = W[i * n + i];
            W[i * n + i] = 1;
        }
        wsync();
        const double h = d[i + 1];
        if (h != 0) {
            if (lane <= i) d[lane] = W[(i + 1) * n + lane] / h;
            wsync();
            if (lane <= i) {
                const int j = lane;
                double g = 0;
                for (int k = 0; k <= i; k++) g += W[(i + 1) * n + k] * W[j * n + k];
                for (int k = 0; k <= i; k++) W[j * n + k] -= g * d[k];
            }
            wsync();
        }
        if (lane <= i) W[(i + 1) * n + lane] = 0;
        wsync();
    }
    if (lane < n) {
        const double dj = W[lane * n + n - 1];
        W[lane * n + n - 1] = 0;
        d[lane] = dj;
    }
    wsync();
    if (lane == 0) {
        W[(n - 1) * n + n - 1] = 1;
        e[0] = 0;
    }
    wsync();
    // tql2
    WEP_STAMP(3);
    {
        const double v = lane >= 1 && lane < n ? e[lane] : 0.0;
        wsync();
        if (lane >= 1 && lane < n) e[lane - 1] = v;
        wsync();
        if (lane == 0) e[n - 1] = 0;
        wsync();
    }
    double f = 0, tst1 = 0;
    const double eps = 2.220446049250313e-16;
    for (int l = 0; l < n; l++) {
        tst1 = fmax(tst1, fabs(d[l]) + fabs(e[l]));
        int m = l;
        while (m < n - 1 && fabs(e[m]) > eps * tst1) m++;
        if (m > l) {
            for (int iter = 0; iter < 60; iter++) {
                double g = d[l];
                double p = (d[l + 1] - g) / (2 * e[l]);
                double r = sqrt(p * p + 1);
                if (p < 0) r = -r;
                const double el = e[l];
                const double dl = el / (p + r);
                const double dl1 = el * (p + r);
                double h = g - dl;
                wsync();
                if (lane == 0) {
                    d[l] = dl;
                    d[l + 1] = dl1;
                }
                if (lane >= l + 2 && lane < n) d[lane] -= h;
                wsync();
                f += h;
                p = d[m];
                double c = 1, c2 = 1, c3 = 1, s = 0, s2 = 0;
                const double el1 = e[l + 1];
                for (int i = m - 1; i >= l; i--) {
                    c3 = c2;
                    c2 = c;
                    s2 = s;
                    const double ei = e[i], di = d[i];
                    g = c * ei;
                    h = c * p;
                    r = sqrt(p * p + ei * ei);
                    const double ei1 = s * r;
                    s = ei / r;
                    c = p / r;
                    p = c * di - s * g;
                    const double di1 = h + s * (c * g + s * di);
                    if (lane < n) {
                        const int k = lane;
                        const double hk = W[(i + 1) * n + k];
                        const double wk = W[i * n + k];
                        W[(i + 1) * n + k] = s * wk + c * hk;
                        W[i * n + k] = c * wk - s * hk;
                    }
                    wsync();
                    if (lane == 0) {
                        e[i + 1] = ei1;
                        d[i + 1] = di1;
                    }
                    wsync();
                }
                const double el0 = e[l];
                p = -s * s2 * c3 * el1 * el0 / dl1;
                const double nel = s * p, ndl = c * p;
                wsync();
                if (lane == 0) {
                    e[l] = nel;
                    d[l] = ndl;
                }
                wsync();
                if (!(fabs(nel) > eps * tst1)) break;
            }
        }
        const double dl = d[l] + f;
        wsync();
        if (lane == 0) {
            d[l] = dl;
            e[l] = 0;
        }
        wsync();
    }
    WEP_STAMP(4);
    // insertion sort, descending (uniform; the index array in LDS)
    if (lane == 0) {
        int* order = S.ord;
        for (int i = 0; i < n; i++) order[i] = i;
        for (int i = 1; i < n; i++) {
            int v = order[i], j = i - 1;
            while (j >= 0 && d[order[j]] < d[v]) {
                order[j + 1] = order[j];
                j--;
            }
            order[j + 1] = v;
        }
    }
    wsync();
    for (int t = lane; t < 4 * n; t += 64) {
        const int r = t / n, k = t - r * n;  // Vt row 8 + r
        S.Vt[r * n + k] = W[S.ord[8 + r] * n + k];
    }
    wsync();
}

// EPnP on 5 points (obj: 5 x xyz floats, img: 5 x xy floats), as epnp_pixels +
// EPnP::solve; returns the validity flag, R / t uniform in every lane.
__device__ inline bool solve5(Work& S, int lane, const float* obj, const float* img, const double K[9], double (&Rout)[9],
                              double (&tout)[3]) {
    constexpr int np = 5;
    const double fu = K[0], fv = K[4], uc = K[2], vc = K[5];
    double pw[3 * np], uv[2 * np];
    {
        const double ifx = 1. / K[0], ify = 1. / K[4];
#pragma unroll
        for (int k = 0; k < np; k++) {
            pw[3 * k] = obj[3 * k];
            pw[3 * k + 1] = obj[3 * k + 1];
            pw[3 * k + 2] = obj[3 * k + 2];
            const double x = ((double)img[2 * k] - K[2]) * ifx, y = ((double)img[2 * k + 1] - K[5]) * ify;
            uv[2 * k] = x * K[0] + K[2];
            uv[2 * k + 1] = y * K[4] + K[5];
        }
    }
    // control points
    double cws[4][3];
    {
        double c0[3] = {0, 0, 0};
#pragma unroll
        for (int i = 0; i < np; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) c0[j] += pw[3 * i + j];
#pragma unroll
        for (int j = 0; j < 3; j++) c0[j] /= np;
        double C[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < np; i++) {
            double dd[3] = {pw[3 * i] - c0[0], pw[3 * i + 1] - c0[1], pw[3 * i + 2] - c0[2]};
#pragma unroll
            for (int a = 0; a < 3; a++)
#pragma unroll
                for (int b = 0; b < 3; b++) C[a * 3 + b] += dd[a] * dd[b];
        }
        double w[3], V[9];
        sym_eig3(C, w, V);
#pragma unroll
        for (int j = 0; j < 3; j++) cws[0][j] = c0[j];
#pragma unroll
        for (int i = 1; i < 4; i++) {
            const double k = sqrt((w[i - 1] > 0 ? w[i - 1] : 0.0) / np);
#pragma unroll
            for (int j = 0; j < 3; j++) cws[i][j] = c0[j] + k * V[3 * (i - 1) + j];
        }
    }
    // barycentric coordinates
    double alphas[4 * np];
    {
        double CC[9], CI[9];
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 1; j < 4; j++) CC[3 * i + j - 1] = cws[j][i] - cws[0][i];
        pinv3(CC, CI);
#pragma unroll
        for (int i = 0; i < np; i++) {
            const double* p = pw + 3 * i;
            double* a = &alphas[4 * i];
            const double dd[3] = {p[0] - cws[0][0], p[1] - cws[0][1], p[2] - cws[0][2]};
#pragma unroll
            for (int j = 0; j < 3; j++) a[1 + j] = CI[3 * j] * dd[0] + CI[3 * j + 1] * dd[1] + CI[3 * j + 2] * dd[2];
            a[0] = 1.0 - a[1] - a[2] - a[3];
        }
    }
    // M^T M (stored transposed, W[q][p] = MtM[p][q]): lane-parallel entries
    for (int t = lane; t < 144; t += 64) {
        const int p = t / 12, q = t - 12 * p;
        const int kp = p / 3, cp = p - 3 * kp, kq = q / 3, cq = q - 3 * kq;
        double acc = 0;
#pragma unroll
        for (int i = 0; i < np; i++) {
            const double* a = &alphas[4 * i];
            const double u = uv[2 * i], v = uv[2 * i + 1];
            const double apk = kp == 0 ? a[0] : kp == 1 ? a[1] : kp == 2 ? a[2] : a[3];
            const double aqk = kq == 0 ? a[0] : kq == 1 ? a[1] : kq == 2 ? a[2] : a[3];
            const double r1p = cp == 0 ? apk * fu : cp == 1 ? 0.0 : apk * (uc - u);
            const double r1q = cq == 0 ? aqk * fu : cq == 1 ? 0.0 : aqk * (uc - u);
            const double r2p = cp == 0 ? 0.0 : cp == 1 ? apk * fv : apk * (vc - v);
            const double r2q = cq == 0 ? 0.0 : cq == 1 ? aqk * fv : aqk * (vc - v);
            acc += r1p * r1q + r2p * r2q;
        }
        S.W[q * 12 + p] = acc;
    }
    wsync();
    eig12(S, lane);
    WEP_STAMP(5);
    // make_L: lane e < 60 forms L[e] (row i = e / 10: control-point pair, col c)
    if (lane < 60) {
        const int i = lane / 10, c = lane - 10 * i;
        constexpr int pa[6] = {0, 0, 0, 1, 1, 2}, pb[6] = {1, 2, 3, 2, 3, 3};
        const int a = i == 0 ? pa[0] : i == 1 ? pa[1] : i == 2 ? pa[2] : i == 3 ? pa[3] : i == 4 ? pa[4] : pa[5];
        const int b = i == 0 ? pb[0] : i == 1 ? pb[1] : i == 2 ? pb[2] : i == 3 ? pb[3] : i == 4 ? pb[4] : pb[5];
        // v[q] = Vt row 11 - q (ut + 12 * (11 - q)) = S.Vt row 3 - q
        auto dv = [&](int q, double* out) {
            const double* v = S.Vt + 12 * (3 - q);
#pragma unroll
            for (int k = 0; k < 3; k++) out[k] = v[3 * a + k] - v[3 * b + k];
        };
        int x = 0, y = 0;
        bool twice = true;
        switch (c) {
            case 0: x = 0, y = 0, twice = false; break;
            case 1: x = 0, y = 1; break;
            case 2: x = 1, y = 1, twice = false; break;
            case 3: x = 0, y = 2; break;
            case 4: x = 1, y = 2; break;
            case 5: x = 2, y = 2, twice = false; break;
            case 6: x = 0, y = 3; break;
            case 7: x = 1, y = 3; break;
            case 8: x = 2, y = 3; break;
            default: x = 3, y = 3, twice = false; break;
        }
        double u[3], w[3];
        dv(x, u);
        dv(y, w);
        const double dt = dot3(u, w);
        S.L[lane] = twice ? 2.0 * dt : dt;
    }
    wsync();
    double rho[6];
    {
        constexpr int pa[6] = {0, 0, 0, 1, 1, 2}, pb[6] = {1, 2, 3, 2, 3, 3};
#pragma unroll
        for (int i = 0; i < 6; i++) {
            const double* a = cws[pa[i]];
            const double* b = cws[pb[i]];
            rho[i] = (a[0] - b[0]) * (a[0] - b[0]) + (a[1] - b[1]) * (a[1] - b[1]) + (a[2] - b[2]) * (a[2] - b[2]);
        }
    }
    WEP_STAMP(6);
    // betas 1..3 + Gauss-Newton + R, t; best by mean reprojection error
    double Rs[3][9], ts[3][3], err[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        double be[4] = {0, 0, 0, 0};
        if (k == 0) betas_approx<1>(S.L, rho, be);
        if (k == 1) betas_approx<2>(S.L, rho, be);
        if (k == 2) betas_approx<3>(S.L, rho, be);
        gauss_newton(S.L, rho, be);
        // r_and_t
        double ccs[4][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const double* v = S.Vt + 12 * (3 - i);
#pragma unroll
            for (int j = 0; j < 4; j++)
#pragma unroll
                for (int q = 0; q < 3; q++) ccs[j][q] += be[i] * v[3 * j + q];
        }
        double pcs[3 * np];
#pragma unroll
        for (int i = 0; i < np; i++) {
            const double* a = &alphas[4 * i];
#pragma unroll
            for (int j = 0; j < 3; j++)
                pcs[3 * i + j] = a[0] * ccs[0][j] + a[1] * ccs[1][j] + a[2] * ccs[2][j] + a[3] * ccs[3][j];
        }
        if (pcs[2] < 0.0) {
#pragma unroll
            for (int i = 0; i < 3 * np; i++) pcs[i] = -pcs[i];
        }
        double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
#pragma unroll
        for (int i = 0; i < np; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) {
                pc0[j] += pcs[3 * i + j];
                pw0[j] += pw[3 * i + j];
            }
#pragma unroll
        for (int j = 0; j < 3; j++) {
            pc0[j] /= np;
            pw0[j] /= np;
        }
        double abt[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < np; i++) {
            const double* pc = &pcs[3 * i];
            const double* pp = pw + 3 * i;
#pragma unroll
            for (int j = 0; j < 3; j++)
#pragma unroll
                for (int q = 0; q < 3; q++) abt[3 * j + q] += (pc[j] - pc0[j]) * (pp[q] - pw0[q]);
        }
        double s[3], U[9], Vt[9];
        svd3(abt, s, U, Vt);
        double* R = Rs[k];
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) R[3 * i + j] = U[3 * i] * Vt[j] + U[3 * i + 1] * Vt[3 + j] + U[3 * i + 2] * Vt[6 + j];
        const double det = R[0] * R[4] * R[8] + R[1] * R[5] * R[6] + R[2] * R[3] * R[7] - R[2] * R[4] * R[6] -
                           R[1] * R[3] * R[8] - R[0] * R[5] * R[7];
        if (det < 0) {
            R[6] = -R[6];
            R[7] = -R[7];
            R[8] = -R[8];
        }
#pragma unroll
        for (int q = 0; q < 3; q++) ts[k][q] = pc0[q] - dot3(R + 3 * q, pw0);
        double sum = 0.0;
#pragma unroll
        for (int i = 0; i < np; i++) {
            const double* pp = pw + 3 * i;
            const double Xc = dot3(R, pp) + ts[k][0], Yc = dot3(R + 3, pp) + ts[k][1];
            const double iz = 1.0 / (dot3(R + 6, pp) + ts[k][2]);
            const double ue = uc + fu * Xc * iz, ve = vc + fv * Yc * iz;
            const double du = uv[2 * i] - ue, dvv = uv[2 * i + 1] - ve;
            sum += sqrt(du * du + dvv * dvv);
        }
        err[k] = sum / np;
    }
    WEP_STAMP(7);
    int N = 0;
    if (err[1] < err[0]) N = 1;
    if (err[2] < (N == 0 ? err[0] : err[1])) N = 2;
#pragma unroll
    for (int i = 0; i < 9; i++) Rout[i] = N == 0 ? Rs[0][i] : N == 1 ? Rs[1][i] : Rs[2][i];
#pragma unroll
    for (int i = 0; i < 3; i++) tout[i] = N == 0 ? ts[0][i] : N == 1 ? ts[1][i] : ts[2][i];
    bool ok = true;
#pragma unroll
    for (int i = 0; i < 9; i++) ok &= Rout[i] - Rout[i] == 0.0;
#pragma unroll
    for (int i = 0; i < 3; i++) ok &= tout[i] - tout[i] == 0.0;
    return ok;
}

}  // namespace wep
}  // namespace svo
