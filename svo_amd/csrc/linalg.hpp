// Small dense double-precision linear algebra for the pose solvers
// (host now; written __host__ __device__ so the minimal solvers can move onto
// the GPU). Fixed maximum sizes, no allocation.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>

namespace svo {
namespace la {

#define SVO_HD __host__ __device__ inline

// Cyclic Jacobi eigen-decomposition of a symmetric n x n (n <= 12) matrix A
// (row-major, destroyed). Eigenvalues descending in w; eigenvector i in row i of V.
// NC > 0: n = NC at compile time (the loops unroll; the same arithmetic in the
// same order, bit-identical to the runtime-n form).
template <int NC>
SVO_HD void sym_eig_impl(double* A, int n_rt, double* w, double* V) {
    const int n = NC > 0 ? NC : n_rt;
    double Q[NC > 0 ? NC * NC : 144];
    for (int i = 0; i < n * n; i++) Q[i] = 0;
    for (int i = 0; i < n; i++) Q[i * n + i] = 1;
    for (int sweep = 0; sweep < 60; sweep++) {
        double off = 0, tot = 0;
        for (int p = 0; p < n; p++)
            for (int q = 0; q < n; q++) {
                double v = A[p * n + q] * A[p * n + q];
                tot += v;
                if (p != q) off += v;
            }
        if (off == 0 || off <= 1e-32 * tot) break;
        for (int p = 0; p < n - 1; p++)
            for (int q = p + 1; q < n; q++) {
                const double apq = A[p * n + q];
                if (apq == 0) continue;
                const double theta = (A[q * n + q] - A[p * n + p]) / (2 * apq);
                const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1));
                const double c = 1 / sqrt(t * t + 1), s = t * c;
                for (int k = 0; k < n; k++) {
                    const double a = A[k * n + p], b = A[k * n + q];
                    A[k * n + p] = c * a - s * b;
                    A[k * n + q] = s * a + c * b;
                }
                for (int k = 0; k < n; k++) {
                    const double a = A[p * n + k], b = A[q * n + k];
                    A[p * n + k] = c * a - s * b;
                    A[q * n + k] = s * a + c * b;
                }
                for (int k = 0; k < n; k++) {
                    const double a = Q[k * n + p], b = Q[k * n + q];
                    Q[k * n + p] = c * a - s * b;
                    Q[k * n + q] = s * a + c * b;
                }
            }
    }
    int order[NC > 0 ? NC : 12];
    for (int i = 0; i < n; i++) order[i] = i;
    for (int i = 1; i < n; i++) {  // insertion sort, descending
        int v = order[i], j = i - 1;
        while (j >= 0 && A[order[j] * n + order[j]] < A[v * n + v]) {
            order[j + 1] = order[j];
            j--;
        }
        order[j + 1] = v;
    }
    for (int i = 0; i < n; i++) {
        w[i] = A[order[i] * n + order[i]];
        for (int k = 0; k < n; k++) V[i * n + k] = Q[k * n + order[i]];
    }
}
SVO_HD void sym_eig(double* A, int n, double* w, double* V) {
    if (n == 3) return sym_eig_impl<3>(A, 3, w, V);  // EPnP's control points
    sym_eig_impl<0>(A, n, w, V);
}

// Symmetric eigen-decomposition by Householder tridiagonalisation and the
// implicit QL algorithm (EISPACK tred2 / tql2): ~10x fewer flops than cyclic
// Jacobi for the 12x12 EPnP system. Same convention as sym_eig: A (n x n,
// n <= 12, row-major) is read only; eigenvalues descending in w; eigenvector
// i in row i of Vt.
// V (n * n), d, e (n each): workspace the caller provides -- the device fit keeps it
// in LDS (launch_sqpnp_fit), the host on the stack (sym_eig_ql_n)
SVO_HD void sym_eig_ql_ws(const double* A, int n, double* w, double* Vt, double* V, double* d, double* e) {
    for (int i = 0; i < n * n; i++) V[i] = A[i];
    // tred2: V <- orthogonal Q, d/e <- diagonal / off-diagonal of Q^T A Q
    for (int j = 0; j < n; j++) d[j] = V[(n - 1) * n + j];
    for (int i = n - 1; i > 0; i--) {
        double scale = 0, h = 0;
        for (int k = 0; k < i; k++) scale += fabs(d[k]);
        if (scale == 0) {
            e[i] = d[i - 1];
            for (int j = 0; j < i; j++) {
                d[j] = V[(i - 1) * n + j];
                V[i * n + j] = 0;
                V[j * n + i] = 0;
            }
        } else {
            for (int k = 0; k < i; k++) {
                d[k] /= scale;
                h += d[k] * d[k];
            }
            double f = d[i - 1];
            double g = sqrt(h);
            if (f > 0) g = -g;
            e[i] = scale * g;
            h = h - f * g;
            d[i - 1] = f - g;
            for (int j = 0; j < i; j++) e[j] = 0;
            for (int j = 0; j < i; j++) {
                f = d[j];
                V[j * n + i] = f;
                g = e[j] + V[j * n + j] * f;
                for (int k = j + 1; k <= i - 1; k++) {
                    g += V[k * n + j] * d[k];
                    e[k] += V[k * n + j] * f;
                }
                e[j] = g;
            }
            f = 0;
            for (int j = 0; j < i; j++) {
                e[j] /= h;
                f += e[j] * d[j];
            }
            const double hh = f / (h + h);
            for (int j = 0; j < i; j++) e[j] -= hh * d[j];
            for (int j = 0; j < i; j++) {
                f = d[j];
                g = e[j];
                for (int k = j; k <= i - 1; k++) V[k * n + j] -= (f * e[k] + g * d[k]);
                d[j] = V[(i - 1) * n + j];
                V[i * n + j] = 0;
            }
        }
        d[i] = h;
    }
    for (int i = 0; i < n - 1; i++) {
        V[(n - 1) * n + i] = V[i * n + i];
        V[i * n + i] = 1;
        const double h = d[i + 1];
        if (h != 0) {
            for (int k = 0; k <= i; k++) d[k] = V[k * n + i + 1] / h;
            for (int j = 0; j <= i; j++) {
                double g = 0;
                for (int k = 0; k <= i; k++) g += V[k * n + i + 1] * V[k * n + j];
                for (int k = 0; k <= i; k++) V[k * n + j] -= g * d[k];
            }
        }
        for (int k = 0; k <= i; k++) V[k * n + i + 1] = 0;
    }
    for (int j = 0; j < n; j++) {
        d[j] = V[(n - 1) * n + j];
        V[(n - 1) * n + j] = 0;
    }
    V[(n - 1) * n + n - 1] = 1;
    e[0] = 0;
    // tql2: diagonalise the tridiagonal form, accumulating into V
    for (int i = 1; i < n; i++) e[i - 1] = e[i];
    e[n - 1] = 0;
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
                d[l] = e[l] / (p + r);
                d[l + 1] = e[l] * (p + r);
                const double dl1 = d[l + 1];
                double h = g - d[l];
                for (int i = l + 2; i < n; i++) d[i] -= h;
                f += h;
                p = d[m];
                double c = 1, c2 = 1, c3 = 1, s = 0, s2 = 0;
                const double el1 = e[l + 1];
                for (int i = m - 1; i >= l; i--) {
                    c3 = c2;
                    c2 = c;
                    s2 = s;
                    g = c * e[i];
                    h = c * p;
                    r = sqrt(p * p + e[i] * e[i]);
                    e[i + 1] = s * r;
                    s = e[i] / r;
                    c = p / r;
                    p = c * d[i] - s * g;
                    d[i + 1] = h + s * (c * g + s * d[i]);
                    for (int k = 0; k < n; k++) {
                        h = V[k * n + i + 1];
                        V[k * n + i + 1] = s * V[k * n + i] + c * h;
                        V[k * n + i] = c * V[k * n + i] - s * h;
                    }
                }
                p = -s * s2 * c3 * el1 * e[l] / dl1;
                e[l] = s * p;
                d[l] = c * p;
                if (!(fabs(e[l]) > eps * tst1)) break;
            }
        }
        d[l] = d[l] + f;
        e[l] = 0;
    }
    int order[12];
    for (int i = 0; i < n; i++) order[i] = i;
    for (int i = 1; i < n; i++) {  // insertion sort, descending
        int v = order[i], j = i - 1;
        while (j >= 0 && d[order[j]] < d[v]) {
            order[j + 1] = order[j];
            j--;
        }
        order[j + 1] = v;
    }
    for (int i = 0; i < n; i++) {
        w[i] = d[order[i]];
        for (int k = 0; k < n; k++) Vt[i * n + k] = V[k * n + order[i]];
    }
}
SVO_HD void sym_eig_ql_n(const double* A, int n, double* w, double* Vt) {
    double V[144], d[12], e[12];
    sym_eig_ql_ws(A, n, w, Vt, V, d, e);
}

// sym_eig_ql for a compile-time n with V stored transposed, so that the column
// updates of tred2 / tql2 (the rotation loop above all) are contiguous and
// unrolled: the same arithmetic per element in the same order, bit-identical.
template <int N>
SVO_HD void sym_eig_ql_t(const double* A, double* w, double* Vt) {
    constexpr int n = N;
    double W[N * N], d[N], e[N];  // W = V^T: the column updates of tred2 / tql2 run contiguous
    for (int r = 0; r < n; r++)
        for (int c = 0; c < n; c++) W[c * n + r] = A[r * n + c];
    // tred2: V <- orthogonal Q, d/e <- diagonal / off-diagonal of Q^T A Q
    for (int j = 0; j < n; j++) d[j] = W[j * n + n - 1];
    for (int i = n - 1; i > 0; i--) {
        double scale = 0, h = 0;
        for (int k = 0; k < i; k++) scale += fabs(d[k]);
        if (scale == 0) {
            e[i] = d[i - 1];
            for (int j = 0; j < i; j++) {
                d[j] = W[j * n + i - 1];
                W[j * n + i] = 0;
                W[i * n + j] = 0;
            }
        } else {
            for (int k = 0; k < i; k++) {
                d[k] /= scale;
                h += d[k] * d[k];
            }
            double f = d[i - 1];
            double g = sqrt(h);
            if (f > 0) g = -g;
            e[i] = scale * g;
            h = h - f * g;
            d[i - 1] = f - g;
            for (int j = 0; j < i; j++) e[j] = 0;
            for (int j = 0; j < i; j++) {
                f = d[j];
                W[i * n + j] = f;
                g = e[j] + W[j * n + j] * f;
                for (int k = j + 1; k <= i - 1; k++) {
                    g += W[j * n + k] * d[k];
                    e[k] += W[j * n + k] * f;
                }
                e[j] = g;
            }
            f = 0;
            for (int j = 0; j < i; j++) {
                e[j] /= h;
                f += e[j] * d[j];
            }
            const double hh = f / (h + h);
            for (int j = 0; j < i; j++) e[j] -= hh * d[j];
            for (int j = 0; j < i; j++) {
                f = d[j];
                g = e[j];
                for (int k = j; k <= i - 1; k++) W[j * n + k] -= (f * e[k] + g * d[k]);
                d[j] = W[j * n + i - 1];
                W[j * n + i] = 0;
            }
        }
        d[i] = h;
    }
    for (int i = 0; i < n - 1; i++) {
        W[i * n + n - 1] = W[i * n + i];
        W[i * n + i] = 1;
        const double h = d[i + 1];
        if (h != 0) {
            for (int k = 0; k <= i; k++) d[k] = W[(i + 1) * n + k] / h;
            for (int j = 0; j <= i; j++) {
                double g = 0;
                for (int k = 0; k <= i; k++) g += W[(i + 1) * n + k] * W[j * n + k];
                for (int k = 0; k <= i; k++) W[j * n + k] -= g * d[k];
            }
        }
        for (int k = 0; k <= i; k++) W[(i + 1) * n + k] = 0;
    }
    for (int j = 0; j < n; j++) {
        d[j] = W[j * n + n - 1];
        W[j * n + n - 1] = 0;
    }
    W[(n - 1) * n + n - 1] = 1;
    e[0] = 0;
    // tql2: diagonalise the tridiagonal form, accumulating into V
    for (int i = 1; i < n; i++) e[i - 1] = e[i];
    e[n - 1] = 0;
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
                d[l] = e[l] / (p + r);
                d[l + 1] = e[l] * (p + r);
                const double dl1 = d[l + 1];
                double h = g - d[l];
                for (int i = l + 2; i < n; i++) d[i] -= h;
                f += h;
                p = d[m];
                double c = 1, c2 = 1, c3 = 1, s = 0, s2 = 0;
                const double el1 = e[l + 1];
                for (int i = m - 1; i >= l; i--) {
                    c3 = c2;
                    c2 = c;
                    s2 = s;
                    g = c * e[i];
                    h = c * p;
                    r = sqrt(p * p + e[i] * e[i]);
                    e[i + 1] = s * r;
                    s = e[i] / r;
                    c = p / r;
                    p = c * d[i] - s * g;
                    d[i + 1] = h + s * (c * g + s * d[i]);
                    for (int k = 0; k < n; k++) {
                        h = W[(i + 1) * n + k];
                        W[(i + 1) * n + k] = s * W[i * n + k] + c * h;
                        W[i * n + k] = c * W[i * n + k] - s * h;
                    }
                }
                p = -s * s2 * c3 * el1 * e[l] / dl1;
                e[l] = s * p;
                d[l] = c * p;
                if (!(fabs(e[l]) > eps * tst1)) break;
            }
        }
        d[l] = d[l] + f;
        e[l] = 0;
    }
    int order[N];
    for (int i = 0; i < n; i++) order[i] = i;
    for (int i = 1; i < n; i++) {  // insertion sort, descending
        int v = order[i], j = i - 1;
        while (j >= 0 && d[order[j]] < d[v]) {
            order[j + 1] = order[j];
            j--;
        }
        order[j + 1] = v;
    }
    for (int i = 0; i < n; i++) {
        w[i] = d[order[i]];
        for (int k = 0; k < n; k++) Vt[i * n + k] = W[order[i] * n + k];
    }
}


SVO_HD void sym_eig_ql(const double* A, int n, double* w, double* Vt) {
    if (n == 12) return sym_eig_ql_t<12>(A, w, Vt);  // the EPnP system
    sym_eig_ql_n(A, n, w, Vt);
}

// One-sided Jacobi SVD of a (m x n, m <= 12, n <= 12): a = U diag(s) V^T,
// s descending; U is m x n (columns), Vt is n x n (rows). MC, NC > 0: the sizes
// at compile time (unrolled, bit-identical to the runtime-size form).
template <int MC, int NC>
SVO_HD void svd_impl(const double* a, int m_rt, int n_rt, double* s, double* U, double* Vt) {
    const int m = MC > 0 ? MC : m_rt, n = NC > 0 ? NC : n_rt;
    double W[MC > 0 ? MC * NC : 144], V[NC > 0 ? NC * NC : 144];
    for (int i = 0; i < m * n; i++) W[i] = a[i];
    for (int i = 0; i < n * n; i++) V[i] = 0;
    for (int i = 0; i < n; i++) V[i * n + i] = 1;
    for (int sweep = 0; sweep < 60; sweep++) {
        bool rotated = false;
        for (int p = 0; p < n - 1; p++)
            for (int q = p + 1; q < n; q++) {
                double al = 0, be = 0, ga = 0;
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
                for (int k = 0; k < m; k++) {
                    const double x = W[k * n + p], y = W[k * n + q];
                    W[k * n + p] = c * x - sn * y;
                    W[k * n + q] = sn * x + c * y;
                }
                for (int k = 0; k < n; k++) {
                    const double x = V[k * n + p], y = V[k * n + q];
                    V[k * n + p] = c * x - sn * y;
                    V[k * n + q] = sn * x + c * y;
                }
            }
        if (!rotated) break;
    }
    double nrm[NC > 0 ? NC : 12];
    int order[NC > 0 ? NC : 12];
    for (int j = 0; j < n; j++) {
        double acc = 0;
        for (int k = 0; k < m; k++) acc += W[k * n + j] * W[k * n + j];
        nrm[j] = sqrt(acc);
        order[j] = j;
    }
    for (int i = 1; i < n; i++) {
        int v = order[i], j = i - 1;
        while (j >= 0 && nrm[order[j]] < nrm[v]) {
            order[j + 1] = order[j];
            j--;
        }
        order[j + 1] = v;
    }
    for (int i = 0; i < n; i++) {
        const int c = order[i];
        s[i] = nrm[c];
        for (int k = 0; k < n; k++) Vt[i * n + k] = V[k * n + c];
        if (U)
            for (int k = 0; k < m; k++) U[k * n + i] = nrm[c] > 0 ? W[k * n + c] / nrm[c] : 0;
    }
}
// svd_impl<3, 3> of NS independent matrices in lock step: each matrix's sweeps,
// rotations and skips exactly as svd_impl (a matrix whose sweep rotated nothing
// stops; the others go on), interleaved so that the host core overlaps the NS
// dependency chains. U may be null.
template <int NS>
SVO_HD void svd3_n(const double (*a)[9], double (*s)[3], double (*U)[9], double (*Vt)[9]) {
    constexpr int m = 3, n = 3;
    double W[NS][9], V[NS][9];
    bool done[NS];
    for (int q = 0; q < NS; q++) {
        for (int i = 0; i < 9; i++) W[q][i] = a[q][i];
        for (int i = 0; i < 9; i++) V[q][i] = 0;
        for (int i = 0; i < n; i++) V[q][i * n + i] = 1;
        done[q] = false;
    }
    for (int sweep = 0; sweep < 60; sweep++) {
        bool rotated[NS], any = false;
        for (int q = 0; q < NS; q++) rotated[q] = false;
        for (int p = 0; p < n - 1; p++)
            for (int r = p + 1; r < n; r++)
                for (int q = 0; q < NS; q++) {
                    if (done[q]) continue;
                    double al = 0, be = 0, ga = 0;
                    for (int k = 0; k < m; k++) {
                        al += W[q][k * n + p] * W[q][k * n + p];
                        be += W[q][k * n + r] * W[q][k * n + r];
                        ga += W[q][k * n + p] * W[q][k * n + r];
                    }
                    if (ga == 0 || fabs(ga) <= 1e-15 * sqrt(al * be)) continue;
                    rotated[q] = true;
                    const double z = (be - al) / (2 * ga);
                    const double t = (z >= 0 ? 1.0 : -1.0) / (fabs(z) + sqrt(1 + z * z));
                    const double c = 1 / sqrt(1 + t * t), sn = c * t;
                    for (int k = 0; k < m; k++) {
                        const double x = W[q][k * n + p], y = W[q][k * n + r];
                        W[q][k * n + p] = c * x - sn * y;
                        W[q][k * n + r] = sn * x + c * y;
                    }
                    for (int k = 0; k < n; k++) {
                        const double x = V[q][k * n + p], y = V[q][k * n + r];
                        V[q][k * n + p] = c * x - sn * y;
                        V[q][k * n + r] = sn * x + c * y;
                    }
                }
        for (int q = 0; q < NS; q++) {
            if (!rotated[q]) done[q] = true;
            any = any || !done[q];
        }
        if (!any) break;
    }
    for (int q = 0; q < NS; q++) {
        double nrm[3];
        int order[3];
        for (int j = 0; j < n; j++) {
            double acc = 0;
            for (int k = 0; k < m; k++) acc += W[q][k * n + j] * W[q][k * n + j];
            nrm[j] = sqrt(acc);
            order[j] = j;
        }
        for (int i = 1; i < n; i++) {
            int v = order[i], j = i - 1;
            while (j >= 0 && nrm[order[j]] < nrm[v]) {
                order[j + 1] = order[j];
                j--;
            }
            order[j + 1] = v;
        }
        for (int i = 0; i < n; i++) {
            const int c = order[i];
            s[q][i] = nrm[c];
            for (int k = 0; k < n; k++) Vt[q][i * n + k] = V[q][k * n + c];
            if (U)
                for (int k = 0; k < m; k++) U[q][k * n + i] = nrm[c] > 0 ? W[q][k * n + c] / nrm[c] : 0;
        }
    }
}

SVO_HD void svd(const double* a, int m, int n, double* s, double* U, double* Vt) {
    if (m == 3 && n == 3) return svd_impl<3, 3>(a, 3, 3, s, U, Vt);  // Procrustes, pinv3, rotations
    svd_impl<0, 0>(a, m, n, s, U, Vt);
}

// Least squares x = pinv(A) b (m x n, m <= 12, n <= 12), as cv::solve(DECOMP_SVD).
SVO_HD void lstsq(const double* A, int m, int n, const double* b, double* x) {
    double s[12], U[144], Vt[144];
    svd(A, m, n, s, U, Vt);
    const double tol = s[0] * (m > n ? m : n) * 2.220446049250313e-16;
    for (int j = 0; j < n; j++) x[j] = 0;
    for (int i = 0; i < n; i++) {
        if (!(s[i] > tol)) continue;
        double ub = 0;
        for (int k = 0; k < m; k++) ub += U[k * n + i] * b[k];
        ub /= s[i];
        for (int j = 0; j < n; j++) x[j] += ub * Vt[i * n + j];
    }
}

// Pseudo-inverse of a 3x3 matrix.
SVO_HD void pinv3(const double* A, double* Ai) {
    double s[3], U[9], Vt[9];
    svd(A, 3, 3, s, U, Vt);
    const double tol = s[0] * 3 * 2.220446049250313e-16;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double acc = 0;
            for (int k = 0; k < 3; k++)
                if (s[k] > tol) acc += Vt[k * 3 + i] * U[j * 3 + k] / s[k];
            Ai[i * 3 + j] = acc;
        }
}

// Nearest rotation (polar factor with det = +1) of a 3x3 matrix.
SVO_HD void nearest_rotation(const double* M, double* R) {
    double s[3], U[9], Vt[9];
    svd(M, 3, 3, s, U, Vt);
    double sg = 1.0;
    for (int pass = 0; pass < 2; pass++) {
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++)
                R[i * 3 + j] = U[i * 3 + 0] * Vt[0 * 3 + j] + U[i * 3 + 1] * Vt[1 * 3 + j] + sg * U[i * 3 + 2] * Vt[2 * 3 + j];
        const double det = R[0] * (R[4] * R[8] - R[5] * R[7]) - R[1] * (R[3] * R[8] - R[5] * R[6]) +
                           R[2] * (R[3] * R[7] - R[4] * R[6]);
        if (det > 0) break;
        sg = -1.0;
    }
}

// Rodrigues vector -> matrix (cv::Rodrigues formula order).
SVO_HD void rodrigues(const double* rv, double* R) {
    double rx = rv[0], ry = rv[1], rz = rv[2];
    const double th = sqrt(rx * rx + ry * ry + rz * rz);
    if (th < 2.220446049250313e-16) {
        for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0) ? 1.0 : 0.0;
        return;
    }
    const double c = cos(th), s = sin(th), c1 = 1. - c, it = th ? 1. / th : 0.;
    rx *= it;
    ry *= it;
    rz *= it;
    const double rrt[9] = {rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz};
    const double rxm[9] = {0, -rz, ry, rz, 0, -rx, -ry, rx, 0};
    for (int i = 0; i < 9; i++) R[i] = (c * ((i % 4 == 0) ? 1.0 : 0.0) + c1 * rrt[i]) + s * rxm[i];
}

// Rodrigues matrix -> vector (re-orthonormalised through the SVD first).
SVO_HD void rodrigues_inv(const double* Rin, double* rv) {
    double R[9];
    nearest_rotation(Rin, R);
    double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
    const double s = sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
    double c = (R[0] + R[4] + R[8] - 1) * 0.5;
    c = c > 1. ? 1. : c < -1. ? -1. : c;
    double th = acos(c);
    if (s < 1e-5) {
        if (c > 0) {
            rx = ry = rz = 0;
        } else {
            double t = (R[0] + 1) * 0.5;
            rx = sqrt(t > 0 ? t : 0.);
            t = (R[4] + 1) * 0.5;
            ry = sqrt(t > 0 ? t : 0.) * (R[1] < 0 ? -1. : 1.);
            t = (R[8] + 1) * 0.5;
            rz = sqrt(t > 0 ? t : 0.) * (R[2] < 0 ? -1. : 1.);
            if (fabs(rx) < fabs(ry) && fabs(rx) < fabs(rz) && (R[5] > 0) != (ry * rz > 0)) rz = -rz;
            th /= sqrt(rx * rx + ry * ry + rz * rz);
            rx *= th;
            ry *= th;
            rz *= th;
        }
    } else {
        double vth = 1 / (2 * s);
        vth *= th;
        rx *= vth;
        ry *= vth;
        rz *= vth;
    }
    rv[0] = rx;
    rv[1] = ry;
    rv[2] = rz;
}

// OpenCV 4.x core/src/lapack.cpp restated: the SVD routines calib3d's EPnP calls
// (cvSVD, cvInvert(CV_SVD), cvSolve(CV_SVD)) and cv::Rodrigues uses, operation by
// operation, so that the minimal solver's results do not depend on which Jacobi
// variant picks a basis of a degenerate singular subspace (the 5-point M^T M has
// a two-dimensional null space). The oracle restates the same functions
// (oracle/cvsvd.c); tests/test_epnp_cpu.py holds the two EPnP solvers bit for bit.
namespace cv {

// lapack.cpp's hypot: the larger operand times sqrt(1 + ratio^2)
SVO_HD double hypot_cv(double a, double b) {
    a = fabs(a);
    b = fabs(b);
    if (a > b) {
        b /= a;
        return a * sqrt(1 + b * b);
    }
    if (b > 0) {
        a /= b;
        return b * sqrt(1 + a * a);
    }
    return 0;
}

// JacobiSVDImpl_<double>(At, ., W, Vt, ., M, N, n1 = N, DBL_MIN, 10 DBL_EPSILON)
// with a right-singular-vector buffer present (compute_uv, as every caller here):
// At (N rows of M) becomes the normalised left singular vectors, W the singular
// values (descending). WANT_V = false skips the rotations of Vt -- its values
// never reach At or W -- while keeping every At-side step of the Vt-present path
// (row swaps in the sort, the normalisation).
template <int M, int N, bool WANT_V>
SVO_HD void jacobi_tail(double* At, double* Wout, double* Vt);
template <int M, int N, bool WANT_V>
SVO_HD void jacobi_svd(double* At, double* Wout, double* Vt) {
    const double eps = 2.220446049250313e-16 * 10;
    double W[N];
    constexpr int max_iter = M > 30 ? M : 30;
    for (int i = 0; i < N; i++) {
        double sd = 0;
        for (int k = 0; k < M; k++) sd += At[i * M + k] * At[i * M + k];
        W[i] = sd;
        if (WANT_V) {
            for (int k = 0; k < N; k++) Vt[i * N + k] = 0;
            Vt[i * N + i] = 1;
        }
    }
    for (int iter = 0; iter < max_iter; iter++) {
        bool changed = false;
        for (int i = 0; i < N - 1; i++)
            for (int j = i + 1; j < N; j++) {
                double* Ai = At + i * M;
                double* Aj = At + j * M;
                double a = W[i], p = 0, b = W[j];
                for (int k = 0; k < M; k++) p += Ai[k] * Aj[k];
                if (fabs(p) <= eps * sqrt(a * b)) continue;
                p *= 2;
                const double beta = a - b, gamma = hypot_cv(p, beta);
                double c, s;
                if (beta < 0) {
                    const double delta = (gamma - beta) * 0.5;
                    s = sqrt(delta / gamma);
                    c = p / (gamma * s * 2);
                } else {
                    c = sqrt((gamma + beta) / (gamma * 2));
                    s = p / (gamma * c * 2);
                }
                a = b = 0;
                for (int k = 0; k < M; k++) {
                    const double t0 = c * Ai[k] + s * Aj[k];
                    const double t1 = -s * Ai[k] + c * Aj[k];
                    Ai[k] = t0;
                    Aj[k] = t1;
                    a += t0 * t0;
                    b += t1 * t1;
                }
                W[i] = a;
                W[j] = b;
                changed = true;
                if (WANT_V) {
                    double* Vi = Vt + i * N;
                    double* Vj = Vt + j * N;
                    for (int k = 0; k < N; k++) {
                        const double t0 = c * Vi[k] + s * Vj[k];
                        const double t1 = -s * Vi[k] + c * Vj[k];
                        Vi[k] = t0;
                        Vj[k] = t1;
                    }
                }
            }
        if (!changed) break;
    }
    jacobi_tail<M, N, WANT_V>(At, Wout, Vt);
}

// jacobi_svd's tail after the sweeps: singular values, the selection sort (rows
// of At / Vt swapped), the normalisation of the left vectors (a zero singular
// value gets a random unit vector orthogonal to the previous ones)
template <int M, int N, bool WANT_V>
SVO_HD void jacobi_tail(double* At, double* Wout, double* Vt) {
    const double minval = 2.2250738585072014e-308, eps = 2.220446049250313e-16 * 10;
    double W[N];
    for (int i = 0; i < N; i++) {
        double sd = 0;
        for (int k = 0; k < M; k++) sd += At[i * M + k] * At[i * M + k];
        W[i] = sqrt(sd);
    }
    for (int i = 0; i < N - 1; i++) {
        int j = i;
        for (int k = i + 1; k < N; k++)
            if (W[j] < W[k]) j = k;
        if (i != j) {
            const double tw = W[i];
            W[i] = W[j];
            W[j] = tw;
            for (int k = 0; k < M; k++) {
                const double t = At[i * M + k];
                At[i * M + k] = At[j * M + k];
                At[j * M + k] = t;
            }
            if (WANT_V)
                for (int k = 0; k < N; k++) {
                    const double t = Vt[i * N + k];
                    Vt[i * N + k] = Vt[j * N + k];
                    Vt[j * N + k] = t;
                }
        }
    }
    for (int i = 0; i < N; i++) Wout[i] = W[i];
    unsigned long long rng = 0x12345678ull;
    for (int i = 0; i < N; i++) {
        double sd = W[i];
        for (int ii = 0; ii < 100 && sd <= minval; ii++) {
            // a zero singular value: a random unit vector orthogonal to the
            // previous left singular vectors (cv::RNG(0x12345678))
            const double val0 = 1. / M;
            for (int k = 0; k < M; k++) {
                rng = (unsigned long long)(unsigned)rng * 4164903690u + (unsigned)(rng >> 32);
                At[i * M + k] = ((unsigned)rng & 256) != 0 ? val0 : -val0;
            }
            for (int it = 0; it < 2; it++)
                for (int j = 0; j < i; j++) {
                    sd = 0;
                    for (int k = 0; k < M; k++) sd += At[i * M + k] * At[j * M + k];
                    double asum = 0;
                    for (int k = 0; k < M; k++) {
                        const double t = At[i * M + k] - sd * At[j * M + k];
                        At[i * M + k] = t;
                        asum += fabs(t);
                    }
                    asum = asum > eps * 100 ? 1 / asum : 0;
                    for (int k = 0; k < M; k++) At[i * M + k] *= asum;
                }
            sd = 0;
            for (int k = 0; k < M; k++) sd += At[i * M + k] * At[i * M + k];
            sd = sqrt(sd);
        }
        const double s = sd > minval ? 1 / sd : 0.;
        for (int k = 0; k < M; k++) At[i * M + k] *= s;
    }
}

// jacobi_svd<M, N, false> of NS independent matrices interleaved pair by pair:
// every matrix's sweeps, skips, rotations and stop exactly as jacobi_svd (a
// matrix whose sweep rotated nothing stops; the others go on), so each result is
// bit-identical to its own jacobi_svd -- the interleaving only lets the host core
// overlap the NS dependency chains of the sequential dot products and the
// rotation coefficients (one problem's Jacobi is a single serial chain).
template <int M, int N, int NS>
SVO_HD void jacobi_svd_n(double (*At)[N * M], double (*Wout)[N]) {
    const double minval = 2.2250738585072014e-308, eps = 2.220446049250313e-16 * 10;
    double W[NS][N];
    bool live[NS];
    constexpr int max_iter = M > 30 ? M : 30;
    for (int q = 0; q < NS; q++) {
        live[q] = true;
        for (int i = 0; i < N; i++) {
            double sd = 0;
            for (int k = 0; k < M; k++) sd += At[q][i * M + k] * At[q][i * M + k];
            W[q][i] = sd;
        }
    }
    for (int iter = 0; iter < max_iter; iter++) {
        bool changed[NS], any = false;
        for (int q = 0; q < NS; q++) changed[q] = false;
        for (int i = 0; i < N - 1; i++)
            for (int j = i + 1; j < N; j++) {
                double p[NS];
                for (int q = 0; q < NS; q++) {
                    p[q] = 0;
                    if (!live[q]) continue;
                    const double* Ai = At[q] + i * M;
                    const double* Aj = At[q] + j * M;
                    for (int k = 0; k < M; k++) p[q] += Ai[k] * Aj[k];
                }
                for (int q = 0; q < NS; q++) {
                    if (!live[q]) continue;
                    double a = W[q][i], b = W[q][j], pq = p[q];
                    if (fabs(pq) <= eps * sqrt(a * b)) continue;
                    pq *= 2;
                    const double beta = a - b, gamma = hypot_cv(pq, beta);
                    double c, s;
                    if (beta < 0) {
                        const double delta = (gamma - beta) * 0.5;
                        s = sqrt(delta / gamma);
                        c = pq / (gamma * s * 2);
                    } else {
                        c = sqrt((gamma + beta) / (gamma * 2));
                        s = pq / (gamma * c * 2);
                    }
                    double* Ai = At[q] + i * M;
                    double* Aj = At[q] + j * M;
                    a = b = 0;
                    for (int k = 0; k < M; k++) {
                        const double t0 = c * Ai[k] + s * Aj[k];
                        const double t1 = -s * Ai[k] + c * Aj[k];
                        Ai[k] = t0;
                        Aj[k] = t1;
                        a += t0 * t0;
                        b += t1 * t1;
                    }
                    W[q][i] = a;
                    W[q][j] = b;
                    changed[q] = true;
                }
            }
        for (int q = 0; q < NS; q++) {
            if (!changed[q]) live[q] = false;
            any = any || live[q];
        }
        if (!any) break;
    }
    for (int q = 0; q < NS; q++) {
        double* A = At[q];
        double* Wq = W[q];
        for (int i = 0; i < N; i++) {
            double sd = 0;
            for (int k = 0; k < M; k++) sd += A[i * M + k] * A[i * M + k];
            Wq[i] = sqrt(sd);
        }
        for (int i = 0; i < N - 1; i++) {
            int j = i;
            for (int k = i + 1; k < N; k++)
                if (Wq[j] < Wq[k]) j = k;
            if (i != j) {
                const double tw = Wq[i];
                Wq[i] = Wq[j];
                Wq[j] = tw;
                for (int k = 0; k < M; k++) {
                    const double t = A[i * M + k];
                    A[i * M + k] = A[j * M + k];
                    A[j * M + k] = t;
                }
            }
        }
        for (int i = 0; i < N; i++) Wout[q][i] = Wq[i];
        unsigned long long rng = 0x12345678ull;
        for (int i = 0; i < N; i++) {
            double sd = Wq[i];
            for (int ii = 0; ii < 100 && sd <= minval; ii++) {
                const double val0 = 1. / M;
                for (int k = 0; k < M; k++) {
                    rng = (unsigned long long)(unsigned)rng * 4164903690u + (unsigned)(rng >> 32);
                    A[i * M + k] = ((unsigned)rng & 256) != 0 ? val0 : -val0;
                }
                for (int it = 0; it < 2; it++)
                    for (int j = 0; j < i; j++) {
                        sd = 0;
                        for (int k = 0; k < M; k++) sd += A[i * M + k] * A[j * M + k];
                        double asum = 0;
                        for (int k = 0; k < M; k++) {
                            const double t = A[i * M + k] - sd * A[j * M + k];
                            A[i * M + k] = t;
                            asum += fabs(t);
                        }
                        asum = asum > eps * 100 ? 1 / asum : 0;
                        for (int k = 0; k < M; k++) A[i * M + k] *= asum;
                    }
                sd = 0;
                for (int k = 0; k < M; k++) sd += A[i * M + k] * A[i * M + k];
                sd = sqrt(sd);
            }
            const double s = sd > minval ? 1 / sd : 0.;
            for (int k = 0; k < M; k++) A[i * M + k] *= s;
        }
    }
}

// cvMulTransposed(src, dst, 1): dst = src^T src (ROWS x COLS src), each upper
// element summed over the rows in order, the lower triangle mirrored
template <int COLS>
SVO_HD void mul_transposed(const double* src, int rows, double* dst) {
    for (int i = 0; i < COLS; i++)
        for (int j = i; j < COLS; j++) {
            double s = 0;
            for (int k = 0; k < rows; k++) s += src[k * COLS + i] * src[k * COLS + j];
            dst[i * COLS + j] = s;
        }
    for (int i = 0; i < COLS; i++)
        for (int j = 0; j < i; j++) dst[i * COLS + j] = dst[j * COLS + i];
}

// cvSVD(A, W, Ut, 0, CV_SVD_U_T) of a square N x N A: rows of ut = left singular
// vectors
template <int N>
SVO_HD void svd_ut(const double* A, double* w, double* ut) {
    for (int i = 0; i < N; i++)
        for (int k = 0; k < N; k++) ut[i * N + k] = A[k * N + i];
    jacobi_svd<N, N, false>(ut, w, nullptr);
}

// SVD::compute of a square N x N A: u (columns = left vectors), vt (rows)
template <int N>
SVO_HD void svd(const double* A, double* w, double* u, double* vt) {
    double At[N * N];
    for (int i = 0; i < N; i++)
        for (int k = 0; k < N; k++) At[i * N + k] = A[k * N + i];
    jacobi_svd<N, N, true>(At, w, vt);
    for (int k = 0; k < N; k++)
        for (int i = 0; i < N; i++) u[k * N + i] = At[i * N + k];
}

// cv::solve(A, b, x, DECOMP_SVD), one right-hand side, A M x N (M >= N)
template <int M, int N>
SVO_HD void solve_svd(const double* A, const double* b, double* x) {
    double At[N * M], V[N * N], w[N];
    for (int i = 0; i < N; i++)
        for (int k = 0; k < M; k++) At[i * M + k] = A[k * N + i];
    jacobi_svd<M, N, true>(At, w, V);
    double threshold = 0;
    for (int j = 0; j < N; j++) x[j] = 0;
    for (int i = 0; i < N; i++) threshold += w[i];
    threshold *= 2.220446049250313e-16 * 2;
    for (int i = 0; i < N; i++) {
        double wi = w[i];
        if (fabs(wi) <= threshold) continue;
        wi = 1 / wi;
        double s = 0;
        for (int j = 0; j < M; j++) s += At[i * M + j] * b[j];
        s *= wi;
        for (int j = 0; j < N; j++) x[j] = x[j] + s * V[i * N + j];
    }
}

// cv::invert(A, Ai, DECOMP_SVD) of an N x N A (SVD::backSubst with the identity)
template <int N>
SVO_HD void invert_svd(const double* A, double* Ai) {
    double u[N * N], vt[N * N], w[N], buf[N];
    svd<N>(A, w, u, vt);
    double threshold = 0;
    for (int i = 0; i < N * N; i++) Ai[i] = 0;
    for (int i = 0; i < N; i++) threshold += w[i];
    threshold *= 2.220446049250313e-16 * 2;
    for (int i = 0; i < N; i++) {
        double wi = w[i];
        if (fabs(wi) <= threshold) continue;
        wi = 1 / wi;
        for (int j = 0; j < N; j++) buf[j] = u[j * N + i] * wi;
        for (int r = 0; r < N; r++) {
            const double sv = vt[i * N + r];
            for (int j = 0; j < N; j++) Ai[r * N + j] = Ai[r * N + j] + sv * buf[j];
        }
    }
}

// cv::Rodrigues matrix -> vector: SVD::compute(R, W, U, Vt), R = U * Vt (Matx
// product), then the axis-angle extraction (same as la::rodrigues_inv's)
SVO_HD void rodrigues_inv(const double* Rin, double* rv) {
    double w[3], u[9], vt[9], R[9];
    svd<3>(Rin, w, u, vt);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double acc = 0;
            for (int k = 0; k < 3; k++) acc += u[i * 3 + k] * vt[k * 3 + j];
            R[i * 3 + j] = acc;
        }
    double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
    const double s = sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
    double c = (R[0] + R[4] + R[8] - 1) * 0.5;
    c = c > 1. ? 1. : c < -1. ? -1. : c;
    double th = acos(c);
    if (s < 1e-5) {
        if (c > 0) {
            rx = ry = rz = 0;
        } else {
            double t = (R[0] + 1) * 0.5;
            rx = sqrt(t > 0 ? t : 0.);
            t = (R[4] + 1) * 0.5;
            ry = sqrt(t > 0 ? t : 0.) * (R[1] < 0 ? -1. : 1.);
            t = (R[8] + 1) * 0.5;
            rz = sqrt(t > 0 ? t : 0.) * (R[2] < 0 ? -1. : 1.);
            if (fabs(rx) < fabs(ry) && fabs(rx) < fabs(rz) && (R[5] > 0) != (ry * rz > 0)) rz = -rz;
            th /= sqrt(rx * rx + ry * ry + rz * rz);
            rx *= th;
            ry *= th;
            rz *= th;
        }
    } else {
        double vth = 1 / (2 * s);
        vth *= th;
        rx *= vth;
        ry *= vth;
        rz *= vth;
    }
    rv[0] = rx;
    rv[1] = ry;
    rv[2] = rz;
}

}  // namespace cv

}  // namespace la
}  // namespace svo
