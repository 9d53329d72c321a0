/*
 * Oracle (TEST INFRASTRUCTURE ONLY -- see svo_oracle.h).
 * Small dense double-precision linear algebra used by the EPnP / PnP oracle
 * (stands in for OpenCV's cvSVD / cvSolve(CV_SVD) / cvInvert(CV_SVD), which
 * are Jacobi SVDs in core/src/lapack.cpp). Results agree with OpenCV's up to
 * floating-point rounding, not bit for bit.
 */
#include "oracle_internal.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

void ora_sym_eig(double* A, int n, double* w, double* vt)
{
    /* V = I; rotate A to diagonal; eigenvectors are columns of V */
    double* V = (double*)malloc(sizeof(double) * n * n);
    for (int i = 0; i < n * n; i++) V[i] = 0;
    for (int i = 0; i < n; i++) V[i * n + i] = 1;
    for (int sweep = 0; sweep < 100; sweep++) {
        double off = 0, diag = 0;
        for (int p = 0; p < n; p++)
            for (int q = 0; q < n; q++) {
                if (p != q) off += A[p * n + q] * A[p * n + q];
                else diag += A[p * n + q] * A[p * n + q];
            }
        if (off <= 1e-30 * diag || off == 0) break;
        for (int p = 0; p < n - 1; p++)
            for (int q = p + 1; q < n; q++) {
                double apq = A[p * n + q];
                if (apq == 0) continue;
                double app = A[p * n + p], aqq = A[q * n + q];
                double theta = (aqq - app) / (2 * apq);
                double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1));
                double c = 1 / sqrt(t * t + 1), s = t * c;
                for (int k = 0; k < n; k++) {
                    double akp = A[k * n + p], akq = A[k * n + q];
                    A[k * n + p] = c * akp - s * akq;
                    A[k * n + q] = s * akp + c * akq;
                }
                for (int k = 0; k < n; k++) {
                    double apk = A[p * n + k], aqk = A[q * n + k];
                    A[p * n + k] = c * apk - s * aqk;
                    A[q * n + k] = s * apk + c * aqk;
                }
                for (int k = 0; k < n; k++) {
                    double vkp = V[k * n + p], vkq = V[k * n + q];
                    V[k * n + p] = c * vkp - s * vkq;
                    V[k * n + q] = s * vkp + c * vkq;
                }
            }
    }
    /* sort descending */
    int* idx = (int*)malloc(sizeof(int) * n);
    for (int i = 0; i < n; i++) idx[i] = i;
    for (int i = 0; i < n; i++)
        for (int j = i + 1; j < n; j++)
            if (A[idx[j] * n + idx[j]] > A[idx[i] * n + idx[i]]) { int t = idx[i]; idx[i] = idx[j]; idx[j] = t; }
    for (int i = 0; i < n; i++) {
        w[i] = A[idx[i] * n + idx[i]];
        for (int k = 0; k < n; k++) vt[i * n + k] = V[k * n + idx[i]];
    }
    free(idx);
    free(V);
}

void ora_svd(const double* a, int m, int n, double* w, double* u, double* vt)
{
    /* one-sided Jacobi on columns of U (m x n) */
    double* U = (double*)malloc(sizeof(double) * m * n);
    double* V = (double*)malloc(sizeof(double) * n * n);
    memcpy(U, a, sizeof(double) * m * n);
    for (int i = 0; i < n * n; i++) V[i] = 0;
    for (int i = 0; i < n; i++) V[i * n + i] = 1;
    for (int sweep = 0; sweep < 100; sweep++) {
        int changed = 0;
        for (int p = 0; p < n - 1; p++)
            for (int q = p + 1; q < n; q++) {
                double alpha = 0, beta = 0, gamma = 0;
                for (int k = 0; k < m; k++) {
                    alpha += U[k * n + p] * U[k * n + p];
                    beta += U[k * n + q] * U[k * n + q];
                    gamma += U[k * n + p] * U[k * n + q];
                }
                if (fabs(gamma) <= 1e-15 * sqrt(alpha * beta) || gamma == 0) continue;
                changed = 1;
                double zeta = (beta - alpha) / (2 * gamma);
                double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1 + zeta * zeta));
                double c = 1 / sqrt(1 + t * t), s = c * t;
                for (int k = 0; k < m; k++) {
                    double up = U[k * n + p], uq = U[k * n + q];
                    U[k * n + p] = c * up - s * uq;
                    U[k * n + q] = s * up + c * uq;
                }
                for (int k = 0; k < n; k++) {
                    double vp = V[k * n + p], vq = V[k * n + q];
                    V[k * n + p] = c * vp - s * vq;
                    V[k * n + q] = s * vp + c * vq;
                }
            }
        if (!changed) break;
    }
    double* sv = (double*)malloc(sizeof(double) * n);
    int* idx = (int*)malloc(sizeof(int) * n);
    for (int j = 0; j < n; j++) {
        double s = 0;
        for (int k = 0; k < m; k++) s += U[k * n + j] * U[k * n + j];
        sv[j] = sqrt(s);
        idx[j] = j;
    }
    for (int i = 0; i < n; i++)
        for (int j = i + 1; j < n; j++)
            if (sv[idx[j]] > sv[idx[i]]) { int t = idx[i]; idx[i] = idx[j]; idx[j] = t; }
    for (int i = 0; i < n; i++) {
        int c = idx[i];
        w[i] = sv[c];
        for (int k = 0; k < n; k++) vt[i * n + k] = V[k * n + c];
        if (u)
            for (int k = 0; k < m; k++) u[k * n + i] = sv[c] > 0 ? U[k * n + c] / sv[c] : 0;
    }
    free(sv);
    free(idx);
    free(U);
    free(V);
}

void ora_svd_solve(const double* A, int m, int n, const double* b, double* x)
{
    double* w = (double*)malloc(sizeof(double) * n);
    double* u = (double*)malloc(sizeof(double) * m * n);
    double* vt = (double*)malloc(sizeof(double) * n * n);
    ora_svd(A, m, n, w, u, vt);
    double tol = (w[0] > 0 ? w[0] : 0) * (m > n ? m : n) * 2.2204460492503131e-16;
    for (int j = 0; j < n; j++) x[j] = 0;
    for (int i = 0; i < n; i++) {
        if (w[i] <= tol) continue;
        double s = 0;
        for (int k = 0; k < m; k++) s += u[k * n + i] * b[k];
        s /= w[i];
        for (int j = 0; j < n; j++) x[j] += s * vt[i * n + j];
    }
    free(w);
    free(u);
    free(vt);
}
