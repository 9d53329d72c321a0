/* Oracle internals (TEST INFRASTRUCTURE ONLY -- see svo_oracle.h). */
#ifndef SVO_ORACLE_INTERNAL_H
#define SVO_ORACLE_INTERNAL_H
#include <stdint.h>

int svo_oracle_reflect101(int p, int len);

/* cvRound / cvFloor on float, as OpenCV defines them on x86 (round-half-even). */
static inline int ora_round_f(float v) { return (int)__builtin_rintf(v); }
static inline int ora_round_d(double v) { return (int)__builtin_rint(v); }
static inline int ora_floor_f(float v) { int i = (int)v; return i - (i > v); }

/* Small dense linear algebra (double), oracle-owned. */
/* Symmetric eigen-decomposition by cyclic Jacobi: A (n x n, row-major) is
 * destroyed; eigenvalues descending in w, eigenvectors as ROWS of vt. */
void ora_sym_eig(double* A, int n, double* w, double* vt);
/* Thin SVD of a (m x n, row-major, m >= n or any) via one-sided Jacobi:
 * a = U diag(w) V^T; w descending (length n), u m x n, vt n x n rows. */
void ora_svd(const double* a, int m, int n, double* w, double* u, double* vt);
/* Least-squares solve via SVD pseudo-inverse (cv::solve(..., DECOMP_SVD)). */
void ora_svd_solve(const double* A, int m, int n, const double* b, double* x);

/* OpenCV's lapack.cpp restated (cvsvd.c): the EPnP solver's SVDs. n <= 16. */
void ora_cv_jacobi_svd(double* At, int m, int n, int n1, double* W, double* Vt);
void ora_cv_svd(const double* A, int m, int n, double* w, double* u, double* vt);
void ora_cv_svd_ut(const double* A, int n, double* w, double* ut);
void ora_cv_solve_svd(const double* A, int m, int n, const double* b, double* x);
void ora_cv_invert_svd(const double* A, int n, double* Ai);
void ora_mul_transposed(const double* src, int rows, int cols, double* dst);

#endif
