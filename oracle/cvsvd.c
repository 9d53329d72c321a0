/*
 * Oracle (TEST INFRASTRUCTURE ONLY -- see svo_oracle.h; parity unpinned).
 *
 * OpenCV 4.x core/src/lapack.cpp restated for the EPnP minimal solver
 * (calib3d/src/epnp.cpp calls cvSVD, cvInvert(CV_SVD) and cvSolve(CV_SVD)):
 *   JacobiSVDImpl_<double>  one-sided Jacobi on the rows of At (= A^T), pairs in
 *                           cyclic order, eps = 10 DBL_EPSILON, at most max(m, 30)
 *                           sweeps, the rotation from lapack.cpp's own hypot,
 *                           selection sort by singular value, rows normalised
 *                           (a zero singular value gets a random unit vector
 *                           orthogonal to the previous ones, RNG 0x12345678);
 *   _SVDcompute             A (m x n, m >= n) -> w, u (m x n, columns), vt (n x n);
 *   SVBkSbImpl_             back substitution x = V diag(1/w) U^T b with the
 *                           threshold 2 DBL_EPSILON * sum(w) (cv::solve /
 *                           SVD::backSubst, nb = 1, and cv::invert's identity rhs).
 * The product restates the same functions (svo_amd/csrc/linalg.hpp, namespace
 * la::cv) so that both EPnP solvers pick the same basis of the 5-point M^T M's
 * two-dimensional null space: tests/test_epnp_cpu.py holds them bit for bit.
 */
#include "oracle_internal.h"

#include <float.h>
#include <math.h>
#include <string.h>

/* lapack.cpp's hypot (not libm's): a sqrt(1 + (b/a)^2) with the larger operand
 * outside */
static double cv_hypot(double a, double b)
{
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

/* cv::RNG::next (the MWC step of operations.hpp) */
static unsigned cv_rng_next(unsigned long long* s)
{
    *s = (unsigned long long)(unsigned)(*s) * 4164903690U + (unsigned)(*s >> 32);
    return (unsigned)*s;
}

/* JacobiSVDImpl_<double>(At, astep, W, Vt, vstep, m, n, n1, DBL_MIN, 10 DBL_EPSILON):
 * At: n rows of m elements (row stride m), overwritten by the left singular
 * vectors (first n1 rows normalised); W: n singular values, descending; Vt:
 * n x n right singular vectors (rows), or NULL. */
void ora_cv_jacobi_svd(double* At, int m, int n, int n1, double* Wout, double* Vt)
{
    const double minval = DBL_MIN, eps = DBL_EPSILON * 10;
    double W[16];
    int max_iter = m > 30 ? m : 30;
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int k = 0; k < m; k++) {
            double t = At[i * m + k];
            sd += t * t;
        }
        W[i] = sd;
        if (Vt) {
            for (int k = 0; k < n; k++) Vt[i * n + k] = 0;
            Vt[i * n + i] = 1;
        }
    }
    for (int iter = 0; iter < max_iter; iter++) {
        int changed = 0;
        for (int i = 0; i < n - 1; i++)
            for (int j = i + 1; j < n; j++) {
                double *Ai = At + i * m, *Aj = At + j * m;
                double a = W[i], p = 0, b = W[j];
                for (int k = 0; k < m; k++) p += Ai[k] * Aj[k];
                if (fabs(p) <= eps * sqrt(a * b)) continue;
                p *= 2;
                double beta = a - b, gamma = cv_hypot(p, beta), c, s;
                if (beta < 0) {
                    double delta = (gamma - beta) * 0.5;
                    s = sqrt(delta / gamma);
                    c = p / (gamma * s * 2);
                } else {
                    c = sqrt((gamma + beta) / (gamma * 2));
                    s = p / (gamma * c * 2);
                }
                a = b = 0;
                for (int k = 0; k < m; k++) {
                    double t0 = c * Ai[k] + s * Aj[k];
                    double t1 = -s * Ai[k] + c * Aj[k];
                    Ai[k] = t0;
                    Aj[k] = t1;
                    a += t0 * t0;
                    b += t1 * t1;
                }
                W[i] = a;
                W[j] = b;
                changed = 1;
                if (Vt) {
                    double *Vi = Vt + i * n, *Vj = Vt + j * n;
                    for (int k = 0; k < n; k++) {
                        double t0 = c * Vi[k] + s * Vj[k];
                        double t1 = -s * Vi[k] + c * Vj[k];
                        Vi[k] = t0;
                        Vj[k] = t1;
                    }
                }
            }
        if (!changed) break;
    }
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int k = 0; k < m; k++) {
            double t = At[i * m + k];
            sd += t * t;
        }
        W[i] = sqrt(sd);
    }
    for (int i = 0; i < n - 1; i++) {
        int j = i;
        for (int k = i + 1; k < n; k++)
            if (W[j] < W[k]) j = k;
        if (i != j) {
            double tw = W[i];
            W[i] = W[j];
            W[j] = tw;
            if (Vt) {
                for (int k = 0; k < m; k++) {
                    double t = At[i * m + k];
                    At[i * m + k] = At[j * m + k];
                    At[j * m + k] = t;
                }
                for (int k = 0; k < n; k++) {
                    double t = Vt[i * n + k];
                    Vt[i * n + k] = Vt[j * n + k];
                    Vt[j * n + k] = t;
                }
            }
        }
    }
    for (int i = 0; i < n; i++) Wout[i] = W[i];
    if (!Vt) return;
    unsigned long long rng = 0x12345678;
    for (int i = 0; i < n1; i++) {
        double sd = i < n ? W[i] : 0;
        for (int ii = 0; ii < 100 && sd <= minval; ii++) {
            /* a zero singular value: a random vector made orthogonal to the
             * previous left singular vectors */
            const double val0 = 1. / m;
            for (int k = 0; k < m; k++) At[i * m + k] = (cv_rng_next(&rng) & 256) != 0 ? val0 : -val0;
            for (int it = 0; it < 2; it++)
                for (int j = 0; j < i; j++) {
                    sd = 0;
                    for (int k = 0; k < m; k++) sd += At[i * m + k] * At[j * m + k];
                    double asum = 0;
                    for (int k = 0; k < m; k++) {
                        double t = At[i * m + k] - sd * At[j * m + k];
                        At[i * m + k] = t;
                        asum += fabs(t);
                    }
                    asum = asum > eps * 100 ? 1 / asum : 0;
                    for (int k = 0; k < m; k++) At[i * m + k] *= asum;
                }
            sd = 0;
            for (int k = 0; k < m; k++) {
                double t = At[i * m + k];
                sd += t * t;
            }
            sd = sqrt(sd);
        }
        double s = sd > minval ? 1 / sd : 0.;
        for (int k = 0; k < m; k++) At[i * m + k] *= s;
    }
}

/* cvSVD / SVD::compute of A (m x n, m >= n <= 16, row-major): w (n), u (m x n:
 * column i = left singular vector i) or NULL, vt (n x n: row i = right singular
 * vector i) or NULL (then the Jacobi runs without V, as with NO_UV -- the left
 * vectors it leaves are the same rows). */
void ora_cv_svd(const double* A, int m, int n, double* w, double* u, double* vt)
{
    double At[16 * 16], V[16 * 16];
    for (int i = 0; i < n; i++)
        for (int k = 0; k < m; k++) At[i * m + k] = A[k * n + i]; /* transpose(src, temp_a) */
    ora_cv_jacobi_svd(At, m, n, n, w, V);
    if (u)
        for (int k = 0; k < m; k++)
            for (int i = 0; i < n; i++) u[k * n + i] = At[i * m + k];
    if (vt) memcpy(vt, V, sizeof(double) * n * n);
}

/* The left singular vectors as rows (cvSVD(..., CV_SVD_U_T) of a square A): ut
 * (n x n). */
void ora_cv_svd_ut(const double* A, int n, double* w, double* ut)
{
    double V[16 * 16];
    for (int i = 0; i < n; i++)
        for (int k = 0; k < n; k++) ut[i * n + k] = A[k * n + i];
    ora_cv_jacobi_svd(ut, n, n, n, w, V);
}

/* cv::solve(A, b, x, DECOMP_SVD) for one right-hand side: A (m x n, m >= n). */
void ora_cv_solve_svd(const double* A, int m, int n, const double* b, double* x)
{
    double At[16 * 16], V[16 * 16], w[16];
    for (int i = 0; i < n; i++)
        for (int k = 0; k < m; k++) At[i * m + k] = A[k * n + i];
    ora_cv_jacobi_svd(At, m, n, n, w, V);
    /* SVBkSbImpl_(m, n, w, 1, u = At (uT), v = V (vT), b, nb = 1, x, eps = 2 DBL_EPSILON) */
    double threshold = 0;
    int nm = m < n ? m : n;
    for (int j = 0; j < n; j++) x[j] = 0;
    for (int i = 0; i < nm; i++) threshold += w[i];
    threshold *= DBL_EPSILON * 2;
    for (int i = 0; i < nm; i++) {
        double wi = w[i];
        if (fabs(wi) <= threshold) continue;
        wi = 1 / wi;
        double s = 0;
        for (int j = 0; j < m; j++) s += At[i * m + j] * b[j];
        s *= wi;
        for (int j = 0; j < n; j++) x[j] = x[j] + s * V[i * n + j];
    }
}

/* cv::invert(A, Ai, DECOMP_SVD) of a square n x n A: SVD::compute, then
 * SVD::backSubst with an empty rhs (the identity: u not transposed, nb = n). */
void ora_cv_invert_svd(const double* A, int n, double* Ai)
{
    double u[16 * 16], vt[16 * 16], w[16], buf[16];
    ora_cv_svd(A, n, n, w, u, vt);
    double threshold = 0;
    for (int i = 0; i < n * n; i++) Ai[i] = 0;
    for (int i = 0; i < n; i++) threshold += w[i];
    threshold *= DBL_EPSILON * 2;
    for (int i = 0; i < n; i++) {
        double wi = w[i];
        if (fabs(wi) <= threshold) continue;
        wi = 1 / wi;
        for (int j = 0; j < n; j++) buf[j] = u[j * n + i] * wi;
        /* MatrAXPY(n, nb, buf, 0, vt row i, 1, Ai, n): Ai[r][j] += vt[i][r] * buf[j] */
        for (int r = 0; r < n; r++) {
            double s = vt[i * n + r];
            for (int j = 0; j < n; j++) Ai[r * n + j] = Ai[r * n + j] + s * buf[j];
        }
    }
}

/* cvMulTransposed(src, dst, 1) (MulTransposedR, scale 1): dst = src^T src,
 * dst[i][j] = sum over the rows k in order of src[k][i] src[k][j] for j >= i,
 * the lower triangle mirrored (completeSymm). src: rows x cols. */
void ora_mul_transposed(const double* src, int rows, int cols, double* dst)
{
    for (int i = 0; i < cols; i++)
        for (int j = i; j < cols; j++) {
            double s = 0;
            for (int k = 0; k < rows; k++) s += src[k * cols + i] * src[k * cols + j];
            dst[i * cols + j] = s * 1.0;
        }
    for (int i = 0; i < cols; i++)
        for (int j = 0; j < i; j++) dst[i * cols + j] = dst[j * cols + i];
}
