/* SQPnP (TEST INFRASTRUCTURE ONLY -- see svo_oracle.h): the final
 * solvePnP(..., SOLVEPNP_SQPNP) of cv::solvePnPRansac at R:src/tracking.cpp:191-196,
 * restated from OpenCV 4.x calib3d/src/sqpnp.cpp (sqpnp::PoseSolver) and the
 * published algorithm (G. Terzakis, M. Lourakis, "A Consistently Fast and
 * Globally Optimal Solution to the Perspective-n-Point Problem", ECCV 2020).
 * OpenCV is not in this container: this follows the published algorithm and
 * OpenCV's structure as recalled, independently of the product's solver
 * (svo_amd/csrc/pose.cpp), and is itself unpinned.
 *
 *   computeOmega: Omega = sum_i B_i^T A_i^T A_i B_i - Q^T..., i.e. the cost
 *     E(r) = r^T Omega r of the algebraic image-space error
 *     A_i (R X_i + t), A_i = [1 0 -x_i; 0 1 -y_i], with t eliminated in closed
 *     form (t = P r); sums as PoseSolver::computeOmega (q = sum A_i^T A_i,
 *     qa_sum = sum A_i^T A_i B_i, point-variance and rank checks)
 *   SVD of Omega; the null-space eigenvectors (singular values below the rank
 *     tolerance, at least the smallest one), sqrt(3)-scaled: an orthogonal one is
 *     taken as is (det-signed), else SQP runs from the nearest rotations of +e
 *     and -e; further eigenvectors while the best error exceeds 3 x their
 *     singular value (PoseSolver::solveInternal)
 *   runSQP: at most 15 SQP steps of the linearised orthogonality constraints
 *     (Gram-Schmidt row space H + null space N of the constraint Jacobian,
 *     lower-triangular K = J H; solveSQPSystem), stop when |delta|^2 <= 1e-10;
 *     det < 0 -> -r; det > 1.001 -> nearest rotation
 *   checkSolution: positive depth of the point mean or a majority of positive
 *     depths; keep the smallest error (errors within 1e-6 and vectors within
 *     1e-10 are the same solution); the first solution is solvePnP's. */
#include <float.h>
#include <math.h>
#include <string.h>

#include "oracle_internal.h"
#include "svo_oracle.h"

enum {
    SQ_MAX_ITER = 15,
};
static const double SQ_RANK_TOL = 1e-7, SQ_SQP_SQ_TOL = 1e-10, SQ_DET_THR = 1.001, SQ_ORTHO_SQ_TOL = 1e-8,
                    SQ_EQ_VEC_SQ = 1e-10, SQ_EQ_ERR = 1e-6, SQ_POINT_VAR = 1e-5;

typedef struct {
    double r[9], t[3], sq_error;
} sq_solution;

typedef struct {
    double Om[81], P[27], s[9], U[81]; /* U: column i = singular vector i (U[9 * k + i]) */
    double mean[3];
    int n_null;
    const double* pw;
    int n;
    sq_solution sol[18];
    int n_sol;
} sq_solver;

static double det3(const double* m)
{
    return m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6]) + m[2] * (m[3] * m[7] - m[4] * m[6]);
}

/* analyticalInverse3x3Symm */
static void inv3_symm(const double* q, double* qi)
{
    const double a = q[0], b = q[1], c = q[2], d = q[4], e = q[5], f = q[8];
    const double t2 = e * e, t4 = a * d, t7 = b * b, t9 = b * c, t12 = c * c;
    const double det = -t4 * f + a * t2 + t7 * f - 2.0 * t9 * e + t12 * d;
    const double t15 = 1.0 / det;
    const double t20 = (-b * f + c * e) * t15, t24 = (b * e - c * d) * t15, t30 = (a * e - t9) * t15;
    qi[0] = (-d * f + t2) * t15;
    qi[1] = qi[3] = -t20;
    qi[2] = qi[6] = -t24;
    qi[4] = -(a * f - t12) * t15;
    qi[5] = qi[7] = t30;
    qi[8] = -(t4 - t7) * t15;
}

/* nearestRotationMatrix: the rotation closest (Frobenius) to the 3x3 row-major e */
static void nearest_rotation(const double* e, double* r)
{
    double w[3], u[9], vt[9];
    ora_svd(e, 3, 3, w, u, vt);
    const double d = det3(u) * det3(vt) < 0 ? -1.0 : 1.0;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) r[3 * i + j] = u[3 * i] * vt[j] + u[3 * i + 1] * vt[3 + j] + d * u[3 * i + 2] * vt[6 + j];
}

static double orthogonality_error(const double* e)
{
    const double n1 = e[0] * e[0] + e[1] * e[1] + e[2] * e[2], n2 = e[3] * e[3] + e[4] * e[4] + e[5] * e[5],
                 n3 = e[6] * e[6] + e[7] * e[7] + e[8] * e[8];
    const double d12 = e[0] * e[3] + e[1] * e[4] + e[2] * e[5], d13 = e[0] * e[6] + e[1] * e[7] + e[2] * e[8],
                 d23 = e[3] * e[6] + e[4] * e[7] + e[5] * e[8];
    return (n1 - 1) * (n1 - 1) + (n2 - 1) * (n2 - 1) + (n3 - 1) * (n3 - 1) + 2 * (d12 * d12 + d13 * d13 + d23 * d23);
}

/* PoseSolver::computeOmega. q: normalised image points (undistortPoints). */
static int compute_omega(sq_solver* S, const double* pw, const double* q, int n)
{
    double* Om = S->Om;
    double qa[27];
    memset(Om, 0, sizeof(S->Om));
    memset(qa, 0, sizeof(qa));
    double sx = 0, sy = 0, sq_sum = 0, so[3] = {0, 0, 0};
    for (int i = 0; i < n; i++) {
        const double x = q[2 * i], y = q[2 * i + 1];
        const double X = pw[3 * i], Y = pw[3 * i + 1], Z = pw[3 * i + 2];
        sx += x;
        sy += y;
        so[0] += X;
        so[1] += Y;
        so[2] += Z;
        const double sqn = x * x + y * y;
        sq_sum += sqn;
        const double X2 = X * X, XY = X * Y, XZ = X * Z, Y2 = Y * Y, YZ = Y * Z, Z2 = Z * Z;
        Om[0 * 9 + 0] += X2; Om[0 * 9 + 1] += XY; Om[0 * 9 + 2] += XZ;
        Om[1 * 9 + 1] += Y2; Om[1 * 9 + 2] += YZ; Om[2 * 9 + 2] += Z2;
        Om[0 * 9 + 6] += -x * X2; Om[0 * 9 + 7] += -x * XY; Om[0 * 9 + 8] += -x * XZ;
        Om[1 * 9 + 7] += -x * Y2; Om[1 * 9 + 8] += -x * YZ; Om[2 * 9 + 8] += -x * Z2;
        Om[3 * 9 + 6] += -y * X2; Om[3 * 9 + 7] += -y * XY; Om[3 * 9 + 8] += -y * XZ;
        Om[4 * 9 + 7] += -y * Y2; Om[4 * 9 + 8] += -y * YZ; Om[5 * 9 + 8] += -y * Z2;
        Om[6 * 9 + 6] += sqn * X2; Om[6 * 9 + 7] += sqn * XY; Om[6 * 9 + 8] += sqn * XZ;
        Om[7 * 9 + 7] += sqn * Y2; Om[7 * 9 + 8] += sqn * YZ; Om[8 * 9 + 8] += sqn * Z2;
        qa[0 * 9 + 0] += X; qa[0 * 9 + 1] += Y; qa[0 * 9 + 2] += Z;
        qa[0 * 9 + 6] += -x * X; qa[0 * 9 + 7] += -x * Y; qa[0 * 9 + 8] += -x * Z;
        qa[1 * 9 + 6] += -y * X; qa[1 * 9 + 7] += -y * Y; qa[1 * 9 + 8] += -y * Z;
        qa[2 * 9 + 6] += sqn * X; qa[2 * 9 + 7] += sqn * Y; qa[2 * 9 + 8] += sqn * Z;
    }
    /* the repeated entries of qa_sum and Omega */
    qa[1 * 9 + 3] = qa[0]; qa[1 * 9 + 4] = qa[1]; qa[1 * 9 + 5] = qa[2];
    qa[2 * 9 + 0] = qa[6]; qa[2 * 9 + 1] = qa[7]; qa[2 * 9 + 2] = qa[8];
    qa[2 * 9 + 3] = qa[9 + 6]; qa[2 * 9 + 4] = qa[9 + 7]; qa[2 * 9 + 5] = qa[9 + 8];
    Om[1 * 9 + 6] = Om[0 * 9 + 7]; Om[2 * 9 + 6] = Om[0 * 9 + 8]; Om[2 * 9 + 7] = Om[1 * 9 + 8];
    Om[4 * 9 + 6] = Om[3 * 9 + 7]; Om[5 * 9 + 6] = Om[3 * 9 + 8]; Om[5 * 9 + 7] = Om[4 * 9 + 8];
    Om[7 * 9 + 6] = Om[6 * 9 + 7]; Om[8 * 9 + 6] = Om[6 * 9 + 8]; Om[8 * 9 + 7] = Om[7 * 9 + 8];
    Om[3 * 9 + 3] = Om[0]; Om[3 * 9 + 4] = Om[1]; Om[3 * 9 + 5] = Om[2];
    Om[4 * 9 + 4] = Om[1 * 9 + 1]; Om[4 * 9 + 5] = Om[1 * 9 + 2]; Om[5 * 9 + 5] = Om[2 * 9 + 2];
    for (int i = 0; i < 9; i++)
        for (int j = 0; j < i; j++) Om[i * 9 + j] = Om[j * 9 + i];
    double Q[9] = {(double)n, 0, -sx, 0, (double)n, -sy, -sx, -sy, sq_sum};
    const double inv_n = 1.0 / n;
    const double detQ = n * (n * sq_sum - sy * sy - sx * sx);
    if (detQ * inv_n * inv_n * inv_n < SQ_POINT_VAR) return -1; /* CV_Assert(point_coordinate_variance >= ...) */
    double Qi[9];
    inv3_symm(Q, Qi);
    /* p_ = -Q^-1 qa_sum ; Omega += qa_sum^T p_ */
    for (int a = 0; a < 3; a++)
        for (int c = 0; c < 9; c++) {
            double s = 0;
            for (int k = 0; k < 3; k++) s += Qi[a * 3 + k] * qa[k * 9 + c];
            S->P[a * 9 + c] = -s;
        }
    for (int i = 0; i < 9; i++)
        for (int j = 0; j < 9; j++) {
            double s = 0;
            for (int k = 0; k < 3; k++) s += qa[k * 9 + i] * S->P[k * 9 + j];
            Om[i * 9 + j] += s;
        }
    /* SVD of Omega (symmetric PSD: U = V); columns of V are the singular vectors */
    double w[9], u[81], vt[81];
    ora_svd(Om, 9, 9, w, u, vt);
    for (int i = 0; i < 9; i++) {
        S->s[i] = w[i];
        for (int k = 0; k < 9; k++) S->U[9 * k + i] = vt[9 * i + k];
    }
    if (S->s[0] < 1e-7) return -1; /* CV_Assert(s_(0) >= 1e-7) */
    int nn = 0;
    while (7 - nn >= 0 && S->s[7 - nn] < SQ_RANK_TOL) nn++;
    if (++nn > 6) return -1;
    S->n_null = nn;
    for (int k = 0; k < 3; k++) S->mean[k] = so[k] / n;
    S->pw = pw;
    S->n = n;
    return 0;
}

/* PoseSolver::computeRowAndNullspace: orthonormal row space H (9x6, Gram-Schmidt of
 * the constraint Jacobian J in row order), K = J H (lower triangular) and an
 * orthonormal null space N (9x3) from the columns of I - H H^T. */
static void row_and_nullspace(const double* r, double* H, double* N, double* K)
{
    memset(H, 0, sizeof(double) * 54);
    memset(K, 0, sizeof(double) * 36);
#define HH(i, j) H[(i) * 6 + (j)]
#define KK(i, j) K[(i) * 6 + (j)]
    const double n1 = sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    const double in1 = n1 > 1e-5 ? 1.0 / n1 : 0.0;
    for (int k = 0; k < 3; k++) HH(k, 0) = r[k] * in1;
    KK(0, 0) = 2 * n1;
    const double n2 = sqrt(r[3] * r[3] + r[4] * r[4] + r[5] * r[5]);
    for (int k = 0; k < 3; k++) HH(3 + k, 1) = r[3 + k] / n2;
    KK(1, 1) = 2 * n2;
    const double n3 = sqrt(r[6] * r[6] + r[7] * r[7] + r[8] * r[8]);
    for (int k = 0; k < 3; k++) HH(6 + k, 2) = r[6 + k] / n3;
    KK(2, 2) = 2 * n3;
    /* q4 from J4 = [r2, r1, 0] */
    const double d41 = r[3] * HH(0, 0) + r[4] * HH(1, 0) + r[5] * HH(2, 0);
    const double d42 = r[0] * HH(3, 1) + r[1] * HH(4, 1) + r[2] * HH(5, 1);
    for (int k = 0; k < 3; k++) {
        HH(k, 3) = r[3 + k] - d41 * HH(k, 0);
        HH(3 + k, 3) = r[k] - d42 * HH(3 + k, 1);
    }
    double nn = 0;
    for (int k = 0; k < 9; k++) nn += HH(k, 3) * HH(k, 3);
    nn = 1.0 / sqrt(nn);
    for (int k = 0; k < 9; k++) HH(k, 3) *= nn;
    KK(3, 0) = d41;
    KK(3, 1) = d42;
    KK(3, 3) = r[3] * HH(0, 3) + r[4] * HH(1, 3) + r[5] * HH(2, 3) + r[0] * HH(3, 3) + r[1] * HH(4, 3) + r[2] * HH(5, 3);
    /* q5 from J5 = [0, r3, r2] */
    const double d52 = r[6] * HH(3, 1) + r[7] * HH(4, 1) + r[8] * HH(5, 1);
    const double d53 = r[3] * HH(6, 2) + r[4] * HH(7, 2) + r[5] * HH(8, 2);
    const double d54 = r[6] * HH(3, 3) + r[7] * HH(4, 3) + r[8] * HH(5, 3);
    for (int k = 0; k < 3; k++) {
        HH(k, 4) = -d54 * HH(k, 3);
        HH(3 + k, 4) = r[6 + k] - d52 * HH(3 + k, 1) - d54 * HH(3 + k, 3);
        HH(6 + k, 4) = r[3 + k] - d53 * HH(6 + k, 2);
    }
    nn = 0;
    for (int k = 0; k < 9; k++) nn += HH(k, 4) * HH(k, 4);
    nn = 1.0 / sqrt(nn);
    for (int k = 0; k < 9; k++) HH(k, 4) *= nn;
    KK(4, 1) = d52;
    KK(4, 2) = d53;
    KK(4, 3) = d54;
    KK(4, 4) = r[6] * HH(3, 4) + r[7] * HH(4, 4) + r[8] * HH(5, 4) + r[3] * HH(6, 4) + r[4] * HH(7, 4) + r[5] * HH(8, 4);
    /* q6 from J6 = [r3, 0, r1] */
    const double d61 = r[6] * HH(0, 0) + r[7] * HH(1, 0) + r[8] * HH(2, 0);
    const double d63 = r[0] * HH(6, 2) + r[1] * HH(7, 2) + r[2] * HH(8, 2);
    const double d64 = r[6] * HH(0, 3) + r[7] * HH(1, 3) + r[8] * HH(2, 3);
    const double d65 = r[0] * HH(6, 4) + r[1] * HH(7, 4) + r[2] * HH(8, 4) + r[6] * HH(0, 4) + r[7] * HH(1, 4) +
                       r[8] * HH(2, 4);
    for (int k = 0; k < 3; k++) {
        HH(k, 5) = r[6 + k] - d61 * HH(k, 0) - d64 * HH(k, 3) - d65 * HH(k, 4);
        HH(3 + k, 5) = -d65 * HH(3 + k, 4) - d64 * HH(3 + k, 3);
        HH(6 + k, 5) = r[k] - d63 * HH(6 + k, 2) - d65 * HH(6 + k, 4);
    }
    nn = 0;
    for (int k = 0; k < 9; k++) nn += HH(k, 5) * HH(k, 5);
    nn = 1.0 / sqrt(nn);
    for (int k = 0; k < 9; k++) HH(k, 5) *= nn;
    KK(5, 0) = d61;
    KK(5, 2) = d63;
    KK(5, 3) = d64;
    KK(5, 4) = d65;
    KK(5, 5) = r[6] * HH(0, 5) + r[7] * HH(1, 5) + r[8] * HH(2, 5) + r[0] * HH(6, 5) + r[1] * HH(7, 5) + r[2] * HH(8, 5);
    /* null space: columns of Pn = I - H H^T, the largest first, then the ones
     * least aligned with those already taken, Gram-Schmidt'ed */
    double Pn[81];
    for (int i = 0; i < 9; i++)
        for (int j = 0; j < 9; j++) {
            double s = (i == j) ? 1.0 : 0.0;
            for (int k = 0; k < 6; k++) s -= HH(i, k) * HH(j, k);
            Pn[i * 9 + j] = s;
        }
    double cn[9];
    for (int j = 0; j < 9; j++) {
        double s = 0;
        for (int i = 0; i < 9; i++) s += Pn[i * 9 + j] * Pn[i * 9 + j];
        cn[j] = sqrt(s);
    }
    int taken[3] = {-1, -1, -1};
    for (int c = 0; c < 3; c++) {
        int best = -1;
        double best_score = DBL_MAX;
        for (int j = 0; j < 9; j++) {
            if (j == taken[0] || j == taken[1] || cn[j] < 0.1) continue;
            double score;
            if (c == 0) {
                score = -cn[j];
            } else {
                score = 0;
                for (int m = 0; m < c; m++) {
                    double d = 0;
                    for (int i = 0; i < 9; i++) d += Pn[i * 9 + j] * N[i * 3 + m];
                    score += fabs(d) / cn[j];
                }
            }
            if (score < best_score) {
                best_score = score;
                best = j;
            }
        }
        double v[9];
        for (int i = 0; i < 9; i++) v[i] = Pn[i * 9 + best];
        for (int m = 0; m < c; m++) {
            double d = 0;
            for (int i = 0; i < 9; i++) d += v[i] * N[i * 3 + m];
            for (int i = 0; i < 9; i++) v[i] -= d * N[i * 3 + m];
        }
        double vn = 0;
        for (int i = 0; i < 9; i++) vn += v[i] * v[i];
        vn = 1.0 / sqrt(vn);
        for (int i = 0; i < 9; i++) N[i * 3 + c] = v[i] * vn;
        taken[c] = best;
    }
#undef HH
#undef KK
}

/* PoseSolver::solveSQPSystem: delta = H x + N y with K x = g (the constraint
 * residuals) by forward substitution and y = -(N^T Om N)^-1 N^T Om (r + H x). */
static void solve_sqp_system(const sq_solver* S, const double* r, double* delta)
{
    double H[54], N[27], K[36];
    row_and_nullspace(r, H, N, K);
    const double g[6] = {1 - (r[0] * r[0] + r[1] * r[1] + r[2] * r[2]), 1 - (r[3] * r[3] + r[4] * r[4] + r[5] * r[5]),
                         1 - (r[6] * r[6] + r[7] * r[7] + r[8] * r[8]), -(r[0] * r[3] + r[1] * r[4] + r[2] * r[5]),
                         -(r[3] * r[6] + r[4] * r[7] + r[5] * r[8]), -(r[0] * r[6] + r[1] * r[7] + r[2] * r[8])};
    double x[6];
    x[0] = g[0] / K[0];
    x[1] = g[1] / K[7];
    x[2] = g[2] / K[14];
    x[3] = (g[3] - K[18] * x[0] - K[19] * x[1]) / K[21];
    x[4] = (g[4] - K[25] * x[1] - K[26] * x[2] - K[27] * x[3]) / K[28];
    x[5] = (g[5] - K[30] * x[0] - K[32] * x[2] - K[33] * x[3] - K[34] * x[4]) / K[35];
    for (int i = 0; i < 9; i++) {
        double s = 0;
        for (int k = 0; k < 6; k++) s += H[i * 6 + k] * x[k];
        delta[i] = s;
    }
    double NtOm[27];
    for (int a = 0; a < 3; a++)
        for (int j = 0; j < 9; j++) {
            double s = 0;
            for (int i = 0; i < 9; i++) s += N[i * 3 + a] * S->Om[i * 9 + j];
            NtOm[a * 9 + j] = s;
        }
    double W[9], Wi[9];
    for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) {
            double s = 0;
            for (int j = 0; j < 9; j++) s += NtOm[a * 9 + j] * N[j * 3 + b];
            W[a * 3 + b] = s;
        }
    inv3_symm(W, Wi);
    double rhs[3];
    for (int a = 0; a < 3; a++) {
        double s = 0;
        for (int j = 0; j < 9; j++) s += NtOm[a * 9 + j] * (delta[j] + r[j]);
        rhs[a] = s;
    }
    double y[3];
    for (int a = 0; a < 3; a++) y[a] = -(Wi[a * 3] * rhs[0] + Wi[a * 3 + 1] * rhs[1] + Wi[a * 3 + 2] * rhs[2]);
    for (int i = 0; i < 9; i++) delta[i] += N[i * 3] * y[0] + N[i * 3 + 1] * y[1] + N[i * 3 + 2] * y[2];
}

static void run_sqp(const sq_solver* S, const double* r0, sq_solution* sol)
{
    double r[9], delta[9];
    memcpy(r, r0, sizeof(r));
    double dsq = DBL_MAX;
    int step = 0;
    while (dsq > SQ_SQP_SQ_TOL && step++ < SQ_MAX_ITER) {
        solve_sqp_system(S, r, delta);
        dsq = 0;
        for (int i = 0; i < 9; i++) {
            r[i] += delta[i];
            dsq += delta[i] * delta[i];
        }
    }
    double d = det3(r);
    if (d < 0) {
        for (int i = 0; i < 9; i++) r[i] = -r[i];
        d = -d;
    }
    if (d > SQ_DET_THR)
        nearest_rotation(r, sol->r);
    else
        memcpy(sol->r, r, sizeof(r));
}

static int positive_depth(const sq_solver* S, const sq_solution* s)
{
    const double* r = s->r;
    return r[6] * S->mean[0] + r[7] * S->mean[1] + r[8] * S->mean[2] + s->t[2] > 0;
}

static int positive_majority(const sq_solver* S, const sq_solution* s)
{
    int npos = 0, nneg = 0;
    for (int i = 0; i < S->n; i++) {
        const double* p = S->pw + 3 * i;
        if (s->r[6] * p[0] + s->r[7] * p[1] + s->r[8] * p[2] + s->t[2] > 0)
            npos++;
        else
            nneg++;
    }
    return npos >= nneg;
}

static void check_solution(sq_solver* S, sq_solution* s, double* min_err)
{
    for (int a = 0; a < 3; a++) {
        double v = 0;
        for (int c = 0; c < 9; c++) v += S->P[a * 9 + c] * s->r[c];
        s->t[a] = v;
    }
    if (!(positive_depth(S, s) || positive_majority(S, s))) return;
    double e = 0;
    for (int i = 0; i < 9; i++) {
        double v = 0;
        for (int j = 0; j < 9; j++) v += S->Om[i * 9 + j] * s->r[j];
        e += v * s->r[i];
    }
    s->sq_error = e;
    if (fabs(*min_err - e) > SQ_EQ_ERR) {
        if (*min_err > e) {
            *min_err = e;
            S->sol[0] = *s;
            S->n_sol = 1;
        }
    } else {
        int found = 0;
        for (int i = 0; i < S->n_sol; i++) {
            double d = 0;
            for (int k = 0; k < 9; k++) d += (S->sol[i].r[k] - s->r[k]) * (S->sol[i].r[k] - s->r[k]);
            if (d < SQ_EQ_VEC_SQ) {
                if (S->sol[i].sq_error > e) S->sol[i] = *s;
                found = 1;
                break;
            }
        }
        if (!found && S->n_sol < 18) S->sol[S->n_sol++] = *s;
        if (*min_err > e) *min_err = e;
    }
}

/* the SQP runs from the nearest rotations of +e and -e */
static void from_eigenvector(sq_solver* S, const double* e, double* min_err)
{
    double m[9], r[9];
    sq_solution s;
    nearest_rotation(e, r);
    run_sqp(S, r, &s);
    check_solution(S, &s, min_err);
    for (int k = 0; k < 9; k++) m[k] = -e[k];
    nearest_rotation(m, r);
    run_sqp(S, r, &s);
    check_solution(S, &s, min_err);
}

int svo_oracle_sqpnp(const double* pw, const double* q, int n, double R[9], double t[3])
{
    if (n < 3) return -1;
    sq_solver S;
    memset(&S, 0, sizeof(S));
    if (compute_omega(&S, pw, q, n) != 0) return -1;
    double min_err = DBL_MAX;
    const int ne = S.n_null > 0 ? S.n_null : 1;
    for (int i = 9 - ne; i < 9; i++) {
        double e[9];
        for (int k = 0; k < 9; k++) e[k] = sqrt(3.0) * S.U[9 * k + i];
        if (orthogonality_error(e) < SQ_ORTHO_SQ_TOL) {
            sq_solution s;
            const double d = det3(e);
            for (int k = 0; k < 9; k++) s.r[k] = d * e[k];
            check_solution(&S, &s, &min_err);
        } else {
            from_eigenvector(&S, e, &min_err);
        }
    }
    for (int c = 1; 9 - ne - c > 0 && min_err > 3 * S.s[9 - ne - c]; c++) {
        double e[9];
        for (int k = 0; k < 9; k++) e[k] = S.U[9 * k + (9 - ne - c)];
        from_eigenvector(&S, e, &min_err);
    }
    if (S.n_sol == 0) return -1;
    memcpy(R, S.sol[0].r, sizeof(double) * 9);
    memcpy(t, S.sol[0].t, sizeof(double) * 3);
    return 0;
}
