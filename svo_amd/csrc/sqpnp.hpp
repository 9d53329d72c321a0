// solvePnPRansac's final fit, solvePnP(SOLVEPNP_SQPNP) on the inliers
// (R:src/tracking.cpp:191-196; OpenCV calib3d/src/sqpnp.cpp), from the 40 sufficient
// statistics of the inlier set (pose.hpp kSqpnpStats): __host__ __device__, fixed
// sizes, no allocation. The host runs it for svo_solve_pnp_sqpnp / svo_solve_pnp_ransac
// (pose.cpp); the batched front end runs it on the device, one wave per sequence
// (launch_sqpnp_fit, pnp.hip): the SQP starts over waves, the KKT rows over lanes.
#pragma once

#include "epnp.hpp"
#include "linalg.hpp"

namespace svo {
namespace sq {

// ---- SQPnP's cost, E(R) = vec(R)^T Omega vec(R) ----
struct SqpnpCost {
    double Om[81];
    double P[27];    // t = P vec(R)
    double mean[3];  // object-point mean (PoseSolver::positiveDepth)
    bool ok;         // computeOmega's point-variance assert held
};

// pinv of SQPnP's 3 x 3 Q (la::pinv3, the same arithmetic) -- here so the device
// build needs nothing from the host-only helpers
SVO_HD void sq_pinv3(const double* A, double* Ai) { la::pinv3(A, Ai); }

// PoseSolver::computeOmega from the statistics: Omega_raw = sum B_i^T A_i^T A_i
// B_i (blocks XX^T, -x XX^T, -y XX^T, (x^2+y^2) XX^T), qa = sum A_i^T A_i B_i,
// Q = sum A_i^T A_i, P = -Q^-1 qa, Omega = Omega_raw + qa^T P; ok = false where
// SQPnP asserts on the points (their variance below 1e-5); Omega's own asserts
// (largest singular value below 1e-7, more than 6 null vectors) are checked on
// its eigenvalues in the solution search.
SVO_HD void sqpnp_assemble(const double* sums, SqpnpCost& c) {
    const int IDX[3][3] = {{0, 1, 2}, {1, 3, 4}, {2, 4, 5}};  // unique entries of a sym 3x3
    const double n = sums[0], sx = sums[1], sy = sums[2], ssq = sums[3];
    auto SX = [&](int u, int j) { return sums[4 + 3 * u + j]; };                  // sum c_u X_j
    auto SXX = [&](int u, int a, int b) { return sums[16 + 6 * u + IDX[a][b]]; };  // sum c_u X_a X_b
    double Om[81], qa[27];
    for (int i = 0; i < 81; i++) Om[i] = 0;
    for (int i = 0; i < 27; i++) qa[i] = 0;
    for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) {
            Om[9 * a + b] = SXX(0, a, b);
            Om[9 * (3 + a) + 3 + b] = SXX(0, a, b);
            Om[9 * a + 6 + b] = Om[9 * (6 + b) + a] = -SXX(1, a, b);
            Om[9 * (3 + a) + 6 + b] = Om[9 * (6 + b) + 3 + a] = -SXX(2, a, b);
            Om[9 * (6 + a) + 6 + b] = SXX(3, a, b);
        }
    for (int j = 0; j < 3; j++) {
        qa[j] = SX(0, j);
        qa[6 + j] = -SX(1, j);
        qa[9 + 3 + j] = SX(0, j);
        qa[9 + 6 + j] = -SX(2, j);
        qa[18 + j] = -SX(1, j);
        qa[18 + 3 + j] = -SX(2, j);
        qa[18 + 6 + j] = SX(3, j);
    }
    const double Q[9] = {n, 0, -sx, 0, n, -sy, -sx, -sy, ssq};
    const double detQ = n * (n * ssq - sy * sy - sx * sx);
    c.ok = n > 0 && detQ / (n * n * n) >= 1e-5;
    double Qi[9];
    sq_pinv3(Q, Qi);
    for (int a = 0; a < 3; a++)
        for (int col = 0; col < 9; col++)
            c.P[9 * a + col] = -(Qi[3 * a] * qa[col] + Qi[3 * a + 1] * qa[9 + col] + Qi[3 * a + 2] * qa[18 + col]);
    for (int i = 0; i < 9; i++)
        for (int j = 0; j < 9; j++)
            c.Om[9 * i + j] = Om[9 * i + j] + (qa[i] * c.P[j] + qa[9 + i] * c.P[9 + j] + qa[18 + i] * c.P[18 + j]);
    for (int r = 0; r < 9; r++)  // symmetrise
        for (int col = 0; col < r; col++) {
            const double v = 0.5 * (c.Om[9 * r + col] + c.Om[9 * col + r]);
            c.Om[9 * r + col] = c.Om[9 * col + r] = v;
        }
    for (int j = 0; j < 3; j++) c.mean[j] = n > 0 ? SX(0, j) / n : 0.0;
}

SVO_HD double quad(const double* Om, const double* r) {
    double s = 0;
    for (int i = 0; i < 9; i++) {
        double t = 0;
        for (int j = 0; j < 9; j++) t += Om[9 * i + j] * r[j];
        s += r[i] * t;
    }
    return s;
}

// One SQP step of SQPnP (PoseSolver::solveSQPSystem) at r: the delta minimising
// (r + delta)^T Om (r + delta) subject to the orthogonality constraints
// linearised at r, J delta = -h(r) (h: the three row norms - 1 and the three row
// dot products), from the KKT system [2 Om, J^T; J, 0] [delta; l] = [-2 Om r; -h]
// solved by Gaussian elimination with partial pivoting (OpenCV solves the same
// system through an orthonormal row / null-space split of J).
SVO_HD void sqp_step(const double* Om, const double* r, double* delta) {
    constexpr int N = 15;
    double A[N][N + 1];
    for (int i = 0; i < N; i++)
        for (int j = 0; j <= N; j++) A[i][j] = 0;
    const double* r1 = r;
    const double* r2 = r + 3;
    const double* r3 = r + 6;
    for (int i = 0; i < 9; i++) {
        double g = 0;
        for (int j = 0; j < 9; j++) {
            A[i][j] = 2 * Om[9 * i + j];
            g += Om[9 * i + j] * r[j];
        }
        A[i][N] = -2 * g;
    }
    double J[6][9];
    for (int i = 0; i < 6; i++)
        for (int j = 0; j < 9; j++) J[i][j] = 0;
    for (int k = 0; k < 3; k++) {
        J[0][k] = 2 * r1[k];
        J[1][3 + k] = 2 * r2[k];
        J[2][6 + k] = 2 * r3[k];
        J[3][k] = r2[k];
        J[3][3 + k] = r1[k];
        J[4][3 + k] = r3[k];
        J[4][6 + k] = r2[k];
        J[5][k] = r3[k];
        J[5][6 + k] = r1[k];
    }
    const double h[6] = {dot3(r1, r1) - 1, dot3(r2, r2) - 1, dot3(r3, r3) - 1, dot3(r1, r2), dot3(r2, r3),
                         dot3(r1, r3)};
    for (int c = 0; c < 6; c++) {
        for (int j = 0; j < 9; j++) {
            A[9 + c][j] = J[c][j];
            A[j][9 + c] = J[c][j];
        }
        A[9 + c][N] = -h[c];
    }
    for (int col = 0; col < N; col++) {
        int piv = col;
        for (int i = col + 1; i < N; i++)
            if (fabs(A[i][col]) > fabs(A[piv][col])) piv = i;
        if (piv != col)
            for (int j = 0; j <= N; j++) {
                const double tmp = A[col][j];
                A[col][j] = A[piv][j];
                A[piv][j] = tmp;
            }
        const double d = A[col][col];
        if (d == 0) continue;
        for (int i = col + 1; i < N; i++) {
            const double f = A[i][col] / d;
            if (f == 0) continue;
            for (int j = col; j <= N; j++) A[i][j] -= f * A[col][j];
        }
    }
    double x[N];
    for (int i = N - 1; i >= 0; i--) {
        double v = A[i][N];
        for (int j = i + 1; j < N; j++) v -= A[i][j] * x[j];
        x[i] = A[i][i] != 0 ? v / A[i][i] : 0.0;
    }
    for (int k = 0; k < 9; k++) delta[k] = x[k];
}

// PoseSolver::runSQP: at most 15 steps while |delta|^2 > 1e-10; then -r if
// det < 0, and the nearest rotation only if det > 1.001 (r as is otherwise --
// its cost and t are taken unprojected, as OpenCV does).
SVO_HD void sqp_run(const double* Om, const double* r0, double* rhat) {
    double r[9], delta[9];
    for (int k = 0; k < 9; k++) r[k] = r0[k];
    double dsq = 1.7976931348623157e308;
    int step = 0;
    while (dsq > 1e-10 && step++ < 15) {
        sqp_step(Om, r, delta);
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

SVO_HD double ortho_err(const double* e) {
    const double n1 = e[0] * e[0] + e[1] * e[1] + e[2] * e[2], n2 = e[3] * e[3] + e[4] * e[4] + e[5] * e[5],
                 n3 = e[6] * e[6] + e[7] * e[7] + e[8] * e[8];
    const double d12 = e[0] * e[3] + e[1] * e[4] + e[2] * e[5], d13 = e[0] * e[6] + e[1] * e[7] + e[2] * e[8],
                 d23 = e[3] * e[6] + e[4] * e[7] + e[5] * e[8];
    return (n1 - 1) * (n1 - 1) + (n2 - 1) * (n2 - 1) + (n3 - 1) * (n3 - 1) + 2 * (d12 * d12 + d13 * d13 + d23 * d23);
}

SVO_HD double det33(const double* m) {
    return m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6]) + m[2] * (m[3] * m[7] - m[4] * m[6]);
}

// The SQP run from start j of Omega's eigenvector i = j / 2 (row i of evec,
// descending eigenvalues): sqrt(3) e, negated for odd j, its nearest rotation,
// then sqp_run. Independent of every other start: the device runs them in lanes.
SVO_HD void sq_start(const SqpnpCost& c, const double* evec, int j, double* r) {
    const double* ev = evec + 9 * (j >> 1);
    double m[9], r0[9];
    for (int k = 0; k < 9; k++) m[k] = (j & 1) ? -(1.7320508075688772 * ev[k]) : 1.7320508075688772 * ev[k];
    la::nearest_rotation(m, r0);
    sqp_run(c.Om, r0, r);
}

// The number of null vectors SQPnP searches from (eigenvalues below the rank
// tolerance 1e-7; at least the smallest); -1 where SQPnP asserts on Omega
// (CV_Assert(s_(0) >= 1e-7): its largest eigenvalue -- Omega is symmetric PSD, its
// singular values are its eigenvalues -- or more than 6 null vectors).
SVO_HD int sq_null_count(const double* ev) {
    if (!(ev[0] >= 1e-7)) return -1;
    int nn = 0;
    while (7 - nn >= 0 && ev[7 - nn] < 1e-7) nn++;
    return ++nn > 6 ? -1 : nn;
}

struct SqSol {
    double r[9], t[3], err;
};

// SQPnP's solution search (PoseSolver::solveInternal) over Omega's eigenvectors:
//   the null-space eigenvectors e, sqrt(3)-scaled: if e is already orthogonal
//   (squared orthogonality error < 1e-8) it is taken as is, det-signed, with t = P e
//   (no refinement -- OpenCV's shortcut); else runs from the nearest rotations of +e
//   and -e; then further eigenvectors while the best error exceeds 3x their
//   eigenvalue. checkSolution: the object-point mean in front of the camera or a
//   majority of positive depths; errors within 1e-6 and rotations within 1e-10
//   are one solution; the first smallest-error solution is solvePnP's.
// run(j, r): start j's SQP result (sq_start, computed here or beforehand);
// n_front(r, t): how many of the n fitted points lie in front of (r, t).
template <class Run, class Front>
SVO_HD void sq_select(const SqpnpCost& c, const double* ev, const double* evec, int nn, int n, Run run,
                      Front n_front, double R[9], double t[3], bool* found) {
    // OpenCV keeps every distinct solution within 1e-6 of the smallest error and
    // returns the first; a later one can replace only the first, when it is the
    // same rotation with a smaller error, so only that one is kept here
    SqSol best{};
    bool have = false;
    double min_err = 1.7976931348623157e308;
    auto check = [&](SqSol& s) {
        for (int a = 0; a < 3; a++) {
            s.t[a] = 0;
            for (int col = 0; col < 9; col++) s.t[a] += c.P[9 * a + col] * s.r[col];
        }
        bool front = dot3(s.r + 6, c.mean) + s.t[2] > 0;
        if (!front) {
            const int pos = n_front(s.r, s.t);
            front = pos >= n - pos;
        }
        if (!front) return;
        s.err = quad(c.Om, s.r);
        if (fabs(min_err - s.err) > 1e-6) {
            if (min_err > s.err) {
                min_err = s.err;
                best = s;
                have = true;
            }
        } else {
            double d = 0;
            for (int k = 0; k < 9; k++) d += (best.r[k] - s.r[k]) * (best.r[k] - s.r[k]);
            if (d < 1e-10 && best.err > s.err) best = s;
            if (min_err > s.err) min_err = s.err;
        }
    };
    auto from_eigen = [&](int i) {
        for (int sg = 0; sg < 2; sg++) {
            SqSol s;
            run(2 * i + sg, s.r);
            check(s);
        }
    };
    for (int i = 9 - nn; i < 9; i++) {
        double e[9];
        for (int k = 0; k < 9; k++) e[k] = 1.7320508075688772 * evec[9 * i + k];
        if (ortho_err(e) < 1e-8) {
            SqSol s;
            const double d = det33(e);
            for (int k = 0; k < 9; k++) s.r[k] = d * e[k];
            check(s);
        } else {
            from_eigen(i);
        }
    }
    for (int k = 1; 9 - nn - k > 0 && min_err > 3 * ev[9 - nn - k]; k++) from_eigen(9 - nn - k);
    *found = have;
    if (!have) return;
    for (int k = 0; k < 9; k++) R[k] = best.r[k];  // (rodrigues_inv re-orthonormalises, as cv::Rodrigues)
    for (int k = 0; k < 3; k++) t[k] = best.t[k];
}

}  // namespace sq
}  // namespace svo
