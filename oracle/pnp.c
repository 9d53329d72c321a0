/*
 * Oracle (TEST INFRASTRUCTURE ONLY -- see svo_oracle.h; parity unpinned).
 *
 * Restates the pose update the reference runs at R:src/tracking.cpp:191-196:
 *   cv::solvePnPRansac(worldPoints(Point3d), leftPoints(Point2f), K(Matx33f),
 *                      zeros(1,4), rvec, tvec, false, 100, 8.0, 0.999,
 *                      inliers, SOLVEPNP_SQPNP)
 * following OpenCV 4.x calib3d/src/solvepnp.cpp (solvePnPRansac, PnPRansacCallback),
 * calib3d/src/ptsetreg.cpp (RANSACPointSetRegistrator::run / getSubset /
 * findInliers, RANSACUpdateNumIters), calib3d/src/epnp.cpp (EPnP minimal kernel),
 * calib3d/src/calibration.cpp (projectPoints, Rodrigues),
 * core/include/opencv2/core/operations.hpp (cv::RNG).
 *
 * The RANSAC stage (subset sequence, scoring, accept rule, iteration update) is
 * restated exactly. EPnP follows epnp.cpp operation by operation, its SVDs /
 * inverse / least-squares solves being OpenCV's lapack.cpp Jacobi restated in
 * cvsvd.c (cvSVD, cvInvert(CV_SVD), cvSolve(CV_SVD)), the image points
 * normalised by undistortPoints into float as OpenCV's CV_32FC2 output, and the
 * model stored through cv::Rodrigues (its SVD the same Jacobi). The product's
 * minimal solver restates the same operations (svo_amd/csrc/epnp.hpp), so the
 * two pick the same basis of the 5-point M^T M's two-dimensional null space and
 * their hypotheses agree bit for bit (tests/test_epnp_cpu.py). The final
 * solvePnP(SQPNP) on the inliers is sqpnp.c.
 */
#include "svo_oracle.h"
#include "oracle_internal.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

uint32_t svo_oracle_rng_next(uint64_t* state)
{
    *state = (uint64_t)(uint32_t)(*state) * 4164903690U + (uint32_t)(*state >> 32);
    return (uint32_t)(*state);
}

static int rng_uniform(uint64_t* state, int a, int b)
{
    return a == b ? a : (int)(svo_oracle_rng_next(state) % (unsigned)(b - a) + a);
}

int svo_oracle_get_subset(uint64_t* rng_state, int count, int k, int* idx)
{
    /* getSubset(maxAttempts = 10000); the PnP callback's checkSubset accepts
     * every subset, so the first attempt always succeeds */
    for (int i = 0; i < k; i++) {
        int idx_i;
        for (;;) {
            idx_i = rng_uniform(rng_state, 0, count);
            int dup = 0;
            for (int j = 0; j < i; j++)
                if (idx[j] == idx_i) { dup = 1; break; }
            if (!dup) break;
        }
        idx[i] = idx_i;
    }
    return 1;
}

void svo_oracle_rodrigues(const double rv[3], double R[9])
{
    double rx = rv[0], ry = rv[1], rz = rv[2];
    double theta = sqrt(rx * rx + ry * ry + rz * rz);
    if (theta < DBL_EPSILON) {
        for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0) ? 1.0 : 0.0;
        return;
    }
    double c = cos(theta), s = sin(theta), c1 = 1. - c;
    double itheta = theta ? 1. / theta : 0.;
    rx *= itheta; ry *= itheta; rz *= itheta;
    double rrt[9] = {rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz};
    double r_x[9] = {0, -rz, ry, rz, 0, -rx, -ry, rx, 0};
    for (int i = 0; i < 9; i++) R[i] = (c * ((i % 4 == 0) ? 1.0 : 0.0) + c1 * rrt[i]) + s * r_x[i];
}

void svo_oracle_rodrigues_inv(const double Rin[9], double rv[3])
{
    /* cv::Rodrigues: SVD::compute(R, W, U, Vt); R = U * Vt (Matx product: s = 0,
     * s += u(i,k) vt(k,j) for k = 0..2) */
    double w[3], u[9], vt[9], R[9];
    ora_cv_svd(Rin, 3, 3, w, u, vt);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double acc = 0;
            for (int k = 0; k < 3; k++) acc += u[i * 3 + k] * vt[k * 3 + j];
            R[i * 3 + j] = acc;
        }
    double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
    double s = sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
    double c = (R[0] + R[4] + R[8] - 1) * 0.5;
    c = c > 1. ? 1. : c < -1. ? -1. : c;
    double theta = acos(c);
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
            theta /= sqrt(rx * rx + ry * ry + rz * rz);
            rx *= theta; ry *= theta; rz *= theta;
        }
    } else {
        double vth = 1 / (2 * s);
        vth *= theta;
        rx *= vth; ry *= vth; rz *= vth;
    }
    rv[0] = rx; rv[1] = ry; rv[2] = rz;
}

/* projectPoints (zero distortion, identity tilt) -> CV_32F, then
 * err = normL2Sqr<float,float>(ipt - ppt), inlier iff err <= thresh2. */
void svo_oracle_pnp_residuals(const float* obj, const float* img, int n, const double* hyp,
                              int m, const double K[9], float thresh2, float* err,
                              uint8_t* mask, int* counts)
{
    double fx = K[0], fy = K[4], cx = K[2], cy = K[5];
    for (int h = 0; h < m; h++) {
        const double* R = hyp + 12 * h;
        const double* t = R + 9;
        int cnt = 0;
        for (int i = 0; i < n; i++) {
            double X = obj[3 * i], Y = obj[3 * i + 1], Z = obj[3 * i + 2];
            double x = R[0] * X + R[1] * Y + R[2] * Z + t[0];
            double y = R[3] * X + R[4] * Y + R[5] * Z + t[1];
            double z = R[6] * X + R[7] * Y + R[8] * Z + t[2];
            z = z ? 1. / z : 1;
            x *= z;
            y *= z;
            float u = (float)(x * fx + cx), v = (float)(y * fy + cy);
            float dx = img[2 * i] - u, dy = img[2 * i + 1] - v;
            float s = 0.f;
            s += dx * dx;
            s += dy * dy;
            if (err) err[(size_t)h * n + i] = s;
            int f = s <= thresh2;
            if (mask) mask[(size_t)h * n + i] = (uint8_t)f;
            cnt += f;
        }
        if (counts) counts[h] = cnt;
    }
}

/* ------------------------------------------------------------------ EPnP */

typedef struct {
    int n;
    double uc, vc, fu, fv;
    double *pws, *us, *alphas, *pcs;
    double cws[4][3], ccs[4][3];
} epnp_t;

static double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static double dist2(const double* a, const double* b)
{
    return (a[0] - b[0]) * (a[0] - b[0]) + (a[1] - b[1]) * (a[1] - b[1]) + (a[2] - b[2]) * (a[2] - b[2]);
}

static void choose_control_points(epnp_t* e)
{
    int n = e->n;
    e->cws[0][0] = e->cws[0][1] = e->cws[0][2] = 0;
    for (int i = 0; i < n; i++)
        for (int j = 0; j < 3; j++) e->cws[0][j] += e->pws[3 * i + j];
    for (int j = 0; j < 3; j++) e->cws[0][j] /= n;
    /* PW0 = pws - c0; cvMulTransposed(PW0, PW0tPW0, 1); cvSVD(U_T) */
    double* pw0 = (double*)malloc(sizeof(double) * 3 * n);
    for (int i = 0; i < n; i++)
        for (int j = 0; j < 3; j++) pw0[3 * i + j] = e->pws[3 * i + j] - e->cws[0][j];
    double M[9];
    ora_mul_transposed(pw0, n, 3, M);
    free(pw0);
    double dc[3], uct[9];
    ora_cv_svd_ut(M, 3, dc, uct);
    for (int i = 1; i < 4; i++) {
        double k = sqrt(dc[i - 1] / n);
        for (int j = 0; j < 3; j++) e->cws[i][j] = e->cws[0][j] + k * uct[3 * (i - 1) + j];
    }
}

static void compute_barycentric(epnp_t* e)
{
    double cc[9], ci[9];
    for (int i = 0; i < 3; i++)
        for (int j = 1; j < 4; j++) cc[3 * i + j - 1] = e->cws[j][i] - e->cws[0][i];
    ora_cv_invert_svd(cc, 3, ci); /* cvInvert(&CC, &CC_inv, CV_SVD) */
    for (int i = 0; i < e->n; i++) {
        double* pi = e->pws + 3 * i;
        double* a = e->alphas + 4 * i;
        for (int j = 0; j < 3; j++)
            a[1 + j] = ci[3 * j] * (pi[0] - e->cws[0][0]) + ci[3 * j + 1] * (pi[1] - e->cws[0][1]) +
                       ci[3 * j + 2] * (pi[2] - e->cws[0][2]);
        a[0] = 1.0 - a[1] - a[2] - a[3];
    }
}

static void compute_L_6x10(const double* ut, double* l)
{
    const double* v[4] = {ut + 12 * 11, ut + 12 * 10, ut + 12 * 9, ut + 12 * 8};
    double dv[4][6][3];
    for (int i = 0; i < 4; i++) {
        int a = 0, b = 1;
        for (int j = 0; j < 6; j++) {
            for (int k = 0; k < 3; k++) dv[i][j][k] = v[i][3 * a + k] - v[i][3 * b + k];
            b++;
            if (b > 3) { a++; b = a + 1; }
        }
    }
    for (int i = 0; i < 6; i++) {
        double* row = l + 10 * i;
        row[0] = dot3(dv[0][i], dv[0][i]);
        row[1] = 2.0 * dot3(dv[0][i], dv[1][i]);
        row[2] = dot3(dv[1][i], dv[1][i]);
        row[3] = 2.0 * dot3(dv[0][i], dv[2][i]);
        row[4] = 2.0 * dot3(dv[1][i], dv[2][i]);
        row[5] = dot3(dv[2][i], dv[2][i]);
        row[6] = 2.0 * dot3(dv[0][i], dv[3][i]);
        row[7] = 2.0 * dot3(dv[1][i], dv[3][i]);
        row[8] = 2.0 * dot3(dv[2][i], dv[3][i]);
        row[9] = dot3(dv[3][i], dv[3][i]);
    }
}

static void find_betas_1(const double* L, const double* rho, double* betas)
{
    double A[24], b4[4];
    for (int i = 0; i < 6; i++) {
        A[4 * i] = L[10 * i]; A[4 * i + 1] = L[10 * i + 1]; A[4 * i + 2] = L[10 * i + 3]; A[4 * i + 3] = L[10 * i + 6];
    }
    ora_cv_solve_svd(A, 6, 4, rho, b4);
    if (b4[0] < 0) {
        betas[0] = sqrt(-b4[0]);
        betas[1] = -b4[1] / betas[0]; betas[2] = -b4[2] / betas[0]; betas[3] = -b4[3] / betas[0];
    } else {
        betas[0] = sqrt(b4[0]);
        betas[1] = b4[1] / betas[0]; betas[2] = b4[2] / betas[0]; betas[3] = b4[3] / betas[0];
    }
}

static void find_betas_2(const double* L, const double* rho, double* betas)
{
    double A[18], b3[3];
    for (int i = 0; i < 6; i++) { A[3 * i] = L[10 * i]; A[3 * i + 1] = L[10 * i + 1]; A[3 * i + 2] = L[10 * i + 2]; }
    ora_cv_solve_svd(A, 6, 3, rho, b3);
    if (b3[0] < 0) {
        betas[0] = sqrt(-b3[0]);
        betas[1] = (b3[2] < 0) ? sqrt(-b3[2]) : 0.0;
    } else {
        betas[0] = sqrt(b3[0]);
        betas[1] = (b3[2] > 0) ? sqrt(b3[2]) : 0.0;
    }
    if (b3[1] < 0) betas[0] = -betas[0];
    betas[2] = 0.0; betas[3] = 0.0;
}

static void find_betas_3(const double* L, const double* rho, double* betas)
{
    double A[30], b5[5];
    for (int i = 0; i < 6; i++)
        for (int k = 0; k < 5; k++) A[5 * i + k] = L[10 * i + k];
    ora_cv_solve_svd(A, 6, 5, rho, b5);
    if (b5[0] < 0) {
        betas[0] = sqrt(-b5[0]);
        betas[1] = (b5[2] < 0) ? sqrt(-b5[2]) : 0.0;
    } else {
        betas[0] = sqrt(b5[0]);
        betas[1] = (b5[2] > 0) ? sqrt(b5[2]) : 0.0;
    }
    if (b5[1] < 0) betas[0] = -betas[0];
    betas[2] = b5[3] / betas[0];
    betas[3] = 0.0;
}

/* epnp::qr_solve (Householder) */
static void qr_solve(double* A, int nr, int nc, double* b, double* X)
{
    double A1[16], A2[16];
    double *pA = A, *ppAkk = pA;
    for (int k = 0; k < nc; k++) {
        double *ppAik1 = ppAkk, eta = fabs(*ppAik1);
        for (int i = k + 1; i < nr; i++) {
            double elt = fabs(*ppAik1);
            if (eta < elt) eta = elt;
            ppAik1 += nc;
        }
        if (eta == 0) {
            A1[k] = A2[k] = 0.0;
            return;
        }
        double *ppAik2 = ppAkk, sum2 = 0.0, inv_eta = 1. / eta;
        for (int i = k; i < nr; i++) {
            *ppAik2 *= inv_eta;
            sum2 += *ppAik2 * *ppAik2;
            ppAik2 += nc;
        }
        double sigma = sqrt(sum2);
        if (*ppAkk < 0) sigma = -sigma;
        *ppAkk += sigma;
        A1[k] = sigma * *ppAkk;
        A2[k] = -eta * sigma;
        for (int j = k + 1; j < nc; j++) {
            double *ppAik = ppAkk, sum = 0;
            for (int i = k; i < nr; i++) { sum += *ppAik * ppAik[j - k]; ppAik += nc; }
            double tau = sum / A1[k];
            ppAik = ppAkk;
            for (int i = k; i < nr; i++) { ppAik[j - k] -= tau * *ppAik; ppAik += nc; }
        }
        ppAkk += nc + 1;
    }
    double *ppAjj = pA, *pb = b;
    for (int j = 0; j < nc; j++) {
        double *ppAij = ppAjj, tau = 0;
        for (int i = j; i < nr; i++) { tau += *ppAij * pb[i]; ppAij += nc; }
        tau /= A1[j];
        ppAij = ppAjj;
        for (int i = j; i < nr; i++) { pb[i] -= tau * *ppAij; ppAij += nc; }
        ppAjj += nc + 1;
    }
    X[nc - 1] = pb[nc - 1] / A2[nc - 1];
    for (int i = nc - 2; i >= 0; i--) {
        double *ppAij = pA + i * nc + (i + 1), sum = 0;
        for (int j = i + 1; j < nc; j++) { sum += *ppAij * X[j]; ppAij++; }
        X[i] = (pb[i] - sum) / A2[i];
    }
}

static void gauss_newton(const double* L, const double* rho, double betas[4])
{
    /* x outlives the iterations, as epnp.cpp's: a qr_solve that returns early
     * (a zero column) leaves the previous step in it */
    double x[4] = {0, 0, 0, 0};
    for (int it = 0; it < 5; it++) {
        double A[24], b[6];
        for (int i = 0; i < 6; i++) {
            const double* r = L + 10 * i;
            A[4 * i + 0] = 2 * r[0] * betas[0] + r[1] * betas[1] + r[3] * betas[2] + r[6] * betas[3];
            A[4 * i + 1] = r[1] * betas[0] + 2 * r[2] * betas[1] + r[4] * betas[2] + r[7] * betas[3];
            A[4 * i + 2] = r[3] * betas[0] + r[4] * betas[1] + 2 * r[5] * betas[2] + r[8] * betas[3];
            A[4 * i + 3] = r[6] * betas[0] + r[7] * betas[1] + r[8] * betas[2] + 2 * r[9] * betas[3];
            b[i] = rho[i] - (r[0] * betas[0] * betas[0] + r[1] * betas[0] * betas[1] + r[2] * betas[1] * betas[1] +
                             r[3] * betas[0] * betas[2] + r[4] * betas[1] * betas[2] + r[5] * betas[2] * betas[2] +
                             r[6] * betas[0] * betas[3] + r[7] * betas[1] * betas[3] + r[8] * betas[2] * betas[3] +
                             r[9] * betas[3] * betas[3]);
        }
        qr_solve(A, 6, 4, b, x);
        for (int i = 0; i < 4; i++) betas[i] += x[i];
    }
}

static double compute_R_and_t(epnp_t* e, const double* ut, const double* betas, double R[9], double t[3])
{
    int n = e->n;
    for (int i = 0; i < 4; i++) e->ccs[i][0] = e->ccs[i][1] = e->ccs[i][2] = 0.0;
    for (int i = 0; i < 4; i++) {
        const double* v = ut + 12 * (11 - i);
        for (int j = 0; j < 4; j++)
            for (int k = 0; k < 3; k++) e->ccs[j][k] += betas[i] * v[3 * j + k];
    }
    for (int i = 0; i < n; i++) {
        double* a = e->alphas + 4 * i;
        double* pc = e->pcs + 3 * i;
        for (int j = 0; j < 3; j++)
            pc[j] = a[0] * e->ccs[0][j] + a[1] * e->ccs[1][j] + a[2] * e->ccs[2][j] + a[3] * e->ccs[3][j];
    }
    if (e->pcs[2] < 0.0) { /* solve_for_sign */
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 3; j++) e->ccs[i][j] = -e->ccs[i][j];
        for (int i = 0; i < 3 * n; i++) e->pcs[i] = -e->pcs[i];
    }
    /* estimate_R_and_t */
    double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
    for (int i = 0; i < n; i++)
        for (int j = 0; j < 3; j++) { pc0[j] += e->pcs[3 * i + j]; pw0[j] += e->pws[3 * i + j]; }
    for (int j = 0; j < 3; j++) { pc0[j] /= n; pw0[j] /= n; }
    double abt[9] = {0};
    for (int i = 0; i < n; i++) {
        double* pc = e->pcs + 3 * i;
        double* pw = e->pws + 3 * i;
        for (int j = 0; j < 3; j++) {
            abt[3 * j] += (pc[j] - pc0[j]) * (pw[0] - pw0[0]);
            abt[3 * j + 1] += (pc[j] - pc0[j]) * (pw[1] - pw0[1]);
            abt[3 * j + 2] += (pc[j] - pc0[j]) * (pw[2] - pw0[2]);
        }
    }
    /* cvSVD(&ABt, &D, &U, &V, CV_SVD_MODIFY_A); R[i][j] = dot(U row i, V row j) */
    double w[3], u[9], vt[9];
    ora_cv_svd(abt, 3, 3, w, u, vt);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            R[3 * i + j] = u[3 * i + 0] * vt[0 * 3 + j] + u[3 * i + 1] * vt[1 * 3 + j] + u[3 * i + 2] * vt[2 * 3 + j];
    double det = R[0] * R[4] * R[8] + R[1] * R[5] * R[6] + R[2] * R[3] * R[7] - R[2] * R[4] * R[6] -
                 R[1] * R[3] * R[8] - R[0] * R[5] * R[7];
    if (det < 0) { R[6] = -R[6]; R[7] = -R[7]; R[8] = -R[8]; }
    t[0] = pc0[0] - dot3(R + 0, pw0);
    t[1] = pc0[1] - dot3(R + 3, pw0);
    t[2] = pc0[2] - dot3(R + 6, pw0);
    /* reprojection_error */
    double sum2 = 0.0;
    for (int i = 0; i < n; i++) {
        double* pw = e->pws + 3 * i;
        double Xc = dot3(R + 0, pw) + t[0];
        double Yc = dot3(R + 3, pw) + t[1];
        double inv_Zc = 1.0 / (dot3(R + 6, pw) + t[2]);
        double ue = e->uc + e->fu * Xc * inv_Zc;
        double ve = e->vc + e->fv * Yc * inv_Zc;
        double uu = e->us[2 * i], vv = e->us[2 * i + 1];
        sum2 += sqrt((uu - ue) * (uu - ue) + (vv - ve) * (vv - ve));
    }
    return sum2 / n;
}

/* solvePnP(SOLVEPNP_EPNP): undistortPoints (zero distortion: x = (u-cx)*(1/fx))
 * then epnp re-projects with fu/uc -> us = x*fu + uc. */
int svo_oracle_epnp(const float* obj, const float* img, int n, const double K[9], double R[9], double t[3])
{
    if (n < 4) return -1;
    epnp_t e;
    e.n = n;
    e.fu = K[0]; e.fv = K[4]; e.uc = K[2]; e.vc = K[5];
    double ifx = 1. / K[0], ify = 1. / K[4];
    e.pws = (double*)malloc(sizeof(double) * 3 * n);
    e.us = (double*)malloc(sizeof(double) * 2 * n);
    e.alphas = (double*)malloc(sizeof(double) * 4 * n);
    e.pcs = (double*)malloc(sizeof(double) * 3 * n);
    for (int i = 0; i < n; i++) {
        e.pws[3 * i] = obj[3 * i]; e.pws[3 * i + 1] = obj[3 * i + 1]; e.pws[3 * i + 2] = obj[3 * i + 2];
        /* undistortPoints of CV_32FC2 points writes CV_32FC2 */
        float x = (float)(((double)img[2 * i] - K[2]) * ifx), y = (float)(((double)img[2 * i + 1] - K[5]) * ify);
        e.us[2 * i] = (double)x * e.fu + e.uc;
        e.us[2 * i + 1] = (double)y * e.fv + e.vc;
    }
    choose_control_points(&e);
    compute_barycentric(&e);
    double* M = (double*)calloc((size_t)2 * n * 12, sizeof(double));
    for (int i = 0; i < n; i++) {
        double* M1 = M + (size_t)2 * i * 12;
        double* M2 = M1 + 12;
        const double* as = e.alphas + 4 * i;
        double u = e.us[2 * i], v = e.us[2 * i + 1];
        for (int k = 0; k < 4; k++) {
            M1[3 * k] = as[k] * e.fu; M1[3 * k + 1] = 0.0; M1[3 * k + 2] = as[k] * (e.uc - u);
            M2[3 * k] = 0.0; M2[3 * k + 1] = as[k] * e.fv; M2[3 * k + 2] = as[k] * (e.vc - v);
        }
    }
    double mtm[144], d[12], ut[144];
    ora_mul_transposed(M, 2 * n, 12, mtm); /* cvMulTransposed(M, &MtM, 1) */
    free(M);
    ora_cv_svd_ut(mtm, 12, d, ut);         /* cvSVD(&MtM, &D, &Ut, 0, MODIFY_A | U_T) */
    double L[60], rho[6];
    compute_L_6x10(ut, L);
    rho[0] = dist2(e.cws[0], e.cws[1]); rho[1] = dist2(e.cws[0], e.cws[2]); rho[2] = dist2(e.cws[0], e.cws[3]);
    rho[3] = dist2(e.cws[1], e.cws[2]); rho[4] = dist2(e.cws[1], e.cws[3]); rho[5] = dist2(e.cws[2], e.cws[3]);
    double Betas[4][4] = {{0}}, rep[4] = {0}, Rs[4][9], ts[4][3];
    find_betas_1(L, rho, Betas[1]);
    gauss_newton(L, rho, Betas[1]);
    rep[1] = compute_R_and_t(&e, ut, Betas[1], Rs[1], ts[1]);
    find_betas_2(L, rho, Betas[2]); gauss_newton(L, rho, Betas[2]);
    rep[2] = compute_R_and_t(&e, ut, Betas[2], Rs[2], ts[2]);
    find_betas_3(L, rho, Betas[3]); gauss_newton(L, rho, Betas[3]);
    rep[3] = compute_R_and_t(&e, ut, Betas[3], Rs[3], ts[3]);
    int N = 1;
    if (rep[2] < rep[1]) N = 2;
    if (rep[3] < rep[N]) N = 3;
    memcpy(R, Rs[N], sizeof(double) * 9);
    memcpy(t, ts[N], sizeof(double) * 3);
    free(e.pws); free(e.us); free(e.alphas); free(e.pcs);
    for (int i = 0; i < 9; i++) if (!isfinite(R[i])) return -2;
    for (int i = 0; i < 3; i++) if (!isfinite(t[i])) return -2;
    return 0;
}

int svo_oracle_ransac_update_num_iters(double p, double ep, int modelPoints, int maxIters)
{
    p = p > 0. ? p : 0.;
    p = p < 1. ? p : 1.;
    ep = ep > 0. ? ep : 0.;
    ep = ep < 1. ? ep : 1.;
    double num = (1. - p) > DBL_MIN ? (1. - p) : DBL_MIN;
    double denom = 1. - pow(1. - ep, modelPoints);
    if (denom < DBL_MIN) return 0;
    num = log(num);
    denom = log(denom);
    return denom >= 0 || -num >= maxIters * (-denom) ? maxIters : ora_round_d(num / denom);
}

int svo_oracle_solve_pnp_ransac(const double* obj_d, const float* img, int n, const double K[9],
                                int iterations, float reproj_err, double confidence,
                                double rvec[3], double tvec[3], uint8_t* inlier_mask,
                                int* n_inliers, int* n_hyp_out)
{
    if (n < 4) return -1;
    const int modelPoints = 5;
    /* opoints (Point3d) are converted to CV_32F inside solvePnPRansac */
    float* obj = (float*)malloc(sizeof(float) * 3 * n);
    for (int i = 0; i < 3 * n; i++) obj[i] = (float)obj_d[i];
    int result = 0, nh = 0;
    double bestR[9], bestt[3], best_rv[3] = {0, 0, 0};
    uint8_t* best = (uint8_t*)calloc((size_t)n, 1);
    uint8_t* cur = (uint8_t*)calloc((size_t)n, 1);
    int maxGood = 0;
    if (n <= modelPoints) {
        /* model_points == npoints: solvePnP(EPnP) on all, everything inlier
         * (n == 4 uses P3P in OpenCV; EPnP here -- see DESIGN.md) */
        if (svo_oracle_epnp(obj, img, n, K, bestR, bestt) == 0) {
            svo_oracle_rodrigues_inv(bestR, rvec);
            memcpy(tvec, bestt, sizeof(bestt));
            for (int i = 0; i < n; i++) inlier_mask[i] = 1;
            if (n_inliers) *n_inliers = n;
            result = 1;
        }
        if (n_hyp_out) *n_hyp_out = 1;
        free(obj); free(best); free(cur);
        return result;
    }
    uint64_t rng = 0xFFFFFFFFFFFFFFFFULL;
    int niters = iterations > 1 ? iterations : 1;
    float thr = (float)((double)reproj_err * (double)reproj_err);
    for (int iter = 0; iter < niters; iter++) {
        int idx[5];
        svo_oracle_get_subset(&rng, n, modelPoints, idx);
        float so[15], si[10];
        for (int k = 0; k < 5; k++) {
            memcpy(so + 3 * k, obj + 3 * idx[k], sizeof(float) * 3);
            memcpy(si + 2 * k, img + 2 * idx[k], sizeof(float) * 2);
        }
        double R[9], t[3], rv[3], hyp[12];
        nh++;
        if (svo_oracle_epnp(so, si, 5, K, R, t) != 0) continue;
        /* the model is stored as (rvec, tvec); computeError re-expands rvec */
        svo_oracle_rodrigues_inv(R, rv);
        svo_oracle_rodrigues(rv, hyp);
        memcpy(hyp + 9, t, sizeof(t));
        int good = 0;
        svo_oracle_pnp_residuals(obj, img, n, hyp, 1, K, thr, NULL, cur, &good);
        if (good > (maxGood > modelPoints - 1 ? maxGood : modelPoints - 1)) {
            uint8_t* tmp = best; best = cur; cur = tmp;
            memcpy(best_rv, rv, sizeof(rv));
            memcpy(bestR, hyp, sizeof(double) * 9);
            memcpy(bestt, t, sizeof(t));
            maxGood = good;
            niters = svo_oracle_ransac_update_num_iters(confidence, (double)(n - good) / n, modelPoints, niters);
        }
    }
    if (n_hyp_out) *n_hyp_out = nh;
    if (maxGood <= 0) {
        free(obj); free(best); free(cur);
        return 0;
    }
    /* final solvePnP(SQPNP) on the inliers (float-rounded points widened back) */
    int ni = 0;
    double* pw = (double*)malloc(sizeof(double) * 3 * n);
    double* q = (double*)malloc(sizeof(double) * 2 * n);
    double ifx = 1. / K[0], ify = 1. / K[4];
    for (int i = 0; i < n; i++) {
        if (!best[i]) continue;
        pw[3 * ni] = obj[3 * i]; pw[3 * ni + 1] = obj[3 * i + 1]; pw[3 * ni + 2] = obj[3 * i + 2];
        q[2 * ni] = ((double)img[2 * i] - K[2]) * ifx;
        q[2 * ni + 1] = ((double)img[2 * i + 1] - K[5]) * ify;
        ni++;
    }
    double Rf[9], tf[3];
    if (svo_oracle_sqpnp(pw, q, ni, Rf, tf) == 0) {
        svo_oracle_rodrigues_inv(Rf, rvec);
        memcpy(tvec, tf, sizeof(tf));
    } else {  /* solvePnP would throw; keep the RANSAC model */
        memcpy(rvec, best_rv, sizeof(best_rv));
        memcpy(tvec, bestt, sizeof(bestt));
    }
    memcpy(inlier_mask, best, (size_t)n);
    if (n_inliers) *n_inliers = maxGood;
    free(pw); free(q); free(obj); free(best); free(cur);
    return 1;
}
