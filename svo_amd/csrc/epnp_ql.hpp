// The round-3 EPnP minimal solver (tred2 / tql2 eigen-decomposition of M^T M,
// Householder least squares for the betas), kept as the host twin of the
// device solver epnp_wave.hpp, which mirrors it bit for bit
// (svo_epnp_subsets(device = 2); test_gpu_parity.py::test_epnp_wave_matches_host).
// The front end's RANSAC uses epnp.hpp (OpenCV's Jacobi SVDs, bit-identical to
// the oracle): the QL basis of the 5-point M^T M's two-dimensional null space
// differs from the Jacobi one, and Gauss-Newton can end in another optimum from
// it.
#pragma once

#include "epnp.hpp"
#include "linalg.hpp"

namespace svo {


// EPnP (Lepetit, Moreno-Noguer, Fua) as OpenCV's calib3d/src/epnp.cpp computes it:
// 4 control points (centroid + PCA), barycentric alphas, M^T M null space (4
// smallest eigenvectors), beta approximations 1/2/3 + 5 Gauss-Newton steps
// (Householder QR), R/t by Procrustes, best of the three by mean reprojection.
// Fixed capacity kMaxPts points (the RANSAC subsets and the direct n <= 5 case),
// no allocation: the same code runs on the host and in the GPU RANSAC kernel.
class EPnPQL {
   public:
    static constexpr int kMaxPts = 5;
    SVO_HD EPnPQL(double fu, double fv, double uc, double vc) : fu_(fu), fv_(fv), uc_(uc), vc_(vc) {}

    // pw: n (<= kMaxPts) world points; uv: n pixels. Returns false on non-finite output.
    SVO_HD bool solve(const double* pw, const double* uv, int n, double R[9], double t[3]) {
        if (n > kMaxPts) return false;
        n_ = n;
        pw_ = pw;
        uv_ = uv;
        for (int i = 0; i < 4 * n; i++) alphas_[i] = 0.0;
        for (int i = 0; i < 3 * n; i++) pcs_[i] = 0.0;
        control_points();
        barycentric();
        double MtM[144] = {0};
        for (int i = 0; i < n; i++) {
            const double* a = &alphas_[4 * i];
            const double u = uv[2 * i], v = uv[2 * i + 1];
            double r1[12], r2[12];
            for (int k = 0; k < 4; k++) {
                r1[3 * k] = a[k] * fu_;
                r1[3 * k + 1] = 0.0;
                r1[3 * k + 2] = a[k] * (uc_ - u);
                r2[3 * k] = 0.0;
                r2[3 * k + 1] = a[k] * fv_;
                r2[3 * k + 2] = a[k] * (vc_ - v);
            }
            for (int p = 0; p < 12; p++)
                for (int q = 0; q < 12; q++) MtM[p * 12 + q] += r1[p] * r1[q] + r2[p] * r2[q];
        }
        double ev[12], ut[144];
        la::sym_eig_ql(MtM, 12, ev, ut);
        double L[60], rho[6];
        make_L(ut, L);
        const int pairs[6][2] = {{0, 1}, {0, 2}, {0, 3}, {1, 2}, {1, 3}, {2, 3}};
        for (int i = 0; i < 6; i++) {
            const double* a = cws_[pairs[i][0]];
            const double* b = cws_[pairs[i][1]];
            rho[i] = (a[0] - b[0]) * (a[0] - b[0]) + (a[1] - b[1]) * (a[1] - b[1]) + (a[2] - b[2]) * (a[2] - b[2]);
        }
        double betas[4][4] = {{0}}, err[4] = {0}, Rs[4][9], ts[4][3];
        for (int k = 1; k <= 3; k++) betas_approx(k, L, rho, betas[k]);
        gauss_newton3(L, rho, betas);
        r_and_t3(ut, betas, Rs, ts, err);
        int N = 1;
        if (err[2] < err[1]) N = 2;
        if (err[3] < err[N]) N = 3;
        for (int i = 0; i < 9; i++) R[i] = Rs[N][i];
        for (int i = 0; i < 3; i++) t[i] = ts[N][i];
        // x - x == 0 fails exactly for NaN / inf
        for (int i = 0; i < 9; i++)
            if (!(R[i] - R[i] == 0.0)) return false;
        for (int i = 0; i < 3; i++)
            if (!(t[i] - t[i] == 0.0)) return false;
        return true;
    }

   private:
    SVO_HD void control_points() {
        double c0[3] = {0, 0, 0};
        for (int i = 0; i < n_; i++)
            for (int j = 0; j < 3; j++) c0[j] += pw_[3 * i + j];
        for (int j = 0; j < 3; j++) c0[j] /= n_;
        double C[9] = {0};
        for (int i = 0; i < n_; i++) {
            double d[3] = {pw_[3 * i] - c0[0], pw_[3 * i + 1] - c0[1], pw_[3 * i + 2] - c0[2]};
            for (int a = 0; a < 3; a++)
                for (int b = 0; b < 3; b++) C[a * 3 + b] += d[a] * d[b];
        }
        double w[3], V[9];
        la::sym_eig(C, 3, w, V);
        for (int j = 0; j < 3; j++) cws_[0][j] = c0[j];
        for (int i = 1; i < 4; i++) {
            const double k = sqrt((w[i - 1] > 0 ? w[i - 1] : 0.0) / n_);
            for (int j = 0; j < 3; j++) cws_[i][j] = c0[j] + k * V[3 * (i - 1) + j];
        }
    }
    SVO_HD void barycentric() {
        double CC[9], CI[9];
        for (int i = 0; i < 3; i++)
            for (int j = 1; j < 4; j++) CC[3 * i + j - 1] = cws_[j][i] - cws_[0][i];
        la::pinv3(CC, CI);
        for (int i = 0; i < n_; i++) {
            const double* p = pw_ + 3 * i;
            double* a = &alphas_[4 * i];
            const double d[3] = {p[0] - cws_[0][0], p[1] - cws_[0][1], p[2] - cws_[0][2]};
            for (int j = 0; j < 3; j++) a[1 + j] = CI[3 * j] * d[0] + CI[3 * j + 1] * d[1] + CI[3 * j + 2] * d[2];
            a[0] = 1.0 - a[1] - a[2] - a[3];
        }
    }
    SVO_HD static void make_L(const double* ut, double* L) {
        const double* v[4] = {ut + 12 * 11, ut + 12 * 10, ut + 12 * 9, ut + 12 * 8};
        double dv[4][6][3];
        for (int i = 0; i < 4; i++) {
            int a = 0, b = 1;
            for (int j = 0; j < 6; j++) {
                for (int k = 0; k < 3; k++) dv[i][j][k] = v[i][3 * a + k] - v[i][3 * b + k];
                if (++b > 3) {
                    a++;
                    b = a + 1;
                }
            }
        }
        for (int i = 0; i < 6; i++) {
            double* r = L + 10 * i;
            r[0] = dot3(dv[0][i], dv[0][i]);
            r[1] = 2.0 * dot3(dv[0][i], dv[1][i]);
            r[2] = dot3(dv[1][i], dv[1][i]);
            r[3] = 2.0 * dot3(dv[0][i], dv[2][i]);
            r[4] = 2.0 * dot3(dv[1][i], dv[2][i]);
            r[5] = dot3(dv[2][i], dv[2][i]);
            r[6] = 2.0 * dot3(dv[0][i], dv[3][i]);
            r[7] = 2.0 * dot3(dv[1][i], dv[3][i]);
            r[8] = 2.0 * dot3(dv[2][i], dv[3][i]);
            r[9] = dot3(dv[3][i], dv[3][i]);
        }
    }
    // The 6 x {4, 3, 5} least-squares systems are solved by Householder QR
    // (qr_solve, as the Gauss-Newton steps): OpenCV solves them by SVD
    // (cvSolve(CV_SVD)); for these full-rank systems both give the unique
    // least-squares solution up to rounding, which the 5 Gauss-Newton steps then
    // refine (measured: the same models as an SVD solve on 600 RANSAC subsets,
    // same speed; the device solver, epnp_wave.hpp, mirrors this one bit for bit).
    template <int NC>
    SVO_HD static void lstsq_qr(const double* A, const double* rho, double* x) {
        double Aq[6 * NC], bq[6];
        for (int i = 0; i < 6 * NC; i++) Aq[i] = A[i];
        for (int i = 0; i < 6; i++) bq[i] = rho[i];
        qr_solve<6, NC>(Aq, bq, x);
    }
    // approximations 2 (NC = 3) and 3 (NC = 5): the first NC columns of L
    template <int NC>
    SVO_HD static void lstsq_L(const double* L, const double* rho, double* x) {
        double A[6 * NC];
        for (int i = 0; i < 6; i++)
            for (int k = 0; k < NC; k++) A[NC * i + k] = L[10 * i + k];
        lstsq_qr<NC>(A, rho, x);
    }
    SVO_HD static void betas_approx(int which, const double* L, const double* rho, double* b) {
        static const int cols1[4] = {0, 1, 3, 6};
        double x[5];
        if (which == 1) {
            double A[24];
            for (int i = 0; i < 6; i++)
                for (int k = 0; k < 4; k++) A[4 * i + k] = L[10 * i + cols1[k]];
            lstsq_qr<4>(A, rho, x);
            const double sg = x[0] < 0 ? -1.0 : 1.0;
            b[0] = sqrt(sg * x[0]);
            b[1] = sg * x[1] / b[0];
            b[2] = sg * x[2] / b[0];
            b[3] = sg * x[3] / b[0];
            return;
        }
        if (which == 2)
            lstsq_L<3>(L, rho, x);
        else
            lstsq_L<5>(L, rho, x);
        if (x[0] < 0) {
            b[0] = sqrt(-x[0]);
            b[1] = (x[2] < 0) ? sqrt(-x[2]) : 0.0;
        } else {
            b[0] = sqrt(x[0]);
            b[1] = (x[2] > 0) ? sqrt(x[2]) : 0.0;
        }
        if (x[1] < 0) b[0] = -b[0];
        b[2] = which == 3 ? x[3] / b[0] : 0.0;
        b[3] = 0.0;
    }
    // nr x nc (compile-time sizes: the loops unroll into registers)
    template <int nr, int nc>
    SVO_HD static void qr_solve(double* A, double* b, double* X) {
        double A1[nc], A2[nc];
        for (int k = 0; k < nc; k++) {
            double eta = 0;
            for (int i = k; i < nr; i++) eta = fmax(eta, fabs(A[i * nc + k]));
            if (eta == 0) {
                for (int j = 0; j < nc; j++) X[j] = 0;
                return;
            }
            double sum2 = 0.0;
            const double ie = 1. / eta;
            for (int i = k; i < nr; i++) {
                A[i * nc + k] *= ie;
                sum2 += A[i * nc + k] * A[i * nc + k];
            }
            double sigma = sqrt(sum2);
            if (A[k * nc + k] < 0) sigma = -sigma;
            A[k * nc + k] += sigma;
            A1[k] = sigma * A[k * nc + k];
            A2[k] = -eta * sigma;
            for (int j = k + 1; j < nc; j++) {
                double s = 0;
                for (int i = k; i < nr; i++) s += A[i * nc + k] * A[i * nc + j];
                const double tau = s / A1[k];
                for (int i = k; i < nr; i++) A[i * nc + j] -= tau * A[i * nc + k];
            }
        }
        for (int j = 0; j < nc; j++) {
            double tau = 0;
            for (int i = j; i < nr; i++) tau += A[i * nc + j] * b[i];
            tau /= A1[j];
            for (int i = j; i < nr; i++) b[i] -= tau * A[i * nc + j];
        }
        X[nc - 1] = b[nc - 1] / A2[nc - 1];
        for (int i = nc - 2; i >= 0; i--) {
            double s = 0;
            for (int j = i + 1; j < nc; j++) s += A[i * nc + j] * X[j];
            X[i] = (b[i] - s) / A2[i];
        }
    }
    // qr_solve of NS independent systems, interleaved column by column (each
    // system's arithmetic and order exactly as qr_solve; the host core overlaps
    // the NS dependency chains of divisions and square roots)
    template <int nr, int nc, int NS>
    SVO_HD static void qr_solve_n(double (*A)[nr * nc], double (*b)[nr], double (*X)[nc]) {
        double A1[NS][nc], A2[NS][nc];
        bool dead[NS];
        for (int q = 0; q < NS; q++) dead[q] = false;
        for (int k = 0; k < nc; k++)
            for (int q = 0; q < NS; q++) {
                if (dead[q]) continue;
                double* a = A[q];
                double eta = 0;
                for (int i = k; i < nr; i++) eta = fmax(eta, fabs(a[i * nc + k]));
                if (eta == 0) {
                    for (int j = 0; j < nc; j++) X[q][j] = 0;
                    dead[q] = true;
                    continue;
                }
                double sum2 = 0.0;
                const double ie = 1. / eta;
                for (int i = k; i < nr; i++) {
                    a[i * nc + k] *= ie;
                    sum2 += a[i * nc + k] * a[i * nc + k];
                }
                double sigma = sqrt(sum2);
                if (a[k * nc + k] < 0) sigma = -sigma;
                a[k * nc + k] += sigma;
                A1[q][k] = sigma * a[k * nc + k];
                A2[q][k] = -eta * sigma;
                for (int j = k + 1; j < nc; j++) {
                    double sj = 0;
                    for (int i = k; i < nr; i++) sj += a[i * nc + k] * a[i * nc + j];
                    const double tau = sj / A1[q][k];
                    for (int i = k; i < nr; i++) a[i * nc + j] -= tau * a[i * nc + k];
                }
            }
        for (int j = 0; j < nc; j++)
            for (int q = 0; q < NS; q++) {
                if (dead[q]) continue;
                double tau = 0;
                for (int i = j; i < nr; i++) tau += A[q][i * nc + j] * b[q][i];
                tau /= A1[q][j];
                for (int i = j; i < nr; i++) b[q][i] -= tau * A[q][i * nc + j];
            }
        for (int q = 0; q < NS; q++)
            if (!dead[q]) X[q][nc - 1] = b[q][nc - 1] / A2[q][nc - 1];
        for (int i = nc - 2; i >= 0; i--)
            for (int q = 0; q < NS; q++) {
                if (dead[q]) continue;
                double sx = 0;
                for (int j = i + 1; j < nc; j++) sx += A[q][i * nc + j] * X[q][j];
                X[q][i] = (b[q][i] - sx) / A2[q][i];
            }
    }
    // gauss_newton of the three approximations (betas[1..3]) in lock step
    SVO_HD static void gauss_newton3(const double* L, const double* rho, double (*betas)[4]) {
        for (int it = 0; it < 5; it++) {
            double A[3][24], b[3][6], x[3][4];
            for (int q = 0; q < 3; q++) {
                const double* be = betas[q + 1];
                for (int i = 0; i < 6; i++) {
                    const double* r = L + 10 * i;
                    A[q][4 * i + 0] = 2 * r[0] * be[0] + r[1] * be[1] + r[3] * be[2] + r[6] * be[3];
                    A[q][4 * i + 1] = r[1] * be[0] + 2 * r[2] * be[1] + r[4] * be[2] + r[7] * be[3];
                    A[q][4 * i + 2] = r[3] * be[0] + r[4] * be[1] + 2 * r[5] * be[2] + r[8] * be[3];
                    A[q][4 * i + 3] = r[6] * be[0] + r[7] * be[1] + r[8] * be[2] + 2 * r[9] * be[3];
                    b[q][i] = rho[i] - (r[0] * be[0] * be[0] + r[1] * be[0] * be[1] + r[2] * be[1] * be[1] +
                                        r[3] * be[0] * be[2] + r[4] * be[1] * be[2] + r[5] * be[2] * be[2] +
                                        r[6] * be[0] * be[3] + r[7] * be[1] * be[3] + r[8] * be[2] * be[3] +
                                        r[9] * be[3] * be[3]);
                }
            }
            qr_solve_n<6, 4, 3>(A, b, x);
            for (int q = 0; q < 3; q++)
                for (int i = 0; i < 4; i++) betas[q + 1][i] += x[q][i];
        }
    }
    SVO_HD static void gauss_newton(const double* L, const double* rho, double* be) {
        for (int it = 0; it < 5; it++) {
            double A[24], b[6], x[4];
            for (int i = 0; i < 6; i++) {
                const double* r = L + 10 * i;
                A[4 * i + 0] = 2 * r[0] * be[0] + r[1] * be[1] + r[3] * be[2] + r[6] * be[3];
                A[4 * i + 1] = r[1] * be[0] + 2 * r[2] * be[1] + r[4] * be[2] + r[7] * be[3];
                A[4 * i + 2] = r[3] * be[0] + r[4] * be[1] + 2 * r[5] * be[2] + r[8] * be[3];
                A[4 * i + 3] = r[6] * be[0] + r[7] * be[1] + r[8] * be[2] + 2 * r[9] * be[3];
                b[i] = rho[i] - (r[0] * be[0] * be[0] + r[1] * be[0] * be[1] + r[2] * be[1] * be[1] +
                                 r[3] * be[0] * be[2] + r[4] * be[1] * be[2] + r[5] * be[2] * be[2] +
                                 r[6] * be[0] * be[3] + r[7] * be[1] * be[3] + r[8] * be[2] * be[3] +
                                 r[9] * be[3] * be[3]);
            }
            qr_solve<6, 4>(A, b, x);
            for (int i = 0; i < 4; i++) be[i] += x[i];
        }
    }
    // r_and_t of the three approximations (betas[1..3] -> Rs / ts / err[1..3]),
    // their Procrustes SVDs in lock step (la::svd3_n); per approximation the same
    // arithmetic in the same order as r_and_t
    SVO_HD void r_and_t3(const double* ut, const double (*betas)[4], double (*Rs)[9], double (*ts)[3], double* err) {
        double pcs[3][3 * kMaxPts], pc0[3][3], pw0[3] = {0, 0, 0}, abt[3][9];
        for (int i = 0; i < n_; i++)
            for (int j = 0; j < 3; j++) pw0[j] += pw_[3 * i + j];
        for (int j = 0; j < 3; j++) pw0[j] /= n_;
        for (int q = 0; q < 3; q++) {
            const double* be = betas[q + 1];
            double ccs[4][3] = {{0}};
            for (int i = 0; i < 4; i++) {
                const double* v = ut + 12 * (11 - i);
                for (int j = 0; j < 4; j++)
                    for (int k = 0; k < 3; k++) ccs[j][k] += be[i] * v[3 * j + k];
            }
            double* P = pcs[q];
            for (int i = 0; i < n_; i++) {
                const double* a = &alphas_[4 * i];
                double* pc = &P[3 * i];
                for (int j = 0; j < 3; j++)
                    pc[j] = a[0] * ccs[0][j] + a[1] * ccs[1][j] + a[2] * ccs[2][j] + a[3] * ccs[3][j];
            }
            if (P[2] < 0.0)
                for (int i = 0; i < 3 * n_; i++) P[i] = -P[i];
            for (int j = 0; j < 3; j++) pc0[q][j] = 0;
            for (int i = 0; i < n_; i++)
                for (int j = 0; j < 3; j++) pc0[q][j] += P[3 * i + j];
            for (int j = 0; j < 3; j++) pc0[q][j] /= n_;
            for (int i = 0; i < 9; i++) abt[q][i] = 0;
            for (int i = 0; i < n_; i++) {
                const double* pc = &P[3 * i];
                const double* pw = pw_ + 3 * i;
                for (int j = 0; j < 3; j++)
                    for (int k = 0; k < 3; k++) abt[q][3 * j + k] += (pc[j] - pc0[q][j]) * (pw[k] - pw0[k]);
            }
        }
        double s[3][3], U[3][9], Vt[3][9];
        la::svd3_n<3>(abt, s, U, Vt);
        for (int q = 0; q < 3; q++) {
            double* R = Rs[q + 1];
            double* t = ts[q + 1];
            const double* u = U[q];
            const double* vt = Vt[q];
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++)
                    R[3 * i + j] = u[3 * i] * vt[j] + u[3 * i + 1] * vt[3 + j] + u[3 * i + 2] * vt[6 + j];
            const double det = R[0] * R[4] * R[8] + R[1] * R[5] * R[6] + R[2] * R[3] * R[7] - R[2] * R[4] * R[6] -
                               R[1] * R[3] * R[8] - R[0] * R[5] * R[7];
            if (det < 0) {
                R[6] = -R[6];
                R[7] = -R[7];
                R[8] = -R[8];
            }
            for (int k = 0; k < 3; k++) t[k] = pc0[q][k] - dot3(R + 3 * k, pw0);
            double sum = 0.0;
            for (int i = 0; i < n_; i++) {
                const double* pw = pw_ + 3 * i;
                const double Xc = dot3(R, pw) + t[0], Yc = dot3(R + 3, pw) + t[1];
                const double iz = 1.0 / (dot3(R + 6, pw) + t[2]);
                const double ue = uc_ + fu_ * Xc * iz, ve = vc_ + fv_ * Yc * iz;
                const double du = uv_[2 * i] - ue, dv = uv_[2 * i + 1] - ve;
                sum += sqrt(du * du + dv * dv);
            }
            err[q + 1] = sum / n_;
        }
    }
    SVO_HD double r_and_t(const double* ut, const double* be, double* R, double* t) {
        double ccs[4][3] = {{0}};
        for (int i = 0; i < 4; i++) {
            const double* v = ut + 12 * (11 - i);
            for (int j = 0; j < 4; j++)
                for (int k = 0; k < 3; k++) ccs[j][k] += be[i] * v[3 * j + k];
        }
        for (int i = 0; i < n_; i++) {
            const double* a = &alphas_[4 * i];
            double* pc = &pcs_[3 * i];
            for (int j = 0; j < 3; j++) pc[j] = a[0] * ccs[0][j] + a[1] * ccs[1][j] + a[2] * ccs[2][j] + a[3] * ccs[3][j];
        }
        if (pcs_[2] < 0.0)
            for (int i = 0; i < 3 * n_; i++) pcs_[i] = -pcs_[i];
        double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
        for (int i = 0; i < n_; i++)
            for (int j = 0; j < 3; j++) {
                pc0[j] += pcs_[3 * i + j];
                pw0[j] += pw_[3 * i + j];
            }
        for (int j = 0; j < 3; j++) {
            pc0[j] /= n_;
            pw0[j] /= n_;
        }
        double abt[9] = {0};
        for (int i = 0; i < n_; i++) {
            const double* pc = &pcs_[3 * i];
            const double* pw = pw_ + 3 * i;
            for (int j = 0; j < 3; j++)
                for (int k = 0; k < 3; k++) abt[3 * j + k] += (pc[j] - pc0[j]) * (pw[k] - pw0[k]);
        }
        double s[3], U[9], Vt[9];
        la::svd(abt, 3, 3, s, U, Vt);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) R[3 * i + j] = U[3 * i] * Vt[j] + U[3 * i + 1] * Vt[3 + j] + U[3 * i + 2] * Vt[6 + j];
        const double det = R[0] * R[4] * R[8] + R[1] * R[5] * R[6] + R[2] * R[3] * R[7] - R[2] * R[4] * R[6] -
                           R[1] * R[3] * R[8] - R[0] * R[5] * R[7];
        if (det < 0) {
            R[6] = -R[6];
            R[7] = -R[7];
            R[8] = -R[8];
        }
        for (int k = 0; k < 3; k++) t[k] = pc0[k] - dot3(R + 3 * k, pw0);
        double sum = 0.0;
        for (int i = 0; i < n_; i++) {
            const double* pw = pw_ + 3 * i;
            const double Xc = dot3(R, pw) + t[0], Yc = dot3(R + 3, pw) + t[1];
            const double iz = 1.0 / (dot3(R + 6, pw) + t[2]);
            const double ue = uc_ + fu_ * Xc * iz, ve = vc_ + fv_ * Yc * iz;
            const double du = uv_[2 * i] - ue, dv = uv_[2 * i + 1] - ve;
            sum += sqrt(du * du + dv * dv);
        }
        return sum / n_;
    }

    double fu_, fv_, uc_, vc_;
    int n_ = 0;
    const double* pw_ = nullptr;
    const double* uv_ = nullptr;
    double cws_[4][3];
    double alphas_[4 * kMaxPts], pcs_[3 * kMaxPts];
};


// solvePnP(EPnP) with the reference's inputs: float object points widened to
// double, pixels normalised by undistortPoints (x = (u - cx) * (1/fx)) and
// re-projected by epnp's init_points (u' = x fu + uc). idx: the subset (or
// null for points 0..n-1); n <= EPnP::kMaxPts.
SVO_HD bool epnp_pixels_ql(const float* obj, const float* img, const int* idx, int n, const double K[9], double R[9],
                        double t[3]) {
    if (n > EPnPQL::kMaxPts) return false;
    double pw[3 * EPnPQL::kMaxPts], uv[2 * EPnPQL::kMaxPts];
    const double ifx = 1. / K[0], ify = 1. / K[4];
    for (int k = 0; k < n; k++) {
        const int i = idx ? idx[k] : k;
        pw[3 * k] = obj[3 * i];
        pw[3 * k + 1] = obj[3 * i + 1];
        pw[3 * k + 2] = obj[3 * i + 2];
        const double x = ((double)img[2 * i] - K[2]) * ifx, y = ((double)img[2 * i + 1] - K[5]) * ify;
        uv[2 * k] = x * K[0] + K[2];
        uv[2 * k + 1] = y * K[4] + K[5];
    }
    EPnPQL e(K[0], K[4], K[2], K[5]);
    return e.solve(pw, uv, n, R, t);
}

}  // namespace svo
