// Pose update: cv::solvePnPRansac(..., SOLVEPNP_SQPNP) as the reference calls it
// at R:src/tracking.cpp:191-196, with the hypothesis scoring on the GPU.
//
//   RANSAC stage (calib3d/src/ptsetreg.cpp RANSACPointSetRegistrator::run):
//     cv::RNG(uint64 -1) MWC; 5-point subsets drawn with duplicate redraw
//     (getSubset); minimal kernel EPnP (solvePnPRansac picks EPnP for SQPNP);
//     model kept as (rvec, tvec); accept iff inliers > max(best, 4);
//     niters = RANSACUpdateNumIters(confidence, outlier ratio, 5, niters).
//   Scoring: svo_pnp_residuals kernel (projectPoints + findInliers, bit-exact).
//   The RNG draws do not depend on the scores, so hypotheses are generated and
//   scored in chunks; the accept rule is then replayed in iteration order, and
//   iterations past the (shrinking) niters are discarded -- identical result
//   to the serial loop.
//   Final fit (solvePnP SQPNP on the inliers): minimiser of SQPnP's object-space
//   cost r^T Omega r over SO(3) (multi-start Gauss-Newton), see DESIGN.md.
#include <cfloat>
#include <cstring>
#include <vector>

#include "common.hpp"
#include "linalg.hpp"
#include "pose.hpp"

namespace svo {

namespace {


inline double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

// EPnP (Lepetit, Moreno-Noguer, Fua) as OpenCV's calib3d/src/epnp.cpp computes it:
// 4 control points (centroid + PCA), barycentric alphas, M^T M null space (4
// smallest eigenvectors), beta approximations 1/2/3 + 5 Gauss-Newton steps
// (Householder QR), R/t by Procrustes, best of the three by mean reprojection.
class EPnP {
   public:
    EPnP(double fu, double fv, double uc, double vc) : fu_(fu), fv_(fv), uc_(uc), vc_(vc) {}

    // pw: n world points; uv: n pixels. Returns false on non-finite output.
    bool solve(const double* pw, const double* uv, int n, double R[9], double t[3]) {
        n_ = n;
        pw_ = pw;
        uv_ = uv;
        alphas_.assign(4 * (size_t)n, 0.0);
        pcs_.assign(3 * (size_t)n, 0.0);
        control_points();
        barycentric();
        double MtM[144] = {0};
        for (int i = 0; i < n; i++) {
            const double* a = &alphas_[4 * (size_t)i];
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
        for (int k = 1; k <= 3; k++) {
            betas_approx(k, L, rho, betas[k]);
            gauss_newton(L, rho, betas[k]);
            err[k] = r_and_t(ut, betas[k], Rs[k], ts[k]);
        }
        int N = 1;
        if (err[2] < err[1]) N = 2;
        if (err[3] < err[N]) N = 3;
        std::memcpy(R, Rs[N], sizeof(double) * 9);
        std::memcpy(t, ts[N], sizeof(double) * 3);
        for (int i = 0; i < 9; i++)
            if (!std::isfinite(R[i])) return false;
        for (int i = 0; i < 3; i++)
            if (!std::isfinite(t[i])) return false;
        return true;
    }

   private:
    void control_points() {
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
    void barycentric() {
        double CC[9], CI[9];
        for (int i = 0; i < 3; i++)
            for (int j = 1; j < 4; j++) CC[3 * i + j - 1] = cws_[j][i] - cws_[0][i];
        la::pinv3(CC, CI);
        for (int i = 0; i < n_; i++) {
            const double* p = pw_ + 3 * i;
            double* a = &alphas_[4 * (size_t)i];
            const double d[3] = {p[0] - cws_[0][0], p[1] - cws_[0][1], p[2] - cws_[0][2]};
            for (int j = 0; j < 3; j++) a[1 + j] = CI[3 * j] * d[0] + CI[3 * j + 1] * d[1] + CI[3 * j + 2] * d[2];
            a[0] = 1.0 - a[1] - a[2] - a[3];
        }
    }
    static void make_L(const double* ut, double* L) {
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
    static void betas_approx(int which, const double* L, const double* rho, double* b) {
        static const int cols1[4] = {0, 1, 3, 6};
        double A[30], x[5];
        if (which == 1) {
            for (int i = 0; i < 6; i++)
                for (int k = 0; k < 4; k++) A[4 * i + k] = L[10 * i + cols1[k]];
            la::lstsq(A, 6, 4, rho, x);
            const double sg = x[0] < 0 ? -1.0 : 1.0;
            b[0] = sqrt(sg * x[0]);
            b[1] = sg * x[1] / b[0];
            b[2] = sg * x[2] / b[0];
            b[3] = sg * x[3] / b[0];
            return;
        }
        const int nc = which == 2 ? 3 : 5;
        for (int i = 0; i < 6; i++)
            for (int k = 0; k < nc; k++) A[nc * i + k] = L[10 * i + k];
        la::lstsq(A, 6, nc, rho, x);
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
    static void qr_solve(double* A, int nr, int nc, double* b, double* X) {
        double A1[8], A2[8];
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
    static void gauss_newton(const double* L, const double* rho, double* be) {
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
            qr_solve(A, 6, 4, b, x);
            for (int i = 0; i < 4; i++) be[i] += x[i];
        }
    }
    double r_and_t(const double* ut, const double* be, double* R, double* t) {
        double ccs[4][3] = {{0}};
        for (int i = 0; i < 4; i++) {
            const double* v = ut + 12 * (11 - i);
            for (int j = 0; j < 4; j++)
                for (int k = 0; k < 3; k++) ccs[j][k] += be[i] * v[3 * j + k];
        }
        for (int i = 0; i < n_; i++) {
            const double* a = &alphas_[4 * (size_t)i];
            double* pc = &pcs_[3 * (size_t)i];
            for (int j = 0; j < 3; j++) pc[j] = a[0] * ccs[0][j] + a[1] * ccs[1][j] + a[2] * ccs[2][j] + a[3] * ccs[3][j];
        }
        if (pcs_[2] < 0.0)
            for (auto& v : pcs_) v = -v;
        double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
        for (int i = 0; i < n_; i++)
            for (int j = 0; j < 3; j++) {
                pc0[j] += pcs_[3 * (size_t)i + j];
                pw0[j] += pw_[3 * i + j];
            }
        for (int j = 0; j < 3; j++) {
            pc0[j] /= n_;
            pw0[j] /= n_;
        }
        double abt[9] = {0};
        for (int i = 0; i < n_; i++) {
            const double* pc = &pcs_[3 * (size_t)i];
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
    std::vector<double> alphas_, pcs_;
};

// solvePnP(EPnP) with the reference's inputs: float object points widened to
// double, pixels normalised by undistortPoints (x = (u - cx) * (1/fx)) and
// re-projected by epnp's init_points (u' = x fu + uc).
bool epnp_pixels(const float* obj, const float* img, const int* idx, int n, const double K[9], double R[9],
                 double t[3]) {
    std::vector<double> pw(3 * (size_t)n), uv(2 * (size_t)n);
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
    EPnP e(K[0], K[4], K[2], K[5]);
    return e.solve(pw.data(), uv.data(), n, R, t);
}

int update_num_iters(double p, double ep, int model_points, int max_iters) {
    p = p > 0. ? (p < 1. ? p : 1.) : 0.;
    ep = ep > 0. ? (ep < 1. ? ep : 1.) : 0.;
    double num = (1. - p) > DBL_MIN ? (1. - p) : DBL_MIN;
    double denom = 1. - pow(1. - ep, model_points);
    if (denom < DBL_MIN) return 0;
    num = log(num);
    denom = log(denom);
    return denom >= 0 || -num >= max_iters * (-denom) ? max_iters : (int)rint(num / denom);
}

// ---- final fit: SQPnP's object-space cost, E(R) = vec(R)^T Omega vec(R) ----
struct SqpnpCost {
    double Om[81];
    double P[27];  // t = P vec(R)
};

// Omega = sum_i (B_i + P)^T A_i (B_i + P) with A_i = I - v v^T / v^T v,
// B_i vec(R) = R p_i, P = -Q^-1 S: expanded through the sufficient statistics
// Q = sum A_i, S = sum A_i B_i, M = sum B_i^T A_i B_i as Omega = M - S^T Q^-1 S
// (one pass, ~130 flops per point).
}  // namespace

// The 60 sufficient statistics of one point set: Q = sum A_i (6 unique),
// T[u][j] = sum A_i,u p_j (18), U[u][v] = sum A_i,u (p p^T)_v (36); A_i as
// symmetric 6-vectors. Host twin of pnp.hip's suffstats kernel.
void sqpnp_sums(const double* pw, const double* q, int n, double* sums) {
    double Qs[6] = {0}, T[6][3] = {{0}}, U[6][6] = {{0}};
    for (int i = 0; i < n; i++) {
        const double x = q[2 * i], y = q[2 * i + 1];
        const double in = 1.0 / (x * x + y * y + 1.0);
        const double As[6] = {1.0 - x * x * in, -x * y * in, -x * in, 1.0 - y * y * in, -y * in, 1.0 - in};
        const double* p = pw + 3 * (size_t)i;
        const double pp[6] = {p[0] * p[0], p[0] * p[1], p[0] * p[2], p[1] * p[1], p[1] * p[2], p[2] * p[2]};
        for (int u = 0; u < 6; u++) {
            Qs[u] += As[u];
            T[u][0] += As[u] * p[0];
            T[u][1] += As[u] * p[1];
            T[u][2] += As[u] * p[2];
            for (int v = 0; v < 6; v++) U[u][v] += As[u] * pp[v];
        }
    }
    std::memcpy(sums, Qs, sizeof(Qs));
    std::memcpy(sums + 6, T, sizeof(T));
    std::memcpy(sums + 24, U, sizeof(U));
}

namespace {

// Omega = sum_i (B_i + P)^T A_i (B_i + P) with A_i = I - v v^T / v^T v,
// B_i vec(R) = R p_i, P = -Q^-1 S, assembled from the sufficient statistics
// as Omega = M - S^T Q^-1 S.
void sqpnp_assemble(const double* sums, SqpnpCost& c) {
    static const int IDX[3][3] = {{0, 1, 2}, {1, 3, 4}, {2, 4, 5}};  // unique entries of a sym 3x3
    const double* Qs = sums;
    auto T = [&](int u, int j) { return sums[6 + 3 * u + j]; };
    auto U = [&](int u, int v) { return sums[24 + 6 * u + v]; };
    double Q[9], S[27], Qi[9];
    for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) Q[3 * a + b] = Qs[IDX[a][b]];
    for (int a = 0; a < 3; a++)
        for (int r = 0; r < 3; r++)
            for (int j = 0; j < 3; j++) S[9 * a + 3 * r + j] = T(IDX[a][r], j);
    la::pinv3(Q, Qi);
    for (int a = 0; a < 3; a++)
        for (int col = 0; col < 9; col++)
            c.P[9 * a + col] = -(Qi[3 * a] * S[col] + Qi[3 * a + 1] * S[9 + col] + Qi[3 * a + 2] * S[18 + col]);
    for (int r = 0; r < 3; r++)
        for (int j = 0; j < 3; j++)
            for (int s2 = 0; s2 < 3; s2++)
                for (int k = 0; k < 3; k++) {
                    // M[(r,j),(s,k)] = sum A_rs p_j p_k ; minus (S^T Qi S) = + S^T P
                    const double m = U(IDX[r][s2], IDX[j][k]);
                    const int R = 3 * r + j, Cc = 3 * s2 + k;
                    double stp = S[R] * c.P[Cc] + S[9 + R] * c.P[9 + Cc] + S[18 + R] * c.P[18 + Cc];
                    c.Om[9 * R + Cc] = m + stp;
                }
    for (int r = 0; r < 9; r++)  // symmetrise
        for (int col = 0; col < r; col++) {
            const double v = 0.5 * (c.Om[9 * r + col] + c.Om[9 * col + r]);
            c.Om[9 * r + col] = c.Om[9 * col + r] = v;
        }
}

double quad(const double* Om, const double* r) {
    double s = 0;
    for (int i = 0; i < 9; i++) {
        double t = 0;
        for (int j = 0; j < 9; j++) t += Om[9 * i + j] * r[j];
        s += r[i] * t;
    }
    return s;
}

double refine_so3(const double* Om, double* R) {
    for (int it = 0; it < 100; it++) {
        double J[27];  // d vec(exp([w]) R) / dw at 0: columns vec(G_k R)
        for (int k = 0; k < 3; k++) {
            double G[9] = {0};
            if (k == 0) { G[5] = -1; G[7] = 1; }
            if (k == 1) { G[2] = 1; G[6] = -1; }
            if (k == 2) { G[1] = -1; G[3] = 1; }
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++) J[3 * (3 * i + j) + k] = G[3 * i] * R[j] + G[3 * i + 1] * R[3 + j] + G[3 * i + 2] * R[6 + j];
        }
        double g[3] = {0, 0, 0}, H[9] = {0};
        for (int i = 0; i < 9; i++) {
            double Or = 0, OJ[3] = {0, 0, 0};
            for (int j = 0; j < 9; j++) {
                Or += Om[9 * i + j] * R[j];
                for (int k = 0; k < 3; k++) OJ[k] += Om[9 * i + j] * J[3 * j + k];
            }
            for (int a = 0; a < 3; a++) {
                g[a] += J[3 * i + a] * Or;
                for (int b = 0; b < 3; b++) H[3 * a + b] += J[3 * i + a] * OJ[b];
            }
        }
        double Hi[9];
        la::pinv3(H, Hi);
        double w[3];
        for (int a = 0; a < 3; a++) w[a] = -(Hi[3 * a] * g[0] + Hi[3 * a + 1] * g[1] + Hi[3 * a + 2] * g[2]);
        double dR[9], Rn[9];
        la::rodrigues(w, dR);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) Rn[3 * i + j] = dR[3 * i] * R[j] + dR[3 * i + 1] * R[3 + j] + dR[3 * i + 2] * R[6 + j];
        if (quad(Om, Rn) > quad(Om, R)) break;
        std::memcpy(R, Rn, sizeof(Rn));
        if (w[0] * w[0] + w[1] * w[1] + w[2] * w[2] < 1e-24) break;
    }
    return quad(Om, R);
}

// Minimiser of r^T Omega r over SO(3): Gauss-Newton from the RANSAC rotation
// and from the nearest rotations of Omega's two smallest eigenvectors (both
// signs); the lowest-cost start whose solution puts at least half the inliers
// in front of the camera wins (SQPnP's cheirality test).
void fit_from_cost(const SqpnpCost& c, const float* obj, const std::vector<int>& inl, const double R0[9],
                   double R[9], double t[3]) {
    const int n = (int)inl.size();
    double Oc[81], ev[9], evec[81];
    std::memcpy(Oc, c.Om, sizeof(Oc));
    la::sym_eig_ql(Oc, 9, ev, evec);
    double starts[5][9], Es[5], ts[5][3];
    std::memcpy(starts[0], R0, sizeof(double) * 9);
    for (int s = 0; s < 4; s++) {
        const double* e = evec + 9 * (8 - (s >> 1));
        double M[9];
        for (int k = 0; k < 9; k++) M[k] = ((s & 1) ? -1.0 : 1.0) * e[k];
        la::nearest_rotation(M, starts[s + 1]);
    }
    for (int s = 0; s < 5; s++) {
        Es[s] = refine_so3(c.Om, starts[s]);
        for (int a = 0; a < 3; a++) {
            ts[s][a] = 0;
            for (int col = 0; col < 9; col++) ts[s][a] += c.P[9 * a + col] * starts[s][col];
        }
    }
    // candidates in cost order (ties: start order), first cheirality pass wins
    int ord[5] = {0, 1, 2, 3, 4};
    for (int i = 1; i < 5; i++)
        for (int j = i; j > 0 && Es[ord[j]] < Es[ord[j - 1]]; j--) std::swap(ord[j], ord[j - 1]);
    for (int k = 0; k < 5; k++) {
        const int s = ord[k];
        const double* cand = starts[s];
        int pos = 0;
        for (int i : inl) {
            const double p[3] = {obj[3 * i], obj[3 * i + 1], obj[3 * i + 2]};
            pos += dot3(cand + 6, p) + ts[s][2] > 0;
        }
        if (2 * pos < n) continue;
        std::memcpy(R, cand, sizeof(double) * 9);
        std::memcpy(t, ts[s], sizeof(double) * 3);
        return;
    }
    std::memcpy(R, R0, sizeof(double) * 9);
    for (int a = 0; a < 3; a++) {
        t[a] = 0;
        for (int col = 0; col < 9; col++) t[a] += c.P[9 * a + col] * R0[col];
    }
}

}  // namespace

// ---- resumable per-sequence RANSAC (batched GPU scoring between chunks) ----
void RansacSeq::begin(const float* o, const float* im, int npts, int iterations) {
    obj = o;
    img = im;
    n = npts;
    rng = 0xFFFFFFFFFFFFFFFFULL;
    niters = iterations > 1 ? iterations : 1;
    iter = 0;
    maxGood = 0;
    nh = 0;
    m = 0;
    rounds = 0;
    best.assign((size_t)(n + 31) / 32, 0u);
    for (int i = 0; i < 9; i++) bestR[i] = (i % 4 == 0) ? 1.0 : 0.0;
    direct = n <= 5;
    done = n < 4;
    ok = false;
}

int RansacSeq::gen_chunk(const double K[9]) {
    m = 0;
    if (done || direct) return 0;
    // chunk schedule 2, 8, 16, 16, ...: below ~1 % outliers RANSACUpdateNumIters
    // (p 0.999, 5 points) brings niters down to 2 after the first accepted
    // hypothesis, so one round suffices; above, round 2 covers up to 10
    const int sched = rounds == 0 ? 2 : rounds == 1 ? 8 : kRansacChunk;
    const int want = (niters - iter) < sched ? (niters - iter) : sched;
    rounds++;
    Rng r{rng};
    for (int j = 0; j < want; j++) {
        int idx[5];
        for (int i = 0; i < 5; i++) {
            int v;
            bool dup;
            do {
                v = r.uniform(0, n);
                dup = false;
                for (int k = 0; k < i; k++) dup |= idx[k] == v;
            } while (dup);
            idx[i] = v;
        }
        double Rj[9], tj[3], rv[3];
        valid[j] = epnp_pixels(obj, img, idx, 5, K, Rj, tj);
        double* hp = hyp + 12 * j;
        if (valid[j]) {
            la::rodrigues_inv(Rj, rv);  // the model is stored as (rvec, tvec)
            la::rodrigues(rv, hp);
            std::memcpy(hp + 9, tj, sizeof(tj));
        } else {
            for (int k = 0; k < 12; k++) hp[k] = 0;
        }
    }
    rng = r.state;
    m = want;
    nh += want;
    return want;
}

void RansacSeq::consume(const int* counts, const uint32_t* bits, int words_cap, double confidence) {
    const int words = (n + 31) / 32;
    for (int j = 0; j < m && iter < niters; j++, iter++) {
        const int good = valid[j] ? counts[j] : 0;
        if (good > (maxGood > 4 ? maxGood : 4)) {
            std::memcpy(best.data(), bits + (size_t)words_cap * j, sizeof(uint32_t) * words);
            std::memcpy(bestR, hyp + 12 * j, sizeof(double) * 9);
            maxGood = good;
            niters = update_num_iters(confidence, (double)(n - good) / n, 5, niters);
        }
    }
    m = 0;
    if (iter >= niters) done = true;
}

void RansacSeq::select(const double K[9], bool list) {
    inliers.clear();
    ok = false;
    fitted = false;
    if (n < 4) return;
    if (direct) {
        double R[9], t[3];
        if (!epnp_pixels(obj, img, nullptr, n, K, R, t)) return;
        la::rodrigues_inv(R, rvec);
        std::memcpy(tvec, t, sizeof(t));
        for (int i = 0; i < n; i++) inliers.push_back(i);
        for (int i = 0; i < n; i++) best[i >> 5] |= 1u << (i & 31);
        maxGood = n;
        ok = true;
        fitted = true;
        return;
    }
    if (maxGood <= 0) return;
    if (list)
        for (int i = 0; i < n; i++)
            if ((best[i >> 5] >> (i & 31)) & 1) inliers.push_back(i);
    ok = true;
}

// Normalised image coordinates and world points of the inliers (as doubles).
static void inlier_arrays(const float* obj, const float* img, const std::vector<int>& inl, const double K[9],
                          std::vector<double>& pw, std::vector<double>& q) {
    const int n = (int)inl.size();
    pw.resize(3 * (size_t)n);
    q.resize(2 * (size_t)n);
    const double ifx = 1. / K[0], ify = 1. / K[4];
    for (int k = 0; k < n; k++) {
        const int i = inl[k];
        for (int j = 0; j < 3; j++) pw[3 * k + j] = obj[3 * i + j];
        q[2 * k] = ((double)img[2 * i] - K[2]) * ifx;
        q[2 * k + 1] = ((double)img[2 * i + 1] - K[5]) * ify;
    }
}

void RansacSeq::fit(const double K[9], const double* sums) {
    if (!ok || fitted) return;
    if (inliers.empty())  // select(..., false) left the list to here
        for (int i = 0; i < n; i++)
            if ((best[i >> 5] >> (i & 31)) & 1) inliers.push_back(i);
    double own[60];
    if (!sums) {
        std::vector<double> pw, q;
        inlier_arrays(obj, img, inliers, K, pw, q);
        sqpnp_sums(pw.data(), q.data(), (int)inliers.size(), own);
        sums = own;
    }
    SqpnpCost c;
    sqpnp_assemble(sums, c);
    double Rf[9], tf[3];
    fit_from_cost(c, obj, inliers, bestR, Rf, tf);
    la::rodrigues_inv(Rf, rvec);
    std::memcpy(tvec, tf, sizeof(tf));
    fitted = true;
}

void RansacSeq::finish(const double K[9]) {
    select(K);
    fit(K, nullptr);
}

}  // namespace svo

extern "C" int svo_solve_pnp_ransac(svo_ctx* ctx, const double* obj_xyz, const float* img_xy, int n,
                                    const double K[9], int iterations, float reproj_err, double confidence,
                                    double rvec[3], double tvec[3], int* inliers, int* n_inliers) {
    using namespace svo;
    if (!ctx || !K || !rvec || !tvec || n < 0 || (n > 0 && (!obj_xyz || !img_xy)))
        return set_error(ctx, SVO_ERR_ARG, "svo_solve_pnp_ransac: bad arguments");
    if (n < 4) return set_error(ctx, SVO_ERR_ARG, "solvePnPRansac: npoints >= 4 required (CV_Assert)");
    if (!(confidence > 0 && confidence < 1)) return set_error(ctx, SVO_ERR_ARG, "confidence in (0,1)");
    std::vector<float> obj(3 * (size_t)n);
    for (size_t i = 0; i < obj.size(); i++) obj[i] = (float)obj_xyz[i];  // Point3d -> CV_32F
    const int words = (n + 31) / 32;
    const size_t dbytes = sizeof(float) * 5 * (size_t)n + sizeof(double) * 12 * kRansacChunk +
                          sizeof(int) * kRansacChunk + sizeof(uint32_t) * (size_t)words * kRansacChunk + 1024;
    char* d = (char*)scratch(ctx, 5, dbytes);
    char* h = (char*)pinned(ctx, sizeof(int) * kRansacChunk + sizeof(uint32_t) * (size_t)words * kRansacChunk +
                                     sizeof(double) * 12 * kRansacChunk + 256);
    if (!d || !h) return set_error(ctx, SVO_ERR_HIP, "scratch alloc");
    double* dh = (double*)d;
    int* dcnt = (int*)(dh + 12 * kRansacChunk);
    uint32_t* dbits = (uint32_t*)(dcnt + kRansacChunk);
    float* dobj = (float*)(dbits + (size_t)words * kRansacChunk);
    float* dimg = dobj + 3 * (size_t)n;
    double* hh = (double*)h;
    int* hcnt = (int*)(hh + 12 * kRansacChunk);
    uint32_t* hbits = (uint32_t*)(hcnt + kRansacChunk);
    SVO_HIP(ctx, hipMemcpyAsync(dobj, obj.data(), sizeof(float) * 3 * n, hipMemcpyHostToDevice, ctx->stream));
    SVO_HIP(ctx, hipMemcpyAsync(dimg, img_xy, sizeof(float) * 2 * n, hipMemcpyHostToDevice, ctx->stream));
    const float thr = (float)((double)reproj_err * (double)reproj_err);
    RansacSeq rs;
    rs.begin(obj.data(), img_xy, n, iterations);
    while (!rs.done && !rs.direct) {
        const int m = rs.gen_chunk(K);
        if (m == 0) break;
        std::memcpy(hh, rs.hyp, sizeof(double) * 12 * m);
        SVO_HIP(ctx, hipMemcpyAsync(dh, hh, sizeof(double) * 12 * m, hipMemcpyHostToDevice, ctx->stream));
        PnpBatch b{dobj, dimg, nullptr, n, n, dh, m, nullptr, dbits, words, dcnt};
        SVO_HIP(ctx, launch_pnp_residuals(b, 1, n, K[0], K[4], K[2], K[5], thr, ctx->stream));
        SVO_HIP(ctx, hipMemcpyAsync(hcnt, dcnt, sizeof(int) * m, hipMemcpyDeviceToHost, ctx->stream));
        SVO_HIP(ctx, hipMemcpyAsync(hbits, dbits, sizeof(uint32_t) * (size_t)words * m, hipMemcpyDeviceToHost,
                                    ctx->stream));
        SVO_HIP(ctx, hipStreamSynchronize(ctx->stream));
        rs.consume(hcnt, hbits, words, confidence);
    }
    rs.finish(K);
    if (!rs.ok) {
        if (n_inliers) *n_inliers = 0;
        return 0;
    }
    std::memcpy(rvec, rs.rvec, sizeof(rs.rvec));
    std::memcpy(tvec, rs.tvec, sizeof(rs.tvec));
    if (inliers)
        for (size_t i = 0; i < rs.inliers.size(); i++) inliers[i] = rs.inliers[i];
    if (n_inliers) *n_inliers = (int)rs.inliers.size();
    return 1;
}
