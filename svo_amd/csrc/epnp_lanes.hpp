// The RANSAC minimal solver (EPnP of 5-point subsets, epnp.hpp) for L * G subsets
// at once, one subset per SIMD lane: every step of EPnP::prepare / svd_ut<12> /
// EPnP::finish -- the control points and their 3 x 3 SVD, the alphas (3 x 3
// cv::invert by SVD), M^T M and its 12 x 12 Jacobi SVD, the three beta
// approximations (6 x {4, 3, 5} cv::solve by SVD), the Gauss-Newton steps
// (epnp.cpp's Householder qr_solve, its early return and stale-x reuse kept per
// lane), the three Procrustes fits and the choice among them -- with each lane
// doing the scalar code's operations in the scalar code's order. A branch of the
// scalar code becomes a per-lane select between both sides' values (each side
// computed with the scalar side's operations), and an early exit a lane mask, so
// every lane's pose is bit-identical to epnp_pixels on its subset
// (tests/test_epnp_cpu.py: every instruction-set path against the oracle).
//
// Host only, included by one translation unit per instruction set (epnp_avx2.cpp,
// epnp_avx512.cpp); like simd_svd.hpp, everything is in an anonymous namespace.
#pragma once

#include "epnp.hpp"
#include "simd_svd.hpp"

namespace svo {
namespace {

template <int L>
struct EPnPLanes {
    using V = la::cv::vd<L>;
    using Mk = la::cv::vm<L>;
    static constexpr int n = 5;

    double fu, fv, uc, vc;
    V pw[3 * n], uv[2 * n];
    V cws[4][3], alphas[4 * n];

    static V sel(Mk m, V a, V b) { return la::cv::vsel<L>(m, a, b); }
    static V vsqrt(V x) { return la::cv::vsqrt<L>(x); }
    static V vabs(V x) { return la::cv::vabs<L>(x); }
    static V dot3(const V* a, const V* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

    // la::cv::svd<3> (At = A^T, Jacobi with V, u = At^T)
    static void svd3(const V* A, V* w, V* u, V* vt) {
        V At[1][9], W[1][3], Vt[1][9];
        for (int i = 0; i < 3; i++)
            for (int k = 0; k < 3; k++) At[0][i * 3 + k] = A[k * 3 + i];
        la::cv::jacobi_svd_lanes<3, 3, L, 1, true>(At, W, Vt);
        for (int i = 0; i < 3; i++) w[i] = W[0][i];
        for (int i = 0; i < 9; i++) vt[i] = Vt[0][i];
        for (int k = 0; k < 3; k++)
            for (int i = 0; i < 3; i++) u[k * 3 + i] = At[0][i * 3 + k];
    }

    // la::cv::solve_svd<M, NC> (cv::solve DECOMP_SVD, one right-hand side)
    template <int M, int NC>
    static void solve_svd(const V* A, const V* b, V* x) {
        V At[1][NC * M], Vt[1][NC * NC], w[1][NC];
        for (int i = 0; i < NC; i++)
            for (int k = 0; k < M; k++) At[0][i * M + k] = A[k * NC + i];
        la::cv::jacobi_svd_lanes<M, NC, L, 1, true>(At, w, Vt);
        V threshold = 0;
        for (int j = 0; j < NC; j++) x[j] = 0;
        for (int i = 0; i < NC; i++) threshold += w[0][i];
        threshold *= 2.220446049250313e-16 * 2;
        for (int i = 0; i < NC; i++) {
            const Mk skip = vabs(w[0][i]) <= threshold;
            const V wi = 1 / w[0][i];
            V s = 0;
            for (int j = 0; j < M; j++) s += At[0][i * M + j] * b[j];
            s *= wi;
            for (int j = 0; j < NC; j++) x[j] = sel(skip, x[j], x[j] + s * Vt[0][i * NC + j]);
        }
    }

    // EPnP::control_points (n = 5)
    void control_points() {
        V c0[3] = {0, 0, 0};
        for (int i = 0; i < n; i++)
            for (int j = 0; j < 3; j++) c0[j] += pw[3 * i + j];
        for (int j = 0; j < 3; j++) c0[j] /= n;
        V pw0[3 * n];
        for (int i = 0; i < n; i++)
            for (int j = 0; j < 3; j++) pw0[3 * i + j] = pw[3 * i + j] - c0[j];
        V C[9];
        for (int i = 0; i < 3; i++)
            for (int j = i; j < 3; j++) {
                V s = 0;
                for (int k = 0; k < n; k++) s += pw0[k * 3 + i] * pw0[k * 3 + j];
                C[i * 3 + j] = s;
            }
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < i; j++) C[i * 3 + j] = C[j * 3 + i];
        V At[1][9], w[1][3];  // svd_ut<3>
        for (int i = 0; i < 3; i++)
            for (int k = 0; k < 3; k++) At[0][i * 3 + k] = C[k * 3 + i];
        la::cv::jacobi_svd_lanes<3, 3, L, 1, false>(At, w, nullptr);
        for (int j = 0; j < 3; j++) cws[0][j] = c0[j];
        for (int i = 1; i < 4; i++) {
            const V k = vsqrt(w[0][i - 1] / n);
            for (int j = 0; j < 3; j++) cws[i][j] = c0[j] + k * At[0][3 * (i - 1) + j];
        }
    }

    // EPnP::barycentric: cv::invert(CC, DECOMP_SVD), then the alphas
    void barycentric() {
        V CC[9], CI[9], w[3], u[9], vt[9], buf[3];
        for (int i = 0; i < 3; i++)
            for (int j = 1; j < 4; j++) CC[3 * i + j - 1] = cws[j][i] - cws[0][i];
        svd3(CC, w, u, vt);
        V threshold = 0;
        for (int i = 0; i < 9; i++) CI[i] = 0;
        for (int i = 0; i < 3; i++) threshold += w[i];
        threshold *= 2.220446049250313e-16 * 2;
        for (int i = 0; i < 3; i++) {
            const Mk skip = vabs(w[i]) <= threshold;
            const V wi = 1 / w[i];
            for (int j = 0; j < 3; j++) buf[j] = u[j * 3 + i] * wi;
            for (int r = 0; r < 3; r++) {
                const V sv = vt[i * 3 + r];
                for (int j = 0; j < 3; j++) CI[r * 3 + j] = sel(skip, CI[r * 3 + j], CI[r * 3 + j] + sv * buf[j]);
            }
        }
        for (int i = 0; i < n; i++) {
            const V* p = pw + 3 * i;
            V* a = &alphas[4 * i];
            const V d[3] = {p[0] - cws[0][0], p[1] - cws[0][1], p[2] - cws[0][2]};
            for (int j = 0; j < 3; j++) a[1 + j] = CI[3 * j] * d[0] + CI[3 * j + 1] * d[1] + CI[3 * j + 2] * d[2];
            a[0] = 1.0 - a[1] - a[2] - a[3];
        }
    }

    // EPnP::prepare: M^T M (12 x 12) of the 10 x 12 M
    void prepare(V* MtM) {
        control_points();
        barycentric();
        V Mm[2 * n * 12];
        for (int i = 0; i < n; i++) {
            const V* a = &alphas[4 * i];
            const V u = uv[2 * i], v = uv[2 * i + 1];
            V* r1 = Mm + 24 * i;
            V* r2 = r1 + 12;
            for (int k = 0; k < 4; k++) {
                r1[3 * k] = a[k] * fu;
                r1[3 * k + 1] = 0.0;
                r1[3 * k + 2] = a[k] * (uc - u);
                r2[3 * k] = 0.0;
                r2[3 * k + 1] = a[k] * fv;
                r2[3 * k + 2] = a[k] * (vc - v);
            }
        }
        for (int i = 0; i < 12; i++)
            for (int j = i; j < 12; j++) {
                V s = 0;
                for (int k = 0; k < 2 * n; k++) s += Mm[k * 12 + i] * Mm[k * 12 + j];
                MtM[i * 12 + j] = s;
            }
        for (int i = 0; i < 12; i++)
            for (int j = 0; j < i; j++) MtM[i * 12 + j] = MtM[j * 12 + i];
    }

    static void make_L(const V* ut, V* Lm) {
        const V* v[4] = {ut + 12 * 11, ut + 12 * 10, ut + 12 * 9, ut + 12 * 8};
        V dv[4][6][3];
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
            V* r = Lm + 10 * i;
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

    // EPnP::betas_approx
    static void betas_approx(int which, const V* Lm, const V* rho, V* b) {
        static const int cols1[4] = {0, 1, 3, 6};
        V x[5];
        if (which == 1) {
            V A[24];
            for (int i = 0; i < 6; i++)
                for (int k = 0; k < 4; k++) A[4 * i + k] = Lm[10 * i + cols1[k]];
            solve_svd<6, 4>(A, rho, x);
            const V sg = sel(x[0] < 0, V(-1.0), V(1.0));
            b[0] = vsqrt(sg * x[0]);
            b[1] = sg * x[1] / b[0];
            b[2] = sg * x[2] / b[0];
            b[3] = sg * x[3] / b[0];
            return;
        }
        if (which == 2) {
            V A[18];
            for (int i = 0; i < 6; i++)
                for (int k = 0; k < 3; k++) A[3 * i + k] = Lm[10 * i + k];
            solve_svd<6, 3>(A, rho, x);
        } else {
            V A[30];
            for (int i = 0; i < 6; i++)
                for (int k = 0; k < 5; k++) A[5 * i + k] = Lm[10 * i + k];
            solve_svd<6, 5>(A, rho, x);
        }
        const Mk neg = x[0] < 0;
        b[0] = sel(neg, vsqrt(-x[0]), vsqrt(x[0]));
        b[1] = sel(neg, sel(x[2] < 0, vsqrt(-x[2]), V(0.0)), sel(x[2] > 0, vsqrt(x[2]), V(0.0)));
        b[0] = sel(x[1] < 0, -b[0], b[0]);
        b[2] = which == 3 ? x[3] / b[0] : V(0.0);
        b[3] = 0.0;
    }

    // EPnP::qr_solve<6, 4>: a lane whose column scale is zero leaves X as it was
    static void qr_solve(V* A, V* b, V* X) {
        constexpr int nr = 6, nc = 4;
        V A1[nc], A2[nc];
        Mk dead = Mk(0);
        for (int k = 0; k < nc; k++) {
            V eta = vabs(A[k * nc + k]);
            for (int i = k + 1; i < nr; i++) eta = __builtin_elementwise_max(eta, vabs(A[(i - 1) * nc + k]));
            dead |= eta == 0;
            V sum2 = 0.0;
            const V ie = 1. / eta;
            for (int i = k; i < nr; i++) {
                A[i * nc + k] *= ie;
                sum2 += A[i * nc + k] * A[i * nc + k];
            }
            V sigma = vsqrt(sum2);
            sigma = sel(A[k * nc + k] < 0, -sigma, sigma);
            A[k * nc + k] += sigma;
            A1[k] = sigma * A[k * nc + k];
            A2[k] = -eta * sigma;
            for (int j = k + 1; j < nc; j++) {
                V s = 0;
                for (int i = k; i < nr; i++) s += A[i * nc + k] * A[i * nc + j];
                const V tau = s / A1[k];
                for (int i = k; i < nr; i++) A[i * nc + j] -= tau * A[i * nc + k];
            }
        }
        for (int j = 0; j < nc; j++) {
            V tau = 0;
            for (int i = j; i < nr; i++) tau += A[i * nc + j] * b[i];
            tau /= A1[j];
            for (int i = j; i < nr; i++) b[i] -= tau * A[i * nc + j];
        }
        V Xn[nc];
        Xn[nc - 1] = b[nc - 1] / A2[nc - 1];
        for (int i = nc - 2; i >= 0; i--) {
            V s = 0;
            for (int j = i + 1; j < nc; j++) s += A[i * nc + j] * Xn[j];
            Xn[i] = (b[i] - s) / A2[i];
        }
        for (int i = 0; i < nc; i++) X[i] = sel(dead, X[i], Xn[i]);
    }

    // EPnP::gauss_newton3: five steps of each approximation, x kept across steps
    static void gauss_newton3(const V* Lm, const V* rho, V (*betas)[4]) {
        V x[3][4];
        for (int q = 0; q < 3; q++)
            for (int i = 0; i < 4; i++) x[q][i] = 0;
        for (int it = 0; it < 5; it++)
            for (int q = 0; q < 3; q++) {
                V A[24], b[6];
                const V* be = betas[q + 1];
                for (int i = 0; i < 6; i++) {
                    const V* r = Lm + 10 * i;
                    A[4 * i + 0] = 2 * r[0] * be[0] + r[1] * be[1] + r[3] * be[2] + r[6] * be[3];
                    A[4 * i + 1] = r[1] * be[0] + 2 * r[2] * be[1] + r[4] * be[2] + r[7] * be[3];
                    A[4 * i + 2] = r[3] * be[0] + r[4] * be[1] + 2 * r[5] * be[2] + r[8] * be[3];
                    A[4 * i + 3] = r[6] * be[0] + r[7] * be[1] + r[8] * be[2] + 2 * r[9] * be[3];
                    b[i] = rho[i] - (r[0] * be[0] * be[0] + r[1] * be[0] * be[1] + r[2] * be[1] * be[1] +
                                     r[3] * be[0] * be[2] + r[4] * be[1] * be[2] + r[5] * be[2] * be[2] +
                                     r[6] * be[0] * be[3] + r[7] * be[1] * be[3] + r[8] * be[2] * be[3] +
                                     r[9] * be[3] * be[3]);
                }
                qr_solve(A, b, x[q]);
                for (int i = 0; i < 4; i++) betas[q + 1][i] += x[q][i];
            }
    }

    // EPnP::r_and_t3: R, t and the mean reprojection error of approximation q
    void r_and_t(const V* ut, const V* be, V* R, V* t, V& err) const {
        V pw0[3] = {0, 0, 0};
        for (int i = 0; i < n; i++)
            for (int j = 0; j < 3; j++) pw0[j] += pw[3 * i + j];
        for (int j = 0; j < 3; j++) pw0[j] /= n;
        V ccs[4][3];
        for (int j = 0; j < 4; j++)
            for (int k = 0; k < 3; k++) ccs[j][k] = 0;
        for (int i = 0; i < 4; i++) {
            const V* v = ut + 12 * (11 - i);
            for (int j = 0; j < 4; j++)
                for (int k = 0; k < 3; k++) ccs[j][k] += be[i] * v[3 * j + k];
        }
        V P[3 * n], pc0[3], abt[9];
        for (int i = 0; i < n; i++) {
            const V* a = &alphas[4 * i];
            for (int j = 0; j < 3; j++)
                P[3 * i + j] = a[0] * ccs[0][j] + a[1] * ccs[1][j] + a[2] * ccs[2][j] + a[3] * ccs[3][j];
        }
        const Mk flip = P[2] < 0.0;
        for (int i = 0; i < 3 * n; i++) P[i] = sel(flip, -P[i], P[i]);
        for (int j = 0; j < 3; j++) pc0[j] = 0;
        for (int i = 0; i < n; i++)
            for (int j = 0; j < 3; j++) pc0[j] += P[3 * i + j];
        for (int j = 0; j < 3; j++) pc0[j] /= n;
        for (int i = 0; i < 9; i++) abt[i] = 0;
        for (int i = 0; i < n; i++) {
            const V* pc = &P[3 * i];
            const V* p = pw + 3 * i;
            for (int j = 0; j < 3; j++)
                for (int k = 0; k < 3; k++) abt[3 * j + k] += (pc[j] - pc0[j]) * (p[k] - pw0[k]);
        }
        V s[3], u[9], vt[9];
        svd3(abt, s, u, vt);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++)
                R[3 * i + j] = u[3 * i] * vt[j] + u[3 * i + 1] * vt[3 + j] + u[3 * i + 2] * vt[6 + j];
        const V det = R[0] * R[4] * R[8] + R[1] * R[5] * R[6] + R[2] * R[3] * R[7] - R[2] * R[4] * R[6] -
                      R[1] * R[3] * R[8] - R[0] * R[5] * R[7];
        const Mk mirror = det < 0;
        for (int k = 6; k < 9; k++) R[k] = sel(mirror, -R[k], R[k]);
        for (int k = 0; k < 3; k++) t[k] = pc0[k] - dot3(R + 3 * k, pw0);
        V sum = 0.0;
        for (int i = 0; i < n; i++) {
            const V* p = pw + 3 * i;
            const V Xc = dot3(R, p) + t[0], Yc = dot3(R + 3, p) + t[1];
            const V iz = 1.0 / (dot3(R + 6, p) + t[2]);
            const V ue = uc + fu * Xc * iz, ve = vc + fv * Yc * iz;
            const V du = uv[2 * i] - ue, dv = uv[2 * i + 1] - ve;
            sum += vsqrt(du * du + dv * dv);
        }
        err = sum / n;
    }

    // EPnP::finish: returns the lanes with a finite model
    Mk finish(const V* ut, V* R, V* t) const {
        V Lm[60], rho[6];
        make_L(ut, Lm);
        const int pairs[6][2] = {{0, 1}, {0, 2}, {0, 3}, {1, 2}, {1, 3}, {2, 3}};
        for (int i = 0; i < 6; i++) {
            const V* a = cws[pairs[i][0]];
            const V* b = cws[pairs[i][1]];
            rho[i] = (a[0] - b[0]) * (a[0] - b[0]) + (a[1] - b[1]) * (a[1] - b[1]) + (a[2] - b[2]) * (a[2] - b[2]);
        }
        V betas[4][4];
        for (int k = 1; k <= 3; k++) betas_approx(k, Lm, rho, betas[k]);
        gauss_newton3(Lm, rho, betas);
        V Rs[4][9], ts[4][3], err[4];
        for (int q = 1; q <= 3; q++) r_and_t(ut, betas[q], Rs[q], ts[q], err[q]);
        const Mk two = err[2] < err[1];
        const Mk three = err[3] < sel(two, err[2], err[1]);
        Mk fin = Mk(-1);
        for (int i = 0; i < 9; i++) {
            R[i] = sel(three, Rs[3][i], sel(two, Rs[2][i], Rs[1][i]));
            fin &= R[i] - R[i] == 0.0;
        }
        for (int i = 0; i < 3; i++) {
            t[i] = sel(three, ts[3][i], sel(two, ts[2][i], ts[1][i]));
            fin &= t[i] - t[i] == 0.0;
        }
        return fin;
    }
};

// epnp_pixels of count <= L * G 5-point subsets (obj[q] / img[q], points idx[q]
// or 0..4); lanes past count repeat subset 0. Bit-identical to epnp_pixels.
template <int L, int G>
inline void epnp_lanes(int count, const float* const* obj, const float* const* img, const int* const* idx,
                       const double K[9], double (*R)[9], double (*t)[3], bool* ok) {
    using V = la::cv::vd<L>;
    constexpr int n = EPnPLanes<L>::n;
    EPnPLanes<L> e[G];
    V At[G][144], W[G][12];
    for (int g = 0; g < G; g++) {
        EPnPLanes<L>& es = e[g];
        es.fu = K[0];
        es.fv = K[4];
        es.uc = K[2];
        es.vc = K[5];
        for (int l = 0; l < L; l++) {
            int q = g * L + l;
            if (q >= count) q = 0;
            double pw[3 * n], uv[2 * n];
            epnp_inputs(obj[q], img[q], idx[q], n, K, pw, uv);
            for (int i = 0; i < 3 * n; i++) es.pw[i][l] = pw[i];
            for (int i = 0; i < 2 * n; i++) es.uv[i][l] = uv[i];
        }
        V MtM[144];
        es.prepare(MtM);
        for (int i = 0; i < 12; i++)  // svd_ut<12>: At = MtM^T
            for (int k = 0; k < 12; k++) At[g][i * 12 + k] = MtM[k * 12 + i];
    }
    la::cv::jacobi_svd_lanes<12, 12, L, G, false>(At, W, nullptr);
    for (int g = 0; g < G; g++) {
        V Rv[9], tv[3];
        const auto fin = e[g].finish(At[g], Rv, tv);
        for (int l = 0; l < L; l++) {
            const int q = g * L + l;
            if (q >= count) break;
            for (int i = 0; i < 9; i++) R[q][i] = Rv[i][l];
            for (int i = 0; i < 3; i++) t[q][i] = tv[i][l];
            ok[q] = fin[l] != 0;
        }
    }
}

}  // namespace
}  // namespace svo
