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
#include "epnp.hpp"
#include "linalg.hpp"
#include "pose.hpp"

namespace svo {

namespace {


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
    samp = nullptr;
    nsamp = 0;
}

// chunk schedule first, 8, 16, 16, ...: first defaults to 2 (below ~1 % outliers
// RANSACUpdateNumIters (p 0.999, 5 points) brings niters down to 2 after the first
// accepted hypothesis, below ~0.6 % to 1, so one round suffices); above, round 2
// covers up to 10
static int chunk_size(int rounds, int first) {
    if (rounds == 0) return first > 0 ? (first < kRansacChunk ? first : kRansacChunk) : 2;
    return rounds == 1 ? 8 : kRansacChunk;
}

int RansacSeq::predict_iters(double confidence, double ep, int max_iters) {
    return update_num_iters(confidence, ep, 5, max_iters);
}

int RansacSeq::next_end() const {
    if (done || direct) return nh;
    const int sched = chunk_size(rounds, first_chunk);
    return nh + ((niters - iter) < sched ? (niters - iter) : sched);
}

int RansacSeq::gen_chunk(const double K[9]) {
    m = 0;
    if (done || direct) return 0;
    const int sched = chunk_size(rounds, first_chunk);
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
        const int h = nh + j;
        if (h < nsamp) {  // the same 5 points, gathered on the device in draw order
            const float* sp = samp + (size_t)kSampleFloats * h;
            valid[j] = epnp_pixels(sp, sp + 15, nullptr, 5, K, Rj, tj);
        } else {
            valid[j] = epnp_pixels(obj, img, idx, 5, K, Rj, tj);
        }
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
