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
//   Final fit (solvePnP SQPNP on the inliers, calib3d/src/sqpnp.cpp): SQPnP's
//   cost r^T Omega r -- Omega as PoseSolver::computeOmega builds it (the
//   algebraic image-space error [1 0 -x; 0 1 -y](R X + t) with t eliminated,
//   t = P r), from statistics summed on the GPU -- and its solution search over
//   Omega's eigenvectors with the same SQP runs (15 steps at most: an unconverged
//   run can win, as in OpenCV).
#include <cfloat>
#include <cstring>
#include <vector>

#include "common.hpp"
#include "epnp.hpp"
#include "simd_svd.hpp"
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

// ---- final fit: SQPnP's cost, E(R) = vec(R)^T Omega vec(R) ----
struct SqpnpCost {
    double Om[81];
    double P[27];    // t = P vec(R)
    double mean[3];  // object-point mean (PoseSolver::positiveDepth)
    bool ok;         // computeOmega's asserts held (point variance, rank)
};
}  // namespace

// The sufficient statistics of one point set (pose.hpp); host twin of pnp.hip's
// suffstats kernel (same per-point arithmetic, same order within a point).
void sqpnp_sums(const double* pw, const double* q, int n, double* sums) {
    std::memset(sums, 0, sizeof(double) * kSqpnpStats);
    for (int i = 0; i < n; i++) {
        const double x = q[2 * i], y = q[2 * i + 1], sq = x * x + y * y;
        const double* p = pw + 3 * (size_t)i;
        const double pp[6] = {p[0] * p[0], p[0] * p[1], p[0] * p[2], p[1] * p[1], p[1] * p[2], p[2] * p[2]};
        const double c[4] = {1.0, x, y, sq};
        sums[0] += 1.0;
        sums[1] += x;
        sums[2] += y;
        sums[3] += sq;
        for (int u = 0; u < 4; u++) {
            for (int j = 0; j < 3; j++) sums[4 + 3 * u + j] += c[u] * p[j];
            for (int v = 0; v < 6; v++) sums[16 + 6 * u + v] += c[u] * pp[v];
        }
    }
}

namespace {

// PoseSolver::computeOmega from the statistics: Omega_raw = sum B_i^T A_i^T A_i
// B_i (blocks XX^T, -x XX^T, -y XX^T, (x^2+y^2) XX^T), qa = sum A_i^T A_i B_i,
// Q = sum A_i^T A_i, P = -Q^-1 qa, Omega = Omega_raw + qa^T P; ok = false where
// SQPnP asserts on the points (their variance below 1e-5); Omega's own asserts
// (largest singular value below 1e-7, more than 6 null vectors) are checked on
// its eigenvalues in fit_from_cost.
void sqpnp_assemble(const double* sums, SqpnpCost& c) {
    static const int IDX[3][3] = {{0, 1, 2}, {1, 3, 4}, {2, 4, 5}};  // unique entries of a sym 3x3
    const double n = sums[0], sx = sums[1], sy = sums[2], ssq = sums[3];
    auto SX = [&](int u, int j) { return sums[4 + 3 * u + j]; };           // sum c_u X_j
    auto SXX = [&](int u, int a, int b) { return sums[16 + 6 * u + IDX[a][b]]; };  // sum c_u X_a X_b
    double Om[81] = {0}, qa[27] = {0};
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
    la::pinv3(Q, Qi);
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

double quad(const double* Om, const double* r) {
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
void sqp_step(const double* Om, const double* r, double* delta) {
    constexpr int N = 15;
    double A[N][N + 1] = {{0}};
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
    double J[6][9] = {{0}};
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
            for (int j = 0; j <= N; j++) std::swap(A[col][j], A[piv][j]);
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
    std::memcpy(delta, x, sizeof(double) * 9);
}

// PoseSolver::runSQP: at most 15 steps while |delta|^2 > 1e-10; then -r if
// det < 0, and the nearest rotation only if det > 1.001 (r as is otherwise --
// its cost and t are taken unprojected, as OpenCV does).
void sqp_run(const double* Om, const double* r0, double* rhat) {
    double r[9], delta[9];
    std::memcpy(r, r0, sizeof(r));
    double dsq = DBL_MAX;
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
        for (double& v : r) v = -v;
        d = -d;
    }
    if (d > 1.001)
        la::nearest_rotation(r, rhat);
    else
        std::memcpy(rhat, r, sizeof(r));
}

// SQPnP's solution search (PoseSolver::solveInternal) over Omega's eigenvectors:
//   the null-space eigenvectors e (eigenvalues below the rank tolerance 1e-7; at
//   least the smallest), sqrt(3)-scaled: if e is already orthogonal (squared
//   orthogonality error < 1e-8) it is taken as is, det-signed, with t = P e (no
//   refinement -- OpenCV's shortcut); else runs from the nearest rotations of +e
//   and -e; then further eigenvectors while the best error exceeds 3x their
//   eigenvalue. checkSolution: the object-point mean in front of the camera or a
//   majority of positive depths; errors within 1e-6 and rotations within 1e-10
//   are one solution; the first smallest-error solution is solvePnP's.
struct SqSol {
    double r[9], t[3], err;
};

double ortho_err(const double* e) {
    const double n1 = e[0] * e[0] + e[1] * e[1] + e[2] * e[2], n2 = e[3] * e[3] + e[4] * e[4] + e[5] * e[5],
                 n3 = e[6] * e[6] + e[7] * e[7] + e[8] * e[8];
    const double d12 = e[0] * e[3] + e[1] * e[4] + e[2] * e[5], d13 = e[0] * e[6] + e[1] * e[7] + e[2] * e[8],
                 d23 = e[3] * e[6] + e[4] * e[7] + e[5] * e[8];
    return (n1 - 1) * (n1 - 1) + (n2 - 1) * (n2 - 1) + (n3 - 1) * (n3 - 1) + 2 * (d12 * d12 + d13 * d13 + d23 * d23);
}

double det33(const double* m) {
    return m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6]) + m[2] * (m[3] * m[7] - m[4] * m[6]);
}

// pt(k, p): object point k of the n fitted points into p[3]. *found: false when
// SQPnP asserts on Omega (CV_Assert(s_(0) >= 1e-7): its largest eigenvalue --
// Omega is symmetric PSD, its singular values are its eigenvalues -- and at most 6
// null vectors, as oracle/sqpnp.c) or finds no solution in front of the camera.
template <class PointAt>
void fit_from_cost(const SqpnpCost& c, int n, PointAt pt, double R[9], double t[3], bool* found) {
    double Oc[81], ev[9], evec[81];
    std::memcpy(Oc, c.Om, sizeof(Oc));
    la::sym_eig_ql(Oc, 9, ev, evec);  // descending; eigenvector k in row k
    *found = false;
    if (!(ev[0] >= 1e-7)) return;
    int nn = 0;
    while (7 - nn >= 0 && ev[7 - nn] < 1e-7) nn++;
    if (++nn > 6) return;
    std::vector<SqSol> sols;
    double min_err = DBL_MAX;
    auto check = [&](SqSol& s) {
        for (int a = 0; a < 3; a++) {
            s.t[a] = 0;
            for (int col = 0; col < 9; col++) s.t[a] += c.P[9 * a + col] * s.r[col];
        }
        bool front = dot3(s.r + 6, c.mean) + s.t[2] > 0;
        if (!front) {
            int pos = 0;
            for (int k = 0; k < n; k++) {
                double p[3];
                pt(k, p);
                pos += dot3(s.r + 6, p) + s.t[2] > 0;
            }
            front = pos >= n - pos;
        }
        if (!front) return;
        s.err = quad(c.Om, s.r);
        if (fabs(min_err - s.err) > 1e-6) {
            if (min_err > s.err) {
                min_err = s.err;
                sols.assign(1, s);
            }
        } else {
            bool same = false;
            for (auto& o : sols) {
                double d = 0;
                for (int k = 0; k < 9; k++) d += (o.r[k] - s.r[k]) * (o.r[k] - s.r[k]);
                if (d < 1e-10) {
                    if (o.err > s.err) o = s;
                    same = true;
                    break;
                }
            }
            if (!same) sols.push_back(s);
            if (min_err > s.err) min_err = s.err;
        }
    };
    auto from_eigen = [&](const double* e) {
        for (int sg = 0; sg < 2; sg++) {
            double m[9];
            SqSol s;
            for (int k = 0; k < 9; k++) m[k] = sg ? -e[k] : e[k];
            double r0[9];
            la::nearest_rotation(m, r0);
            sqp_run(c.Om, r0, s.r);
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
            from_eigen(e);
        }
    }
    for (int k = 1; 9 - nn - k > 0 && min_err > 3 * ev[9 - nn - k]; k++) from_eigen(evec + 9 * (9 - nn - k));
    *found = !sols.empty();
    if (!*found) return;
    std::memcpy(R, sols[0].r, sizeof(double) * 9);  // (rodrigues_inv re-orthonormalises, as cv::Rodrigues)
    std::memcpy(t, sols[0].t, sizeof(double) * 3);
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
    bestt[0] = bestt[1] = bestt[2] = 0.0;
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

int RansacSeq::draw_chunk() {
    m = 0;
    if (done || direct) return 0;
    const int sched = chunk_size(rounds, first_chunk);
    const int want = (niters - iter) < sched ? (niters - iter) : sched;
    rounds++;
    Rng r{rng};
    for (int j = 0; j < want; j++)
        for (int i = 0; i < 5; i++) {
            int v;
            bool dup;
            do {
                v = r.uniform(0, n);
                dup = false;
                for (int k = 0; k < i; k++) dup |= idx[j][k] == v;
            } while (dup);
            idx[j][i] = v;
        }
    rng = r.state;
    m = want;
    return want;
}

void RansacSeq::subset(int j, const float** o, const float** im, const int** id) const {
    const int h = nh + j;
    if (h < nsamp) {  // the same 5 points, gathered on the device in draw order
        const float* sp = samp + (size_t)kSampleFloats * h;
        *o = sp;
        *im = sp + 15;
        *id = nullptr;
    } else {
        *o = obj;
        *im = img;
        *id = idx[j];
    }
}

void RansacSeq::store(int j, bool valid_model, const double R[9], const double t[3]) {
    valid[j] = valid_model;
    double* hp = hyp + 12 * j;
    if (valid_model) {
        double rv[3];
        la::cv::rodrigues_inv(R, rv);  // the model is stored as (rvec, tvec)
        la::rodrigues(rv, hp);
        std::memcpy(hp + 9, t, sizeof(double) * 3);
    } else {
        for (int k = 0; k < 12; k++) hp[k] = 0;
    }
}

void RansacSeq::solve(int j, const double K[9]) {
    const float *o, *im;
    const int* id;
    subset(j, &o, &im, &id);
    double Rj[9], tj[3];
    const bool v = epnp_pixels(o, im, id, 5, K, Rj, tj);
    store(j, v, Rj, tj);
}

void epnp_pixels_batch(int count, const float* const* obj, const float* const* img, const int* const* idx,
                       const double K[9], double (*R)[9], double (*t)[3], bool* ok) {
    constexpr int L = kEpnpLanes;
    if (count <= 0) return;
    if (count > L) count = L;
    double pw[L][15], uv[L][10], MtM[L][144], ev[L][12], ut[L][144];
    EPnP es[L] = {EPnP(K[0], K[4], K[2], K[5]), EPnP(K[0], K[4], K[2], K[5]), EPnP(K[0], K[4], K[2], K[5]),
                  EPnP(K[0], K[4], K[2], K[5])};
    for (int q = 0; q < count; q++) {
        epnp_inputs(obj[q], img[q], idx[q], 5, K, pw[q], uv[q]);
        es[q].prepare(pw[q], uv[q], 5, MtM[q]);
    }
    if (count > 1 && la::cv::simd_svd_ok()) {
        const double* pa[L];
        double *pe[L], *pu[L];
        for (int q = 0; q < L; q++) {
            pa[q] = MtM[q < count ? q : count - 1];  // idle lanes repeat a live problem
            pe[q] = ev[q];
            pu[q] = ut[q];
        }
        la::cv::svd_ut_lanes<12, L, 1>(pa, pe, pu);
    } else {
        for (int q = 0; q < count; q++) la::cv::svd_ut<12>(MtM[q], ev[q], ut[q]);
    }
    for (int q = 0; q < count; q++) ok[q] = es[q].finish(ut[q], R[q], t[q]);
}

int RansacSeq::gen_chunk(const double K[9]) {
    const int want = draw_chunk();
    for (int j0 = 0; j0 < want; j0 += kEpnpLanes) {
        RansacSeq* seqs[kEpnpLanes];
        int js[kEpnpLanes];
        const int c = want - j0 < kEpnpLanes ? want - j0 : kEpnpLanes;
        for (int q = 0; q < c; q++) {
            seqs[q] = this;
            js[q] = j0 + q;
        }
        solve_hypotheses(seqs, js, c, K);
    }
    nh += want;
    return want;
}

void solve_hypotheses(RansacSeq* const* seqs, const int* js, int count, const double K[9]) {
    const float *o[kEpnpLanes], *im[kEpnpLanes];
    const int* id[kEpnpLanes];
    double R[kEpnpLanes][9], t[kEpnpLanes][3];
    bool ok[kEpnpLanes];
    for (int q = 0; q < count; q++) seqs[q]->subset(js[q], &o[q], &im[q], &id[q]);
    epnp_pixels_batch(count, o, im, id, K, R, t, ok);
    for (int q = 0; q < count; q++) seqs[q]->store(js[q], ok[q], R[q], t[q]);
}

void RansacSeq::consume(const int* counts, const uint32_t* bits, int words_cap, double confidence) {
    const int words = (n + 31) / 32;
    for (int j = 0; j < m && iter < niters; j++, iter++) {
        const int good = valid[j] ? counts[j] : 0;
        if (good > (maxGood > 4 ? maxGood : 4)) {
            std::memcpy(best.data(), bits + (size_t)words_cap * j, sizeof(uint32_t) * words);
            std::memcpy(bestR, hyp + 12 * j, sizeof(double) * 9);
            std::memcpy(bestt, hyp + 12 * j + 9, sizeof(double) * 3);
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
        la::cv::rodrigues_inv(R, rvec);
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
    double own[kSqpnpStats];
    if (!sums) {
        std::vector<double> pw, q;
        inlier_arrays(obj, img, inliers, K, pw, q);
        sqpnp_sums(pw.data(), q.data(), (int)inliers.size(), own);
        sums = own;
    }
    SqpnpCost c;
    sqpnp_assemble(sums, c);
    fitted = true;
    if (!c.ok) {  // solvePnP(SQPNP) would assert: keep the RANSAC model (as the oracle)
        la::cv::rodrigues_inv(bestR, rvec);
        std::memcpy(tvec, bestt, sizeof(bestt));
        return;
    }
    double Rf[9], tf[3];
    bool found = false;
    fit_from_cost(
        c, (int)inliers.size(),
        [&](int k, double* p) {
            const int i = inliers[k];
            p[0] = obj[3 * i];
            p[1] = obj[3 * i + 1];
            p[2] = obj[3 * i + 2];
        },
        Rf, tf, &found);
    if (!found) {  // no solution in front of the camera: solvePnP fails, keep the RANSAC model
        la::cv::rodrigues_inv(bestR, rvec);
        std::memcpy(tvec, bestt, sizeof(bestt));
        return;
    }
    la::cv::rodrigues_inv(Rf, rvec);
    std::memcpy(tvec, tf, sizeof(tf));
}

void RansacSeq::finish(const double K[9]) {
    select(K);
    fit(K, nullptr);
}

}  // namespace svo

// cv::solvePnP(obj, img, K, zeros, rvec, tvec, false, SOLVEPNP_SQPNP) on the host
// (the fit solvePnPRansac ends with, R:src/tracking.cpp:191-196)
extern "C" int svo_solve_pnp_sqpnp(const double* obj_xyz, const float* img_xy, int n, const double K[9],
                                   double rvec[3], double tvec[3]) {
    using namespace svo;
    if (!obj_xyz || !img_xy || !K || !rvec || !tvec || n < 3) return SVO_ERR_ARG;
    std::vector<double> q(2 * (size_t)n);
    const double ifx = 1. / K[0], ify = 1. / K[4];
    for (int i = 0; i < n; i++) {
        q[2 * i] = ((double)img_xy[2 * i] - K[2]) * ifx;
        q[2 * i + 1] = ((double)img_xy[2 * i + 1] - K[5]) * ify;
    }
    double sums[kSqpnpStats];
    sqpnp_sums(obj_xyz, q.data(), n, sums);
    SqpnpCost c;
    sqpnp_assemble(sums, c);
    if (!c.ok) return 0;
    double R[9], t[3];
    bool found = false;
    fit_from_cost(
        c, n, [&](int k, double* p) { std::memcpy(p, obj_xyz + 3 * (size_t)k, sizeof(double) * 3); }, R, t, &found);
    if (!found) return 0;
    la::cv::rodrigues_inv(R, rvec);
    std::memcpy(tvec, t, sizeof(t));
    return 1;
}

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
