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
#include "linalg.hpp"
#include "pose.hpp"
#include "sqpnp.hpp"

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

using sq::SqpnpCost;
using sq::sqpnp_assemble;

// The SQPnP solution search on the host (sqpnp.hpp): Omega's eigen-decomposition,
// SQPnP's asserts on it, the starts run in order as the search asks for them.
// pt(k, p): object point k of the n fitted points into p[3]. *found: false when
// SQPnP asserts on Omega or finds no solution in front of the camera.
template <class PointAt>
void fit_from_cost(const SqpnpCost& c, int n, PointAt pt, double R[9], double t[3], bool* found) {
    double Oc[81], ev[9], evec[81];
    std::memcpy(Oc, c.Om, sizeof(Oc));
    la::sym_eig_ql(Oc, 9, ev, evec);  // descending; eigenvector k in row k
    *found = false;
    const int nn = sq::sq_null_count(ev);
    if (nn < 0) return;
    sq::sq_select(
        c, ev, evec, nn, n, [&](int j, double* r) { sq::sq_start(c, evec, j, r); },
        [&](const double* r, const double* tt) {
            int pos = 0;
            for (int k = 0; k < n; k++) {
                double p[3];
                pt(k, p);
                pos += dot3(r + 6, p) + tt[2] > 0;
            }
            return pos;
        },
        R, t, found);
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

bool epnp_isa_supported(int isa) {
    static const bool avx2 = __builtin_cpu_supports("avx2"), avx512 = __builtin_cpu_supports("avx512f");
    return isa == kEpnpScalar || (isa == kEpnpAvx2 && avx2) || (isa == kEpnpAvx512 && avx512);
}

void epnp_pixels_batch(int count, const float* const* obj, const float* const* img, const int* const* idx,
                       const double K[9], double (*R)[9], double (*t)[3], bool* ok, int isa) {
    if (count <= 0) return;
    if (count > kEpnpLanes) count = kEpnpLanes;
    if (isa == kEpnpAuto)
        isa = count == 1                            ? kEpnpScalar
              : epnp_isa_supported(kEpnpAvx512) ? kEpnpAvx512
              : epnp_isa_supported(kEpnpAvx2)   ? kEpnpAvx2
                                                : kEpnpScalar;
    if (isa == kEpnpAvx512) {
        epnp_batch_avx512(count, obj, img, idx, K, R, t, ok);
    } else if (isa == kEpnpAvx2) {
        epnp_batch_avx2(count, obj, img, idx, K, R, t, ok);
    } else {
        for (int q = 0; q < count; q++) ok[q] = epnp_pixels(obj[q], img[q], idx[q], 5, K, R[q], t[q]);
    }
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
