// Host side of the pose update (solvePnPRansac with GPU hypothesis scoring).
#pragma once

#include <cstdint>
#include <vector>

namespace svo {

struct Rng {  // cv::RNG (core/include/opencv2/core/operations.hpp): multiply-with-carry
    uint64_t state;
    uint32_t next() {
        state = (uint64_t)(uint32_t)state * 4164903690U + (uint32_t)(state >> 32);
        return (uint32_t)state;
    }
    int uniform(int a, int b) { return a == b ? a : (int)(next() % (unsigned)(b - a) + a); }
};

constexpr int kRansacChunk = 16;  // hypotheses generated per scoring launch
// hypotheses whose 5-point subsets the device gathers ahead of the host RANSAC
// (chunk schedule 2 + 8 + 16): the host then needs no full copy of the points
constexpr int kRansacPrefetch = 26;
constexpr int kSampleFloats = 25;  // 5 points x (obj xyz, pixel xy)

// The RANSAC minimal solver batched: EPnP of count <= kEpnpLanes 5-point subsets
// (subset q: points idx[q][0..5) of obj[q] / img[q], or points 0..4 when idx[q]
// is null), bit-identical to epnp_pixels on each: the whole solver runs in SIMD
// lanes (epnp_lanes.hpp), AVX-512 (8 lanes x 2 interleaved groups) or AVX2 (4 x
// 4) as the CPU has it, else scalar. ok[q]: finite model.
constexpr int kEpnpLanes = 16;
enum EpnpIsa { kEpnpAuto = -1, kEpnpScalar = 0, kEpnpAvx2 = 1, kEpnpAvx512 = 2 };
bool epnp_isa_supported(int isa);
void epnp_pixels_batch(int count, const float* const* obj, const float* const* img, const int* const* idx,
                       const double K[9], double (*R)[9], double (*t)[3], bool* ok, int isa = kEpnpAuto);
// the per-instruction-set bodies (epnp_avx2.cpp, epnp_avx512.cpp; count <= 16)
void epnp_batch_avx2(int count, const float* const* obj, const float* const* img, const int* const* idx,
                     const double K[9], double (*R)[9], double (*t)[3], bool* ok);
void epnp_batch_avx512(int count, const float* const* obj, const float* const* img, const int* const* idx,
                       const double K[9], double (*R)[9], double (*t)[3], bool* ok);
struct RansacSeq;
// hypotheses js[q] of sequences seqs[q] (q < count <= kEpnpLanes; drawn by
// draw_chunk) solved as one epnp_pixels_batch and stored (RansacSeq::store)
void solve_hypotheses(RansacSeq* const* seqs, const int* js, int count, const double K[9]);

// RANSACPointSetRegistrator::run for PnP (5-point EPnP kernel), split so the
// hypotheses of many sequences are scored by one batched kernel launch:
//   begin -> { gen_chunk -> [GPU: score m hypotheses] -> consume } until done -> finish
struct RansacSeq {
    const float* obj = nullptr;  // n x 3 (float, as OpenCV converts Point3d)
    const float* img = nullptr;  // n x 2
    // optional: the subsets of hypotheses [0, nsamp) gathered by the device, in
    // draw order (kSampleFloats per hypothesis); obj / img are then only read
    // for hypotheses past nsamp, the n <= 5 direct solve and the final fit
    const float* samp = nullptr;
    int nsamp = 0;
    int n = 0;
    uint64_t rng = 0;
    int niters = 0, iter = 0, maxGood = 0, nh = 0, m = 0, rounds = 0;
    // size of the first hypothesis chunk (a scheduling choice only: the draws and
    // the accept replay are the same for any chunking). 0: the default 2.
    int first_chunk = 0;
    bool done = true, direct = false, ok = false, fitted = false;
    bool valid[kRansacChunk];
    double hyp[12 * kRansacChunk];
    int idx[kRansacChunk][5];  // the subsets of the chunk drawn by draw_chunk
    std::vector<uint32_t> best;
    double bestR[9], bestt[3];
    std::vector<int> inliers;
    double rvec[3] = {0, 0, 0}, tvec[3] = {0, 0, 0};

    void begin(const float* obj, const float* img, int n, int iterations);
    // RANSACUpdateNumIters' niters for outlier ratio ep: a prediction of how many
    // hypotheses this sequence needs, from its previous frame
    static int predict_iters(double confidence, double ep, int max_iters);
    int gen_chunk(const double K[9]);  // fills hyp[0..m) (R row-major + t); returns m
    // gen_chunk in two parts, so a pool can solve one chunk's hypotheses on several
    // threads: draw_chunk draws the chunk's subsets (the RNG's order) and returns
    // m; solve(j) fills hypothesis j < m
    int draw_chunk();
    void solve(int j, const double K[9]);
    // solve(j) in two halves around a batched EPnP (epnp_pixels_batch): the
    // subset's points, and the model stored as (rvec, tvec) -> hyp[j]
    void subset(int j, const float** o, const float** im, const int** id) const;
    void store(int j, bool valid_model, const double R[9], const double t[3]);
    // hypotheses generated once the next gen_chunk has run (for deciding whether
    // the full point arrays must be on the host first)
    int next_end() const;
    void consume(const int* counts, const uint32_t* bits, int words_cap, double confidence);
    // inlier set of the best model (the output): `best` bits, and the index list
    // too unless list = false (fit() then builds it)
    void select(const double K[9], bool list = true);
    // final SQPnP-objective fit on the inliers; sums = their kSqpnpStats
    // sufficient statistics (sqpnp_sums / the suffstats kernel) or null to compute here
    void fit(const double K[9], const double* sums);
    void finish(const double K[9]);    // select + fit
};

// Sufficient statistics of SQPnP's cost over n points (kSqpnpStats doubles):
// [0] n, [1] sum x, [2] sum y, [3] sum (x^2 + y^2), [4..15] sum c X for c in
// (1, x, y, x^2 + y^2), [16..39] sum c X X^T (6 unique entries each), with (x, y)
// the normalised image point and X the object point.
constexpr int kSqpnpStats = 40;
void sqpnp_sums(const double* pw, const double* q, int n, double* sums);

}  // namespace svo
