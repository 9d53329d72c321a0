// Batched tracking front end (device-resident state + launch helpers).
#pragma once

#include "common.hpp"

namespace svo {

struct CompactBatch {
    const int* n_in;
    const uint8_t* status;  // either status (u8 per point) ...
    const uint32_t* bits;   // ... or a bitmask (words_cap words per sequence)
    int words_cap;
    const float* xy_in;
    const int* mid_in;
    const int* iters;        // nullable: per-point LK iterations to sum
    long long* iters_sum;    // nullable: per-sequence sum
    float* xy_out;
    int* mid_out;
    int* n_out;
    int cap;
};
hipError_t launch_compact(const CompactBatch& b, int nseq, hipStream_t st);
hipError_t launch_gather(const int* n, const int* mid, const double* map, int cap, int map_cap, float* obj,
                         int nseq, int max_n, hipStream_t st);

// The 5-point subsets of the first nh (<= 64) RANSAC hypotheses of every
// sequence (cv::RNG(-1) draws over counts[s] points), gathered as obj[5][3] +
// img[5][2] floats per hypothesis into samp[s][nh][25].
hipError_t launch_ransac_samples(const int* counts, const float* obj, const float* img, int cap, int nh, int nseq,
                                 float* samp, hipStream_t st);

// Everything between temporal LK and the host's RANSAC, one 1024-thread block
// per sequence: stable compaction of the tracked features (status == 1) into
// xy_out / mid_out / n_out, the LK iteration sum, the map-point gather into obj
// (float, as solvePnPRansac converts), and the 5-point subsets of the first nh
// RANSAC hypotheses (cv::RNG(-1) draws over the new count) gathered as
// obj[5][3] + img[5][2] floats. h_n / h_iters / h_samp are host-coherent
// (zero-copy): the host reads them once the kernel is done.
struct PostLkBatch {
    const int* n_in;
    const uint8_t* status;
    const float* xy_in;
    const int* mid_in;
    const int* iters;
    float* xy_out;
    int* mid_out;
    int* n_out;
    const double* map;
    int map_cap;
    float* obj;
    int cap, nh;
    int* h_n;
    long long* h_iters;
    float* h_samp;  // [s][nh][25]
    // streamed mode (rec != null): the block of sequence s first waits until all
    // n_in LK records (LKBatch::rec) of s show lk_stamp, reads them with sc1
    // loads, and at its end publishes h_ready[s] = stamp (system scope) after its
    // host-coherent writes; h_fail[0] = 1 if the wait timed out
    const unsigned* rec = nullptr;
    int lk_stamp = 0;
    int* h_ready = nullptr;
    int stamp = 0;
    int* h_fail = nullptr;
};
hipError_t launch_post_lk(const PostLkBatch& b, int nseq, hipStream_t st);

// The step's tail, one block per sequence: stable compaction by the RANSAC
// inlier bits (read from host-coherent memory), then the keyframe top-up
// (append_kernel's body). h_n / h_added: host-coherent copies of the counts.
struct TailBatch {
    const int* n_in;
    const uint32_t* bits;  // [s][words_cap], host-coherent
    int words_cap;
    const float* xy_in;
    const int* mid_in;
    int* h_n;
    int* h_added;
};

struct AppendBatch {
    int* n;             // features per sequence (in/out)
    float* xy;          // [s][cap] xy
    int* mid;           // [s][cap]
    int cap, n_target;
    const float* cand;  // candidates, cand_elem floats each, cand_cap per sequence
    int cand_elem, cand_cap;
    const int* cand_n;
    double* map;        // [s][map_cap] xyz
    int* map_n;
    int map_cap;
    const double* rot;  // [s] 3x3 world->camera of this frame
    const int* depth_seed;
    int* added;         // nullable
    double K[9];
};
hipError_t launch_append(const AppendBatch& b, int nseq, hipStream_t st);
// compaction (TailBatch: into ab.xy / ab.mid / ab.n) + top-up (AppendBatch)
hipError_t launch_tail(const TailBatch& tb, const AppendBatch& ab, int nseq, hipStream_t st);

}  // namespace svo
