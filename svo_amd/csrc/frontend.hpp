// Batched tracking front end (device-resident state + launch helpers).
#pragma once

#include "common.hpp"

namespace svo {

// Keyframe map points of the previous step are stored in the left camera frame
// of their keyframe until that frame's pose is known (the host's final SQPnP fit
// runs while the GPU tracks the next frame): map[pend0[s] .. pend0[s] + pend_n[s])
// of sequence s are moved to the world frame by pose[s] = {R (row-major 3x3),
// t} (camera -> world, Frame::pose(), R:src/tracking.cpp:141) before anything
// reads them; pend_n[s] is zeroed then, so the step is idempotent.
struct PendingMap {
    double* map;         // [s][map_cap] xyz
    int map_cap;
    const int* pend0;    // [s]
    int* pend_n;         // [s]
    const double* pose;  // [s][12], host-coherent
};

// Everything between temporal LK and the host's RANSAC, one block per
// sequence: the pending keyframe map points to the world frame (PendingMap),
// stable compaction of the tracked features (status == 1,
// R:src/tracking.cpp:169-175) into xy_out / mid_out / n_out, the LK iteration
// sum, the map-point gather into obj (float, as solvePnPRansac converts
// Point3d, :182-187), and the 5-point subsets of the first nh RANSAC hypotheses
// (cv::RNG(-1) draws over the new count) gathered as obj[5][3] + img[5][2]
// floats. h_n / h_iters / h_samp are host-coherent (zero-copy): the host reads
// them once the kernel is done.
struct PostLkBatch {
    const int* n_in;
    const uint8_t* status;
    const float* xy_in;
    const int* mid_in;
    const int* iters;
    float* xy_out;
    int* mid_out;
    int* n_out;
    PendingMap pm;
    float* obj;
    int cap, nh;
    int* h_n;
    long long* h_iters;
    float* h_samp;  // [s][nh][25]
};
hipError_t launch_post_lk(const PostLkBatch& b, int nseq, hipStream_t st);
// PendingMap alone (before the map is read by anything but post_lk)
hipError_t launch_finalize_map(const PendingMap& pm, int nseq, hipStream_t st);

// The step's tail, part 1, one block per sequence: stable compaction by the
// RANSAC inlier bits (read from host-coherent memory; R:src/tracking.cpp:218-229)
// into xy_out / mid_out / n_out, then the keyframe's new-feature candidates: the
// first take = min(n_target[s] - n, candidates, capacity) masked FAST corners
// (extractFeatures, :74-92), copied to st_xy (the stereo LK's input) with their
// count in st_n.
struct TailBatch {
    const int* n_in;
    const uint32_t* bits;  // [s][words_cap], host-coherent
    int words_cap;
    const float* xy_in;
    const int* mid_in;
    float* xy_out;
    int* mid_out;
    int* n_out;
    int cap;
    const int* n_target;  // [s] host-coherent: n_features on a keyframe, 0 otherwise
    const float* cand;  // candidates, cand_elem floats each, cand_cap per sequence
    int cand_elem, cand_cap;
    const int* cand_n;
    const int* map_n;
    int map_cap;
    float* st_xy;  // [s][cap]
    int* st_n;     // [s]
    // nullable, host-coherent: candidates beyond the take, cand_n - take (the
    // detector's raw count: a keyframe under Tracking::nextFrame's rule takes every
    // masked corner, so anything here is a capacity overflow there)
    int* h_over;
    // nullable: SQPnP's sufficient statistics of the inliers (suffstats.hpp) into
    // stats_out[s][40] (host-coherent), from xy_in / stats_obj / bits -- computed by
    // the same workgroup, so the statistics are done when the keyframe is
    const float* stats_obj = nullptr;
    double* stats_out = nullptr;
    double ifx = 0, ify = 0, cx = 0, cy = 0;
};
hipError_t launch_tail(const TailBatch& tb, int nseq, hipStream_t st);

// The step's tail, part 2 (after the stereo LK of st_xy into the right image and
// stereo_tri_kernel's filter + DLT of its matches, st_X), one block per sequence:
// the survivors of findLeftFeaturesInRight's filter (status and |yR - yL| <
// y_threshold, R:src/tracking.cpp:109-114) and triangulateNewMapPoints' z > 0
// (:120-152) appended in order as new features with new map points (left camera
// frame, pending the frame's pose: PendingMap) -- a compaction only. h_n /
// h_added: host-coherent copies of the counts.
struct AppendBatch {
    int* n;       // features per sequence (in/out)
    float* xy;    // [s][cap]
    int* mid;     // [s][cap]
    int cap;
    const float* st_xy;      // [s][cap] left points
    const int* st_n;
    double* map;  // [s][map_cap]
    int* map_n;
    int map_cap;
    int* pend0;
    int* pend_n;
    int* added;   // nullable
    int* h_n;     // nullable, host-coherent
    int* h_added; // nullable, host-coherent
    const float4* st_X;  // stereo_tri_kernel's filter + DLT of st_xy[0, n) (x, y, z, keep)
};
hipError_t launch_append(const AppendBatch& b, int nseq, hipStream_t st);

// Speculative stereo input, one block per sequence, queued as soon as the step's
// tracked count n_tracked (post-LK) and the FAST candidates are known, i.e. before
// the RANSAC: the keyframe takes the first take = min(n_target - kept, ...)
// candidates, kept <= n_tracked inliers, so the first
//   spec = min(n_target[s] - n_tracked + margin, cand_n, cand_cap, cap, map_cap - map_n)
// candidates cover take whenever RANSAC drops at most `margin` points. They are
// copied to st_xy with their count in spec_n, and their stereo LK runs beside
// the host's RANSAC (a feature's LK depends on nothing but its own point).
struct StereoPrepBatch {
    const int* n_tracked;
    const float* cand;
    int cand_elem, cand_cap;
    const int* cand_n;
    const int* map_n;
    int map_cap, cap, margin;
    const int* n_target;  // [s], as TailBatch::n_target
    float* st_xy;
    int* spec_n;
};
hipError_t launch_stereo_prep(const StereoPrepBatch& b, int nseq, hipStream_t st);

// findLeftFeaturesInRight's filter + triangulateNewMapPoints' DLT and z > 0 test of
// the candidates st_xy[0, spec_n[s]) right behind their stereo LK (a candidate's
// point depends only on its own match and the fixed stereo projections), so the
// keyframe only compacts and appends: st_X[s][j] = (x, y, z, keep) in the left
// camera frame. The speculative candidates (spec_n), or the serial keyframe's
// exact take (st_n).
struct StereoTriBatch {
    const float* st_xy;
    const float* st_next;
    const uint8_t* st_status;
    const int* spec_n;
    int cap;
    float y_threshold;
    float P[24];  // P_left, P_right
    float4* st_X;
};
hipError_t launch_stereo_tri(const StereoTriBatch& b, int nseq, int max_n, hipStream_t st);

// tail_kernel + append_kernel in one launch, for a step whose speculative stereo
// LK covered every sequence's take (st_next / st_status already hold the matches
// of st_xy[0, take)); same results as the two kernels with the LK between them.
hipError_t launch_keyframe_fused(const TailBatch& tb, const AppendBatch& ab, int nseq, hipStream_t st);

}  // namespace svo
