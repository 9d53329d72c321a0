// ORB detection shared by svo_orb_detect (one frame) and the batched front end
// (one frame per sequence, SVO_FE use_orb): level geometry, the host's
// per-level selection (computeKeyPoints' runByImageBorder + retainBest), and the
// batched device pipeline (orb_detect.cpp, orb.hip).
#pragma once

#include <functional>
#include <vector>

#include "common.hpp"

namespace svo {

struct OrbGeometry {
    int nlev = 0;
    int lw[kMaxLevels], lh[kMaxLevels], pitch[kMaxLevels], kcap[kMaxLevels], nf[kMaxLevels];
    float lscale[kMaxLevels];
    int maxcap = 0, maxh = 0, maxnseg = 0;
    // INTER_LINEAR_EXACT tables of levels 1.. (x offsets, x coefficients, y offsets,
    // y coefficients, each level at tab_at[l])
    std::vector<uint32_t> tabs;
    size_t tab_at[kMaxLevels] = {0};
};

// false: parameters outside what the detector supports (err names the reason)
bool orb_geometry(int W, int H, const svo_orb_params& p, OrbGeometry& g, const char** err);

// computeKeyPoints' selection from the per-level FAST keypoints kps[l][0..n[l])
// (level coordinates) and, with HARRIS, their responses resp[l]: runByImageBorder,
// retainBest(2 n_l) by FAST response, retainBest(n_l) by Harris response, level
// order, pt *= s_l. Writes min(total, cap) keypoints; returns the total.
int orb_select(const OrbGeometry& g, const svo_orb_params& p, const svo_keypoint* const* kps,
               const float* const* resp, const int* n, svo_keypoint* out, int* octave, int cap);

// ORB detection of one frame per sequence for the batched front end. The level
// images, masks, FAST scratch and keypoints of all sequences live in one
// allocation; detect() runs the device stages batched over the sequences (scale
// pyramid + mask pyramid, FAST per level, Harris) and the host selection per
// sequence (par(S, fn): fn(s) for every s, possibly in parallel), then writes the
// selected keypoints (level-0 coordinates) to out[s * cap_out ..] and their counts
// to nout[s] on the device. Synchronous on the host.
struct OrbBatch;
OrbBatch* orb_batch_create(int S, int W, int H, const svo_orb_params& p);
void orb_batch_destroy(OrbBatch* ob);
// lv0[s]: level 0 (the frame) of sequence s. Mask: boxes of +-half around
// box_counts[s] points of box_pts + 2 s box_stride (device), or none when box_pts
// is null. overflow[s] (host, nullable): keypoints beyond cap_out.
hipError_t orb_batch_detect(OrbBatch* ob, const ImgLevel* lv0, const float* box_pts, const int* box_counts,
                            int box_stride, int box_max, float half, svo_keypoint* out, int* nout, int cap_out,
                            hipStream_t st, const std::function<void(int, const std::function<void(int)>&)>& par,
                            int* overflow);

hipError_t launch_orb_resize(const uint8_t* src, int spitch, const uint8_t* smask, int sw, uint8_t* dst, int dpitch,
                             uint8_t* dmask, int dw, int dh, const int* xofs, const uint32_t* xc, const int* yofs,
                             const uint32_t* yc, hipStream_t st);
// every sequence's level: src[s].lv[0] -> dst[s].lv[0] (all of size dw x dh), masks
// smask + s * smask_stride (width sw) -> dmask + s * dmask_stride (nullable)
hipError_t launch_orb_resize_batched(const PyrDesc* src, const PyrDesc* dst, const uint8_t* smask,
                                     size_t smask_stride, int sw, uint8_t* dmask, size_t dmask_stride, int dw, int dh,
                                     int nseq, const int* xofs, const uint32_t* xc, const int* yofs,
                                     const uint32_t* yc, hipStream_t st);
hipError_t launch_orb_harris(const PyrDesc& levels, int nlevels, const svo_keypoint* kps, const int* n, int cap,
                             int max_n, float* resp, hipStream_t st);
// levels[l * nseq + s].lv[0]: level l of sequence s; kps / resp [l][s][cap], n [l][s]
hipError_t launch_orb_harris_batched(const PyrDesc* levels, int nlevels, int nseq, const svo_keypoint* kps,
                                     const int* n, int cap, int max_n, float* resp, hipStream_t st);

}  // namespace svo
