// Shared host/device definitions for libsvo_gpu.so (MI355X / gfx950).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "svo_gpu.h"

namespace svo {

constexpr int kMaxLevels = 8;  // pyramid levels kept per image (0..7)

// Every pyramid level is stored with a kPyrPad-pixel REFLECT_101 border on all
// four sides (OpenCV pads its LK pyramid levels the same way, by the window
// size) and every derivative level with a kDerPad-element zero border (OpenCV's
// zero-padded derivative levels): the LK kernels read windows and staged
// regions reaching up to win + margin pixels outside a level without any
// border test. `data` points at pixel (0, 0) of the interior.
constexpr int kPyrPad = 32;
constexpr int kDerPad = 32;

// One pyramid level in HBM: u8 rows (pitch multiple of 64 B), padded as above.
struct ImgLevel {
    const uint8_t* data;
    int w, h, pitch;
};

// A whole pyramid, passed by value to kernels (small) or by pointer for batches.
struct PyrDesc {
    ImgLevel lv[kMaxLevels];
    int nlevels;  // levels present (>= 1)
};

// Mirror of buildOpticalFlowPyramid's early stop (lkpyramid.cpp): the level
// index reached before the next size would be <= the window.
inline int lk_levels_for_window(int w, int h, int win_w, int win_h, int max_level) {
    int sw = w, sh = h;
    for (int level = 0; level <= max_level; level++) {
        sw = (sw + 1) / 2;
        sh = (sh + 1) / 2;
        if (sw <= win_w || sh <= win_h) return level;
    }
    return max_level;
}

}  // namespace svo

struct svo_image {
    int w = 0, h = 0;
    int nlevels = 0;  // allocated levels (max_levels + 1)
    uint8_t* base = nullptr;
    size_t bytes = 0;
    svo::PyrDesc desc{};
};

// Per-context scratch buffers, grown on demand (never inside a capture).
struct svo_scratch {
    void* p = nullptr;
    size_t bytes = 0;
};

struct svo_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    int64_t lk_iters = 0;
    svo_scratch s[12];
    void* pinned = nullptr;
    size_t pinned_bytes = 0;
    // colour ingest: pinned double buffer (host copy of frame k+1 overlaps the
    // H2D of frame k), reused once its event shows the H2D is done
    void* ingest_host[2] = {nullptr, nullptr};
    size_t ingest_bytes[2] = {0, 0};
    hipEvent_t ingest_ev[2] = {nullptr, nullptr};
    int ingest_next = 0;
    // The batched front ends' streams (LK: highest priority, FAST: lowest, copies,
    // uploads), created with the first front end and shared by every later one on
    // this context: each stream binds a hardware queue, so a long-lived process
    // that creates and destroys front ends (a second one made while the first lived
    // bound three more) keeps one fixed set of queues, and front ends on one
    // context are ordered on them.
    hipStream_t fe_lk = nullptr, fe_fast = nullptr, fe_copy = nullptr, fe_up = nullptr;
};

namespace svo {

int set_error(svo_ctx* ctx, int code, const char* fmt, ...);
// Grow scratch slot `slot` to >= bytes; returns device pointer or nullptr.
void* scratch(svo_ctx* ctx, int slot, size_t bytes);
void* pinned(svo_ctx* ctx, size_t bytes);

// Kernel launchers (implemented in the .hip files).
hipError_t launch_pyramid(const svo_image* img, int first_level, hipStream_t st);
hipError_t launch_bgr_to_gray(const uint8_t* bgr, int bpitch, uint8_t* dst, int pitch, int w, int h,
                              hipStream_t st);
// H2D of a host BGR image through the context's pinned double buffer and its
// grey conversion into `level0` (w x h, row pitch `pitch`), on ctx->stream.
int ingest_bgr(svo_ctx* ctx, const uint8_t* bgr, int stride, int w, int h, uint8_t* level0, int pitch);
// level 0 of S sequences (descs[s].lv[0]) from a staging block [S][h][spitch]
// (grey bytes, or BGR converted as launch_bgr_to_gray)
hipError_t launch_ingest_batched(const uint8_t* stage, size_t seq_stride, int spitch, const PyrDesc* descs, int S,
                                 int w, int h, bool bgr, hipStream_t st);
hipError_t launch_pyramid_batched(const PyrDesc* d_descs, int nseq, int w, int h, int nlevels,
                                  hipStream_t st);

// Batched FAST: sequence z reads level 0 of descs[z]; per-sequence slices of
// cs/mask (npx each), rowcnt (h each), out (cap each), n_out (1 each).
struct FastBatch {
    const PyrDesc* descs;
    uint16_t* cs;
    const uint8_t* mask;  // nullable
    int* rowcnt;
    svo_keypoint* out;
    int* n_out;
    size_t npx;
    int cap;
};
hipError_t launch_fast_score(const FastBatch& b, int nseq, int w, int h, int threshold, int nonmax,
                             hipStream_t st);
hipError_t launch_fast_collect(const FastBatch& b, int nseq, int w, int h, int nonmax, hipStream_t st);

// Fused detection path: detect (score + NMS + mask -> 64-bit keep masks per row
// segment + row counts), scan (row offsets), emit (raster-order keypoints).
struct FastDetBatch {
    const PyrDesc* descs;
    const uint8_t* mask;        // nullable, npx per sequence
    unsigned long long* bits;   // [s][nseg][h]: one block's rows of a segment contiguous
    int* rowcnt;                // [s][h]
    int* rowoff;                // [s][h]
    svo_keypoint* out;          // [s][cap]
    int* n_out;                 // [s]
    size_t npx;
    int nseg, cap;
    // alternatively (mask null): boxes of +-box_half around box_counts[s] points
    // of box_pts + 2*s*box_stride, rasterised per tile inside the kernel
    const float* box_pts = nullptr;
    const int* box_counts = nullptr;
    int box_stride = 0;
    float box_half = 0.f;
    // scratch for binning the box centres by (16-row band, 64-column tile) cell:
    // [s][box_stride] float2 and [s][fast_box_cells(w, h)] offsets
    float* box_binned = nullptr;
    int* box_band = nullptr;
    bool box_prebinned = false;  // launch_box_bin already ran (e.g. ahead, off the critical path)
    // nullable [s][npx]: fast_detect_q_kernel writes the score of every kept corner
    // there, so the emit pass reads one byte instead of re-scoring from the image
    uint8_t* score_map = nullptr;
    // the images carry the kPyrPad border of svo_image levels (any content: the
    // detector never uses a pixel outside the image), so every tile stages its
    // pixels with dword loads; false for unpadded images (ORB's scale levels)
    bool padded = false;
};
// stage: kFastAll detect + scan + emit, kFastDetect detect only (the row counts
// are cleared first); kFastBoxes: the detection already ran without the box mask
// (kFastDetect with no box_pts): AND the rasterised boxes into its row words,
// recount, scan + emit
constexpr int kFastAll = 0, kFastDetect = 1, kFastBoxes = 3;
// ints of band-offset scratch per sequence for an image of height h
// Box centres are binned by cell: 16-row band x 64-column tile (the FAST tile
// grid), cell-major per band; [s][cells + 1] offsets.
inline int fast_box_cells(int w, int h) { return ((h + 15) / 16) * ((w + 63) / 64) + 1; }
hipError_t launch_fast_detect(const FastDetBatch& b, int nseq, int w, int h, int threshold, int nonmax,
                              hipStream_t st, int stage = kFastAll);
// The band binning of the box centres alone (needs only box_pts / box_counts).
hipError_t launch_box_bin(const FastDetBatch& b, int nseq, int w, int h, hipStream_t st);
// Masks for nseq sequences (w*h each): 255 + filled boxes around counts[s] (or n)
// points of pts + s*pts_stride.
hipError_t launch_mask_boxes(int w, int h, const float* pts, const int* counts, int n, int pts_stride,
                             int nseq, float half, uint8_t* mask, hipStream_t st);

// Scharr derivative pyramid of one image (packed int16 Ix | Iy << 16 per pixel),
// stored scaled by 2^kDerShift (|Ix|, |Iy| <= 4080, so 4x still fits int16): a
// bilinear sum of the scaled values carries the CV_DESCALE(., W_BITS) result in
// its high 16 bits (W_BITS + kDerShift == 16), which the LK kernels pack by byte
// permutes instead of shifting every sum.
constexpr int kDerShift = 2;
struct DerivDesc {
    uint32_t* data[kMaxLevels];
    int pitch[kMaxLevels];  // elements
};
// off[l] = element-0 offset (bytes) of level l's interior from the buffer start;
// the buffer must be zeroed once (the borders are never written).
size_t deriv_layout(int w, int h, int nlevels, size_t* off, int* pitch);
// level `level` (w x h) of a derivative pyramid to the host, split into ix / iy
// (int16, x 2^kDerShift as stored); either output may be null (capi.cpp)
int download_deriv_level(svo_ctx* ctx, const DerivDesc& dd, int level, int w, int h, int16_t* ix, int16_t* iy,
                         int stride);
// REFLECT_101 border of levels [0, nlevels) of nseq pyramids (after they are built)
hipError_t launch_pyramid_pad(const PyrDesc* d_descs, int nseq, int w, int h, int nlevels, hipStream_t st);
// one level's derivative (level dims lw x lh)
hipError_t launch_scharr_level(const PyrDesc* d_pyrs, const DerivDesc* d_ders, int nseq, int lw, int lh, int level,
                               hipStream_t st);
// pyramid levels 1.. and derivative levels 0.. in one pass per level (pyramid.hip)
hipError_t launch_pyramid_scharr_batched(const PyrDesc* d_descs, const DerivDesc* d_ders, int nseq, int w, int h,
                                         int nlevels, hipStream_t st);
hipError_t launch_scharr(const PyrDesc* d_pyrs, const DerivDesc* d_ders, int nseq, int w, int h, int nlevels,
                         hipStream_t st);

struct LKParams {
    int win_w, win_h;
    int max_level;  // effective (already clamped)
    int max_count;
    double eps2;
    int flags;
    float min_eig;
    int want_err;
    int generic = 0;  // 1: always use the runtime-window kernel (tests compare both)
    int quad = 1;     // 21x21: four features per wave; 0: one per wave (lk_fast_kernel)
    int cv_order = 0; // 1: OpenCV's float summation order (SVO_LK_OPENCV_ORDER, lk_cv_kernel)
};
// A/B and test hooks of the kernel choice, read per call: SVO_LK_GENERIC=1 (the
// runtime-window kernel for every window), SVO_LK_QUAD=0 (21x21 one per wave)
void lk_apply_env(LKParams& p);
// Batched LK: blockIdx.y = sequence; sequence s owns points [s*cap, s*cap + n_s)
// of every array, n_s = counts[s] (device) or n when counts is null.
struct LKBatch {
    const PyrDesc* prev;     // [nseq] device
    const PyrDesc* next;     // [nseq] device
    const DerivDesc* dprev;  // [nseq] device: Scharr pyramid of prev (launch_scharr)
    const float* prev_xy;
    float* next_xy;
    uint8_t* status;
    float* err;   // nullable
    int* iters;   // nullable
    const int* counts;  // nullable
    int n, cap;
    // > 0 (one-feature-per-wave kernel only): grid for this many features per
    // sequence; waves loop over any beyond it (a device-side count the host only
    // bounds loosely, e.g. the speculative stereo candidates)
    int grid_hint = 0;
};
hipError_t launch_lk(const LKBatch& b, int nseq, int max_n, const LKParams& p, hipStream_t st);
bool lk_supported(int win_w, int win_h);

// Batched residual scoring: blockIdx.z = sequence, blockIdx.y = hypothesis.
// Sequence s: obj/img points [s*cap, s*cap + n_s), hypotheses [s*m, s*m + m),
// err rows of cap floats, bits rows of words_cap words, cnt per hypothesis.
struct PnpBatch {
    const float* obj;
    const float* img;
    const int* counts;  // nullable -> n
    int n, cap;
    const double* hyp;
    int m;
    float* err;      // nullable
    uint32_t* bits;  // nullable
    int words_cap;
    int* cnt;        // nullable
    int mstride = 0; // hypothesis-row stride of hyp/err/bits/cnt per sequence (0: m)
};
hipError_t launch_pnp_residuals(const PnpBatch& b, int nseq, int max_n, double fx, double fy, double cx,
                                double cy, float thresh2, hipStream_t st);
// The same scoring, one block per (hypothesis, sequence): bits as above and ONE
// inlier count per hypothesis in b.cnt (required; no memset needed)
// RANSAC's EPnP on m 5-point subsets (25 floats each: obj xyz x5, img xy x5), one
// wave per subset (epnp_wave.hip); Rt: m x 12 doubles, ok: m ints; K on the device
hipError_t launch_epnp_wave(const float* subsets, int m, const double* K, double* Rt, int* ok, hipStream_t st);
// one lane per subset, the front end's host solver run in each lane (epnp_lane.hip)
hipError_t launch_epnp_lanes(const float* subsets, int m, const double* K, double* Rt, int* ok, hipStream_t st);
hipError_t launch_pnp_score(const PnpBatch& b, int nseq, double fx, double fy, double cx, double cy, float thresh2,
                            hipStream_t st);

// Batched bucket selection: blockIdx.x = sequence. Input points are in_elem
// floats apart (2 = xy pairs, 3 = svo_keypoint), in_cap per sequence.
struct BucketBatch {
    const float* xy;
    int in_elem, in_cap;
    const int* in_counts;  // nullable -> n
    int n;
    const int* ages;  // nullable
    float* xy_out;
    int* ages_out;  // nullable
    int out_cap;
    int* n_out;
    int* scr;
    size_t scr_stride;
};
hipError_t launch_triangulate(const float* d_P, const float* d_p1, const float* d_p2, int n, float* d_xyzw,
                              float* d_xyz, hipStream_t st);
size_t reproj_partial_doubles(int n_problems, int max_n);
hipError_t launch_reproj(const double* d_obj, const float* d_img, const int* d_counts, int n_problems, int cap,
                         int max_n, const double* d_poses, const double K[9], double delta, double* d_res,
                         double* d_jac, double* d_partial, double* d_normal, hipStream_t st);
hipError_t launch_suffstats(const float* obj, const float* img, const int* counts, int cap, const uint32_t* bits,
                            int words_cap, int nseq, const double K[9], double* out, hipStream_t st);
// solvePnPRansac's outcome per sequence as the host's RANSAC left it, the input of
// the device's final fit: mode 0 no model (identity pose), 1 SQPnP fit on the
// inliers (R / t: the RANSAC model, kept where SQPnP asserts or finds nothing in
// front of the camera), 2 given (rv / t: the n <= 5 direct EPnP solve)
struct SqpnpFitIn {
    int mode, pad;
    double R[9], t[3], rv[3];
};
// The final SQPnP fits of every sequence (sqpnp.hpp), three launches: the cost
// from the statistics `stats` of suffstats_kernel and Omega's eigenvectors (one
// wave per sequence), the SQP runs from the 18 starts (a wave per eigenvector and
// sequence, the KKT rows over lanes), the solution search replayed in order; then
// Frame::pose() of the result: pose6[s] = (rvec, tvec), pose12[s] = camera -> world
// (R^T, -R^T t) for PendingMap. obj / counts / bits: the fitted points (the
// cheirality majority test). work: sqpnp_fit_work_bytes(nseq) of device memory.
size_t sqpnp_fit_work_bytes(int nseq);
hipError_t launch_sqpnp_fit(const double* stats, const SqpnpFitIn* in, const float* obj, const int* counts, int cap,
                            const uint32_t* bits, int words_cap, int nseq, double* pose6, double* pose12, void* work,
                            hipStream_t st);
size_t bucket_scratch_ints(int img_w, int img_h, int bucket, int per_bucket, int n);
hipError_t launch_bucket(const BucketBatch& b, int nseq, int img_w, int img_h, int bucket, int per_bucket,
                         hipStream_t st);

}  // namespace svo

#define SVO_HIP(ctx, expr)                                                                   \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return svo::set_error((ctx), SVO_ERR_HIP, "%s:%d %s: %s", __FILE__, __LINE__, #expr, \
                                  hipGetErrorString(e_));                                    \
    } while (0)
