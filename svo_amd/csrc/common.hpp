// Shared host/device definitions for libsvo_gpu.so (MI355X / gfx950).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "svo_gpu.h"

namespace svo {

constexpr int kMaxLevels = 8;  // pyramid levels kept per image (0..7)

// One pyramid level in HBM: tightly pitched u8 rows (pitch multiple of 64 B).
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
    svo_scratch s[8];
    void* pinned = nullptr;
    size_t pinned_bytes = 0;
};

namespace svo {

int set_error(svo_ctx* ctx, int code, const char* fmt, ...);
// Grow scratch slot `slot` to >= bytes; returns device pointer or nullptr.
void* scratch(svo_ctx* ctx, int slot, size_t bytes);
void* pinned(svo_ctx* ctx, size_t bytes);

// Kernel launchers (implemented in the .hip files).
hipError_t launch_pyramid(const svo_image* img, int first_level, hipStream_t st);
hipError_t launch_fast_score(const ImgLevel& L, int threshold, int nonmax, uint16_t* cs,
                             hipStream_t st);
hipError_t launch_fast_collect(const ImgLevel& L, const uint16_t* cs, int nonmax,
                               const uint8_t* mask, int* rowcnt, svo_keypoint* out, int cap,
                               int* n_out, hipStream_t st);
hipError_t launch_mask_boxes(int w, int h, const float* pts, int n, float half, uint8_t* mask,
                             hipStream_t st);

struct LKParams {
    int win_w, win_h;
    int max_level;  // effective (already clamped)
    int max_count;
    double eps2;
    int flags;
    float min_eig;
    int want_err;
};
// Single-sequence LK over device arrays.
hipError_t launch_lk(const PyrDesc& prev, const PyrDesc& next, const float* prev_xy, float* next_xy,
                     uint8_t* status, float* err, int* iters, int n, const LKParams& p,
                     hipStream_t st);
bool lk_supported(int win_w, int win_h);

hipError_t launch_pnp_residuals(const float* obj, const float* img, int n, const double* hyp,
                                int m, double fx, double fy, double cx, double cy, float thresh2,
                                float* err, uint32_t* bits, int* counts, hipStream_t st);

hipError_t launch_bucket(const float* xy, const int* ages, int n, int img_w, int img_h,
                         int bucket, int per_bucket, float* xy_out, int* ages_out, int cap,
                         int* n_out, int* scratch_counts, hipStream_t st);

}  // namespace svo

#define SVO_HIP(ctx, expr)                                                                   \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return svo::set_error((ctx), SVO_ERR_HIP, "%s:%d %s: %s", __FILE__, __LINE__, #expr, \
                                  hipGetErrorString(e_));                                    \
    } while (0)
