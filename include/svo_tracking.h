/*
 * svo_tracking.h -- C ABI of the host Tracking mirror (libsvo_tracking.so).
 *
 * libsvo_tracking.so is the reference's Frame / Feature / Map / Tracking
 * (R:include/tracking.h, frame.h, feature.h, map.h) rebuilt in C++ on top of
 * libsvo_gpu.so (the headers under include/svo/ are its C++ API). This C shim lets non-C++
 * callers (the parity tests) drive it frame by frame: push stereo pairs (the
 * AsyncImageLoader's role), step the startStereo loop, read back the frame's
 * features, pose and a per-stage trace.
 */
#ifndef SVO_TRACKING_H
#define SVO_TRACKING_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct svo_tracking svo_tracking;

typedef struct svo_tracking_config {
    int fast_threshold;      /* R:configs/config.yaml:30 -> 20 */
    int fast_nonmax;         /* R:include/config_reader.h:37 -> 1 */
    float y_threshold;       /* R:configs/config.yaml:16 -> 40 */
    int features_to_track;   /* R:configs/config.yaml:17 -> 70 */
    int device;
    /* detector choice, R:configs/config.yaml:20-27 (use_orb: 1 ships) */
    int use_orb;
    int orb_nfeatures;       /* 150 */
    float orb_scale_factor;  /* 1.2 */
    int orb_pyr_levels;      /* 8 */
    int orb_patch_size;      /* 31 (also the edge threshold) */
    int orb_fast_threshold;  /* 20 */
} svo_tracking_config;

/* calib: P0 then P1, 3x4 row-major floats (R:src/main.cpp:25-32). */
int svo_tracking_create(const svo_tracking_config* cfg, const float calib[24], svo_tracking** out);
void svo_tracking_destroy(svo_tracking* tr);
const char* svo_tracking_last_error(const svo_tracking* tr);
/* Queue one rectified stereo pair (8-bit gray, w x h, row stride in bytes). */
int svo_tracking_push_stereo(svo_tracking* tr, const uint8_t* left, const uint8_t* right, int w, int h,
                             int stride);
/* Same from colour frames (8UC3 BGR, row stride in bytes >= 3w): the loader's
 * cvtColor(COLOR_BGR2GRAY) runs on the device as the frame is uploaded. */
int svo_tracking_push_stereo_bgr(svo_tracking* tr, const uint8_t* left, const uint8_t* right, int w, int h,
                                 int stride);
/* First call: the initial keyframe (extractFeatures + triangulateNewMapPoints);
 * later calls: one iteration of startStereo's loop. Returns 1 if a frame was
 * processed, 0 if no frame was queued, < 0 on error (message in last_error). */
int svo_tracking_step(svo_tracking* tr);
/* The frame the last step produced: ID, keyframe flag, feature count, map size,
 * inlier ratio, pose (camera -> world: R row-major then t, 12 doubles). */
int svo_tracking_frame_info(const svo_tracking* tr, int64_t* frame_id, int* is_keyframe, int64_t* n_features,
                            int64_t* n_map_points, double* inlier_ratio, double pose[12]);
/* Its left features: positions (2n floats), map point world positions (3n
 * doubles) and map point IDs (n); any output may be NULL. *n = count. */
int svo_tracking_features(const svo_tracking* tr, float* xy, double* world, int64_t* mp_ids, int cap, int* n);
/* Per-stage trace of the last step. field: "lk_prev", "lk_next" (2 f32 per
 * point), "lk_status" (u8), "pnp_obj" (3 f64), "pnp_img" (2 f32),
 * "pnp_inliers" (i32), "pnp_pose" (rvec, tvec: 6 f64, then ok as f64),
 * "mask_pts", "kps", "stereo_right", "kept_left", "kept_right" (2 f32),
 * "stereo_status" (u8), "tri_xyz" (3 f32). Copies min(size, cap_bytes) bytes
 * into dst (may be NULL) and returns the field's size in bytes, < 0 if the
 * field is unknown. */
int64_t svo_tracking_trace(const svo_tracking* tr, const char* field, void* dst, int64_t cap_bytes);

#ifdef __cplusplus
}
#endif
#endif /* SVO_TRACKING_H */
