/*
 * svo_gpu.h -- C ABI of the MI355X-native ikryukov/svo front end (libsvo_gpu.so).
 *
 * This is the drop-in boundary for the four OpenCV calls the reference's
 * Tracking makes on its hot path:
 *
 *   reference call (R: = ikryukov/svo)                         replaced by
 *   ---------------------------------------------------------  ------------------------------
 *   buildOpticalFlowPyramid inside calcOpticalFlowPyrLK          svo_image_upload /
 *     R:src/tracking.cpp:101, :160                               svo_image_build_pyramid
 *   mDetector->detect(img, kps, mask)  (FastFeatureDetector)     svo_fast_detect
 *     R:src/tracking.cpp:82 (created :54-57)
 *   cv::rectangle(mask, p-(10,10), p+(10,10), 0, FILLED)         svo_mask_boxes
 *     R:src/tracking.cpp:76-79
 *   FeatureSet::bucketingFeatures  R:src/bucket.cpp:24-68        svo_bucket_features
 *   cv::calcOpticalFlowPyrLK(...)  R:src/tracking.cpp:101-105,   svo_calc_optical_flow_pyr_lk
 *     :160-165
 *   PnPRansacCallback::computeError + findInliers (inside        svo_pnp_residuals
 *     cv::solvePnPRansac, R:src/tracking.cpp:191-196)
 *   cv::solvePnPRansac(..., SOLVEPNP_SQPNP)                      svo_solve_pnp_ransac
 *     R:src/tracking.cpp:191-196
 *   cv::solvePnP(..., SOLVEPNP_SQPNP)  (solvePnPRansac's final   svo_solve_pnp_sqpnp
 *     fit on the inliers, R:src/tracking.cpp:191-196)
 *   cv::triangulatePoints + convertPointsFromHomogeneous          svo_triangulate_points
 *     R:src/tracking.cpp:125-131
 *
 * Conventions (no exceptions cross this ABI; no torch types):
 *   - Host memory is caller-owned. Device memory is owned by the context.
 *   - Every int-returning entry point returns SVO_OK (0) or a negative error
 *     class; svo_last_error(ctx) holds the message. Where OpenCV would throw a
 *     cv::Exception from CV_Assert (bad window, maxLevel < 0, < 4 PnP points),
 *     the call returns SVO_ERR_ARG and writes nothing.
 *   - One svo_ctx per (device, HIP stream, camera sequence). A context is not
 *     thread-safe; distinct contexts may be used concurrently from different
 *     threads and devices.
 *   - Points are float (x, y) pairs laid out exactly like std::vector<cv::Point2f>.
 */
#ifndef SVO_GPU_H
#define SVO_GPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SVO_OK 0
#define SVO_ERR_ARG (-1)      /* argument outside the OpenCV contract */
#define SVO_ERR_HIP (-2)      /* HIP runtime error */
#define SVO_ERR_CAPACITY (-3) /* a fixed capacity was exceeded */
#define SVO_ERR_NODEVICE (-4) /* no HIP device / extension not usable */

/* cv::TermCriteria type bits and cv::calcOpticalFlowPyrLK flags */
#define SVO_TERM_COUNT 1
#define SVO_TERM_EPS 2
#define SVO_LK_USE_INITIAL_FLOW 4
#define SVO_LK_GET_MIN_EIGENVALS 8
/* Not an OpenCV flag: sum LK's normal equations in OpenCV's own float order
 * (LKTrackerInvoker's SSE build: four float lanes + a scalar tail, then its
 * lane reduction) instead of exactly. With it the results are those of
 * cv::calcOpticalFlowPyrLK's x86 build bit for bit; without it the sums are
 * exact integers rounded once (order-independent). */
#define SVO_LK_OPENCV_ORDER 0x10000

typedef struct svo_ctx svo_ctx;
typedef struct svo_image svo_image; /* a device-resident 8U image + its pyramid */

typedef struct svo_keypoint {
    float x, y;     /* cv::KeyPoint::pt */
    float response; /* cv::KeyPoint::response (FAST score with NMS, else 0) */
} svo_keypoint;

/* ------------------------------------------------------------ context */
int svo_ctx_create(int device, svo_ctx** out);
void svo_ctx_destroy(svo_ctx* ctx);
const char* svo_last_error(const svo_ctx* ctx);
int svo_ctx_synchronize(svo_ctx* ctx);
/* Build identification, e.g. "svo_gpu gfx950 hip 7.2". */
const char* svo_version(void);

/* ------------------------------------------------------------ images / pyramids
 * An svo_image holds a W x H 8U image and up to `max_levels` pyrDown levels in
 * one device allocation (level l is ((w_{l-1}+1)/2, (h_{l-1}+1)/2), OpenCV
 * pyrDown, BORDER_REFLECT_101). The number of levels a given LK call uses is
 * clamped exactly as buildOpticalFlowPyramid clamps it for that call's window. */
int svo_image_create(svo_ctx* ctx, int w, int h, int max_levels, svo_image** out);
void svo_image_destroy(svo_ctx* ctx, svo_image* img);
/* H2D copy of level 0 (row stride in bytes) and pyramid build. */
int svo_image_upload(svo_ctx* ctx, svo_image* img, const uint8_t* gray, int stride);
/* Colour ingest (R:include/async_image_loader.h:63-69, imread + cvtColor(
 * COLOR_BGR2GRAY)): H2D of a host 8UC3 BGR image (row stride in bytes >= 3w)
 * through a pinned double buffer, grey conversion written straight into level
 * 0 (OpenCV's fixed-point weights, bit-exact), then the pyramid build. Returns
 * once the copy is queued: `bgr` may be reused immediately. */
int svo_image_upload_bgr(svo_ctx* ctx, svo_image* img, const uint8_t* bgr, int stride);
/* Rebuild levels 1..max_levels from the device-resident level 0. */
int svo_image_build_pyramid(svo_ctx* ctx, svo_image* img);
int svo_image_level_size(const svo_image* img, int level, int* w, int* h);
int svo_image_download_level(svo_ctx* ctx, const svo_image* img, int level, uint8_t* dst, int stride);
/* The Scharr derivatives of pyramid level `level` (built pyramid required) as the
 * LK kernels read them: calcSharrDeriv (inside calcOpticalFlowPyrLK,
 * R:src/tracking.cpp:101, :160) scaled by 4, int16 ix / iy of that level's w x h
 * with `stride` elements per row; either output may be null. */
int svo_image_scharr_level(svo_ctx* ctx, const svo_image* img, int level, int16_t* ix, int16_t* iy, int stride);

/* ------------------------------------------------------------ FAST
 * cv::FastFeatureDetector(threshold, nonmaxSuppression, TYPE_9_16)::detect(
 * image, keypoints, mask): keypoints in OpenCV's raster emission order, NMS
 * strict-greater over 8 neighbours, then runByPixelsMask. mask: host W*H u8
 * (row stride w) or NULL. Writes min(n, cap) keypoints; *n_out = n. */
int svo_fast_detect(svo_ctx* ctx, const svo_image* img, int threshold, int nonmax,
                    const uint8_t* mask, svo_keypoint* out, int cap, int* n_out);
/* Kernel-level view for parity tests: per-pixel FAST score (0 = no corner)
 * and corner flag, both W*H u8. */
int svo_fast_score_map(svo_ctx* ctx, const svo_image* img, int threshold,
                       uint8_t* score, uint8_t* corner);
/* ------------------------------------------------------------ ORB (detect only)
 * The reference's shipped default detector (use_orb: 1, R:configs/config.yaml:20-27):
 * cv::ORB::create(nfeatures, scaleFactor, nlevels, edgeThreshold, firstLevel, WTA_K,
 * scoreType, patchSize, fastThreshold) at R:src/tracking.cpp:33-50, used through
 * detect(img, keypoints, mask) at :82. Keypoints in OpenCV's order (level by level,
 * retainBest's order within a level), pt scaled to level 0; response = Harris (or
 * FAST) score; octave optional (may be NULL). Angles are not computed (the
 * reference keeps positions only, R:src/tracking.cpp:85). firstLevel must be 0. */
#define SVO_ORB_HARRIS_SCORE 0
#define SVO_ORB_FAST_SCORE 1
typedef struct svo_orb_params {
    int nfeatures;        /* R:configs/config.yaml:22 (150) */
    float scale_factor;   /* 1.2 */
    int nlevels;          /* 8 (<= 8) */
    int edge_threshold;   /* the reference passes patch_size (31) */
    int first_level;      /* 0 */
    int wta_k;            /* 4 (descriptors only; unused by detect) */
    int score_type;       /* SVO_ORB_HARRIS_SCORE */
    int patch_size;       /* 31 */
    int fast_threshold;   /* 20 */
} svo_orb_params;
int svo_orb_detect(svo_ctx* ctx, const svo_image* img, const svo_orb_params* params,
                   const uint8_t* mask, svo_keypoint* out, int* octave, int cap, int* n_out);

/* R:src/tracking.cpp:76-79: W*H mask of 255 with a filled box of +-half around
 * each point (cvRound corners, inclusive, clipped). Host output. */
int svo_mask_boxes(svo_ctx* ctx, int w, int h, const float* pts_xy, int n, float half,
                   uint8_t* mask);

/* ------------------------------------------------------------ bucketing
 * FeatureSet::bucketingFeatures(image(w,h), bucket_size, features_per_bucket)
 * with the reference's exact output (R:src/bucket.cpp:24-106 quirks included).
 * ages may be NULL (all 0, as appendNewFeatures sets them). */
int svo_bucket_features(svo_ctx* ctx, const float* xy, const int* ages, int n, int img_w,
                        int img_h, int bucket_size, int per_bucket, float* xy_out,
                        int* ages_out, int cap, int* n_out);

/* ------------------------------------------------------------ LK
 * cv::calcOpticalFlowPyrLK(prev, next, prevPts, nextPts, status, err,
 * Size(win_w, win_h), max_level, TermCriteria(crit_type, max_count, epsilon),
 * flags, min_eig_threshold). next_xy is read as the initial guess when
 * SVO_LK_USE_INITIAL_FLOW is set. err may be NULL. Pyramids must have been
 * built with at least the levels this window allows. */
int svo_calc_optical_flow_pyr_lk(svo_ctx* ctx, const svo_image* prev, const svo_image* next,
                                 const float* prev_xy, int n, float* next_xy,
                                 uint8_t* status, float* err, int win_w, int win_h,
                                 int max_level, int crit_type, int max_count, double epsilon,
                                 int flags, double min_eig_threshold);
/* Gauss-Newton iterations executed by the last LK call, summed over points and
 * levels (the "LK iters/s" metric numerator). */
int64_t svo_lk_last_iterations(const svo_ctx* ctx);

/* ------------------------------------------------------------ PnP
 * Batched reprojection residual: M hypotheses (R row-major 3x3, t 3: 12
 * doubles each) x N points. Equals PnPRansacCallback::computeError (projectPoints
 * with K, zero distortion, CV_32F output; err = |ipt - ppt|^2 in float) and
 * findInliers (err <= thresh2). err (M*N floats), mask (M*N bytes), counts (M)
 * may each be NULL. obj_xyz are floats (OpenCV converts Point3d to CV_32F). */
int svo_pnp_residuals(svo_ctx* ctx, const float* obj_xyz, const float* img_xy, int n,
                      const double* hyp_Rt, int m, const double K[9], float thresh2,
                      float* err, uint8_t* mask, int* counts);

/* cv::solvePnPRansac(obj(Point3d), img(Point2f), K, zeros(1,4), rvec, tvec,
 * useExtrinsicGuess=false, iterations, reproj_err, confidence, inliers,
 * SOLVEPNP_SQPNP). Returns 1 (model found), 0 (no model) or < 0 (error).
 * inliers: capacity n ints, written in ascending order. */
int svo_solve_pnp_ransac(svo_ctx* ctx, const double* obj_xyz, const float* img_xy, int n,
                         const double K[9], int iterations, float reproj_err,
                         double confidence, double rvec[3], double tvec[3], int* inliers,
                         int* n_inliers);

/* cv::solvePnP(obj(Point3d), img(Point2f), K, zeros(1,4), rvec, tvec, false,
 * SOLVEPNP_SQPNP): the fit solvePnPRansac ends with (calib3d/src/sqpnp.cpp's cost
 * and solution search; host only, no context). Returns 1 (pose found), 0
 * (SQPnP's asserts -- degenerate points -- or no solution in front of the
 * camera) or SVO_ERR_ARG (null pointers, n < 3). */
int svo_solve_pnp_sqpnp(const double* obj_xyz, const float* img_xy, int n, const double K[9], double rvec[3],
                        double tvec[3]);

/* RANSAC's minimal solver alone: SOLVEPNP_EPNP on 5 points, the model estimator
 * solvePnPRansac runs per hypothesis (R:src/tracking.cpp:191-196), for m subsets
 * given as 25 floats each (obj xyz x5, then img xy x5, as the front end gathers
 * them). device = 0: the host solver the RANSAC uses (OpenCV's epnp.cpp with its
 * Jacobi SVDs, bit-identical to the oracle's restatement; no context needed);
 * device = 1: one 64-lane wave per subset on the GPU (epnp_wave.hpp), a QL-based
 * variant kept off the path; device = 2: that variant's host twin (bit-identical
 * to device 1; no context needed); device = 3 / 4 / 5: the device = 0 solver
 * forced to its scalar / AVX2-lane / AVX-512-lane form (SVO_ERR_NODEVICE when the
 * CPU lacks the instruction set); device = 6: the device = 0 solver on the GPU, one
 * lane per subset (epnp_lane.hip; bit-identical to device 0). Rt: m x 12 doubles
 * (R row-major, t); ok: m ints (0: non-finite model). */
int svo_epnp_subsets(svo_ctx* ctx, const float* subsets, int m, const double K[9], int device, double* Rt,
                     int* ok);

/* ------------------------------------------------------------ triangulation
 * cv::triangulatePoints(P1, P2, pts1, pts2, points4D) then
 * cv::convertPointsFromHomogeneous (R:src/tracking.cpp:125-131). P1, P2: 3x4
 * row-major float (cv::Matx34f). Per point the DLT null vector of the 4x4
 * system, unit length with w >= 0 (OpenCV's sign is arbitrary and cancels),
 * rounded to float -> xyzw (4n, may be NULL); xyz = xyzw[0:3] * (1/w) in float
 * (3n, may be NULL). */
int svo_triangulate_points(svo_ctx* ctx, const float P1[12], const float P2[12], const float* pts1,
                           const float* pts2, int n, float* xyzw, float* xyz);

/* ------------------------------------------------------------ reprojection cost (§8 a11)
 * The north star's "ceres reprojection cost": Ceres is linked by the reference
 * but never called (R:CMakeLists.txt:22,33), so there is no
 * reference implementation; pinned by finite differences.
 * P problems of up to max_n points each (obj: P*max_n*3 doubles, img:
 * P*max_n*2 floats, counts: P or NULL = max_n each), poses: P x 12 doubles
 * ([R|t], world -> camera, R row-major). Per point: r = pi(K (R X + t)) - u and
 * J = dr/dxi (2x6 row-major) for T <- exp(xi^) T, xi = (rho, phi). normal:
 * P x 28 = H (upper triangle of sum w J^T J, row-major, 21), g (sum w J^T r,
 * 6), cost (sum of rho(|r|)); w, rho: Huber with delta > 0, else least
 * squares. Points behind the camera contribute 0. Outputs may be NULL;
 * results are deterministic (fixed reduction order). */
int svo_reprojection_jacobians(svo_ctx* ctx, const double* obj_xyz, const float* img_xy, const int* counts,
                               int n_problems, int max_n, const double* poses, const double K[9],
                               double huber_delta, double* res, double* jac, double* normal);
/* Host Levenberg-Marquardt over SE(3) (motion-only bundle adjustment), one
 * batched GPU evaluation per iteration for all P problems. poses: in/out.
 * costs (P, final cost) and iterations may be NULL. */
int svo_refine_poses(svo_ctx* ctx, const double* obj_xyz, const float* img_xy, const int* counts, int n_problems,
                     int max_n, const double K[9], double huber_delta, int max_iterations, double* poses,
                     double* costs, int* iterations);

/* ------------------------------------------------------------ batched front end
 * The reference's per-frame loop (Tracking::startStereo, R:src/tracking.cpp:232-276:
 * trackFrames -> calculatePose -> keyframe extractFeatures + findLeftFeaturesInRight
 * + triangulateNewMapPoints) for n_seq independent stereo sequences advanced in
 * lockstep: every kernel launch covers the whole batch, all state (left / right
 * pyramids, features, map points) stays in HBM, and only the RANSAC minimal solver
 * (EPnP) and the final SQPnP-objective fit run on the host between GPU launches.
 * A keyframe's new features are the first (n_features - n) masked FAST corners,
 * matched in the right image (stereo LK), filtered (status, |yR - yL| <
 * y_threshold), triangulated with P_left / P_right (z > 0) and moved to the world
 * frame by the frame's estimated pose. Which frames are keyframes: keyframe_rule
 * SVO_KF_EVERY (every frame, topping the set up to n_features: the benchmark's
 * upper bound) or SVO_KF_REFERENCE (Tracking::nextFrame, R:src/tracking.cpp:68-69:
 * frame 0, and a frame whose predecessor was no keyframe and kept fewer than
 * features_to_track features; it takes every masked corner, n_features being
 * the feature capacity). */
#define SVO_KF_EVERY 0
#define SVO_KF_REFERENCE 1
typedef struct svo_frontend svo_frontend;

typedef struct svo_frontend_config {
    int width, height;      /* frame size */
    int n_seq;              /* sequences per batch */
    int n_frames;           /* frames kept resident per sequence */
    int n_features;         /* features kept per frame (top-up target), e.g. 2000 */
    int max_level;          /* LK maxLevel, R:src/tracking.cpp:163 -> 3 */
    int win;                /* LK window, :163 -> 21 */
    int lk_max_count;       /* :157 -> 50 */
    double lk_epsilon;      /* :157 -> 1e-3 */
    double min_eig;         /* OpenCV default 1e-4 */
    int lk_flags;           /* :164 -> SVO_LK_GET_MIN_EIGENVALS */
    int fast_threshold;     /* R:configs/config.yaml:30 -> 20 */
    int fast_nonmax;        /* R:include/config_reader.h:37 -> 1 */
    float mask_half;        /* R:src/tracking.cpp:78 -> 10 */
    int bucket_size;        /* 0 = no bucketing (the reference never calls it) */
    int per_bucket;
    int pnp_iterations;     /* R:src/tracking.cpp:195 -> 100 */
    float pnp_reproj;       /* -> 8.0 */
    double pnp_confidence;  /* -> 0.999 */
    double K[9];            /* camera matrix (float-rounded, as the Matx33f K) */
    int host_threads;       /* RANSAC host threads; 0 = auto */
    int timing;             /* 1 = per-phase HIP events; 2 = only LK, pyramid, FAST; 3 = only LK */
    int keyframe_rule;      /* SVO_KF_EVERY (default) or SVO_KF_REFERENCE */
    int features_to_track;  /* SVO_KF_REFERENCE threshold, R:configs/config.yaml:15 -> 70 */
    /* stereo keyframe path (R:src/tracking.cpp:94-152) */
    float P_left[12];       /* mProjectionMatrixLeft (KITTI calib P2, R:src/main.cpp:25-28), row-major 3x4 */
    float P_right[12];      /* mProjectionMatrixRight (P3, :29-32) */
    float y_threshold;      /* R:configs/config.yaml:16 -> 40 */
    int stereo_win;         /* R:src/tracking.cpp:104 -> 11 */
    int stereo_max_level;   /* -> 3 */
    int stereo_max_count;   /* :97 -> 30 */
    double stereo_epsilon;  /* -> 1e-3 */
    /* keyframe detector (R:src/tracking.cpp:33-57): 0 = FAST(fast_threshold,
     * fast_nonmax); 1 = cv::ORB with `orb` (the shipped config, use_orb: 1,
     * R:configs/config.yaml:19-27) -- ORB keypoints (level-0 coordinates, level
     * order) replace FAST's as the keyframe's candidates; detected only on the
     * steps where some sequence takes a keyframe, through the serial keyframe path
     * (no speculative stereo LK, no FAST pre-detection, no bucketing) */
    int use_orb;
    svo_orb_params orb;
} svo_frontend_config;

typedef struct svo_frontend_stats {
    int64_t lk_iterations;  /* GN iterations this step (all sequences, levels) */
    int64_t tracked;        /* features with status 1 after LK */
    int64_t inliers;        /* PnP inliers kept */
    int64_t added;          /* new features from the keyframe top-up */
    int64_t features;       /* features after the step */
    int64_t hypotheses;     /* RANSAC hypotheses scored on the GPU */
    double host_ms_hyp;     /* host wall time generating hypotheses (EPnP) */
    double host_ms_fit;     /* host wall time in the final fits */
    double host_ms_wait;    /* host wall time blocked on the GPU (= the three waits below) */
    int64_t keyframes;      /* sequences whose frame was a keyframe this step */
    /* per-step diagnostics (what a slow step spent its time on) */
    double host_ms_wait_post;   /* waiting for the post-LK results (LK + compaction) */
    double host_ms_wait_score;  /* waiting for the RANSAC scoring launches, all rounds */
    double host_ms_wait_kf;     /* waiting for the keyframe at the step's end */
    double host_ms_enqueue;     /* issuing the step's launches (incl. the next front half) */
    double host_ms_step;        /* the whole call */
    int64_t ransac_rounds;      /* host <-> GPU RANSAC rounds (chunks) */
    int64_t max_hypotheses;     /* most hypotheses any one sequence scored */
    int64_t serial_keyframe;    /* 1: the speculative stereo LK missed, serial keyframe ran */
    int64_t full_copy;          /* 1: the full point copy was waited for (long RANSAC / n <= 5) */
    int64_t kf_overflow;        /* SVO_KF_REFERENCE: masked corners a keyframe left out for
                                   lack of capacity (n_features); 0 = every corner taken,
                                   as extractFeatures (R:src/tracking.cpp:74-92); with use_orb
                                   it includes the ORB keypoints its detector dropped at the
                                   candidate capacity */
    double host_ms_orb;         /* use_orb: the keyframe's ORB detection (device stages and the
                                   host's retainBest, synchronous on the FAST stream) */
    int64_t spec_margin;        /* the speculative stereo LK's margin over the expected top-up
                                   (spec_margin + the last step's largest RANSAC / LK losses) */
} svo_frontend_stats;

int svo_frontend_create(svo_ctx* ctx, const svo_frontend_config* cfg, svo_frontend** out);
void svo_frontend_destroy(svo_frontend* fe);
/* Stereo pair t of sequence seq (left / right grey, same stride): level-0 uploads
 * (H2D, untimed; R:include/async_image_loader.h:57-69 delivers the pair). */
int svo_frontend_set_frame(svo_frontend* fe, int seq, int t, const uint8_t* left, const uint8_t* right,
                           int stride);
/* Same from BGR 8UC3 frames (svo_image_upload_bgr's conversion). */
int svo_frontend_set_frame_bgr(svo_frontend* fe, int seq, int t, const uint8_t* left_bgr,
                               const uint8_t* right_bgr, int stride);
/* Streamed frames (R:include/async_image_loader.h:36-69: the loader hands each
 * stereo pair to Tracking as it arrives; here a whole step's worth at once):
 * queue frame t of every sequence -- left[s] / right[s] (grey, or BGR 8UC3 when
 * bgr != 0: cv::cvtColor(BGR2GRAY) on the device), rows `stride` bytes apart --
 * as asynchronous H2D copies on the front end's upload stream into ring slot
 * t % n_frames, converted into level 0 there; frame t's pyramid builds wait for
 * it. Returns at once: the host buffers must stay untouched until
 * svo_frontend_upload_wait(fe, t) (page-locked memory, svo_pinned_alloc, gives
 * full PCIe rate; sequences whose buffers follow each other in memory go in one
 * copy). Ring discipline (n_frames >= 4): before init, any frame; after it,
 * frame t is queued before step t - 2 is called (t >= last step + 3) and no
 * earlier than step t - n_frames + 1 returned (t <= last step + n_frames - 1):
 * a loop queues frames 0 .. 2, calls init(0), then queue(t + 2), step(t). A frame
 * at or before the last step restarts the loop (everything queued is finished and
 * forgotten; queue frames t0 .. t0 + 2 and init(t0) again). set_frame(seq, t)
 * after streaming makes slot t hold frame t, resident. The copy into a slot waits
 * on the device for the last read of the slot's previous frame. */
int svo_frontend_queue_frames(svo_frontend* fe, int t, const uint8_t* const* left, const uint8_t* const* right,
                              int stride, int bgr);
int svo_frontend_upload_wait(svo_frontend* fe, int t);
int svo_pinned_alloc(size_t bytes, void** out);
void svo_pinned_free(void* p);
/* Build every resident frame's pyramid now (else each step builds its own). */
int svo_frontend_prebuild_pyramids(svo_frontend* fe);
/* First keyframe: FAST (+bucket) on frame t0 of every sequence, map points. */
int svo_frontend_init(svo_frontend* fe, int t0);
/* One step: frame t-1 -> t for every sequence (pyramid of t, temporal LK,
 * compaction, PnP RANSAC, outlier removal, masked FAST top-up). */
int svo_frontend_step(svo_frontend* fe, int t, svo_frontend_stats* stats);
/* Wait for every stream of the front end (a step returns with the next frame's
 * pyramid and the pose statistics still running) and finish the pose fits. */
int svo_frontend_synchronize(svo_frontend* fe);
int svo_frontend_pose(svo_frontend* fe, int seq, double rvec[3], double tvec[3]);
int svo_frontend_features(svo_frontend* fe, int seq, float* xy, int cap, int* n);
/* World positions (MapPoint::mWorldPos) of the current features' map points, in
 * feature order (synchronises the front end first). */
int svo_frontend_map_points(svo_frontend* fe, int seq, double* xyz, int cap, int* n);
/* Accumulated per-phase device time (ms) and launch counts since create/reset:
 * phases: 0 pyramid (left + Scharr), 1 lk, 2 post_lk, 3 stereo_lk, 4 pnp_score,
 * 5 tail (keyframe), 6 fast, 7 bucket, 8 append, 9 pyramid_right. Returns the number
 * of phases. */
int svo_frontend_phase_times(svo_frontend* fe, double* ms, int64_t* launches, int cap);
void svo_frontend_reset_times(svo_frontend* fe);
/* The Scharr derivatives (svo_image_scharr_level's layout) of frame t of sequence
 * seq as the front end's fused pyrDown + Scharr pass built them; frame t must be
 * one of the last three frames whose pyramid was built (the derivative pyramids
 * are triple-buffered): after svo_frontend_init(t0) frame t0, after
 * svo_frontend_step(t) frames t and t + 1. Synchronises the front end first. */
int svo_frontend_scharr_level(svo_frontend* fe, int seq, int t, int level, int16_t* ix, int16_t* iy, int stride);
/* Level `level` of frame t's left (right = 0) or right (right = 1) pyramid with
 * its stored REFLECT_101 border: (h + 2 * SVO_PYR_PAD) rows of (w + 2 *
 * SVO_PYR_PAD) bytes at `stride`, pixel (0, 0) of the level at row / column
 * SVO_PYR_PAD (the LK kernels read the border instead of testing coordinates).
 * Same frames as svo_frontend_scharr_level (right: the frame of the last step or
 * init). Synchronises the front end first. */
#define SVO_PYR_PAD 32
int svo_frontend_pyramid_level(svo_frontend* fe, int seq, int t, int right, int level, uint8_t* out, int stride);
/* The pyramid + Scharr launch chain of frame t (every sequence) timed alone on the
 * context stream: reps rebuilds (identical contents) after one warm-up, HIP
 * events around them; ms per chain. Synchronises the front end first. */
int svo_frontend_time_pyramid(svo_frontend* fe, int t, int reps, double* ms_per_launch);
/* The front end's FAST detection of frame t (every sequence; FAST-9 + cornerScore +
 * NMS without the box mask, i.e. the pre-detection stage: extractFeatures' detector,
 * R:src/tracking.cpp:82) timed alone the same way; ms per launch (row-count reset +
 * detection kernel). Synchronises the front end first; the next step re-detects. */
int svo_frontend_time_fast(svo_frontend* fe, int t, int reps, double* ms_per_launch);

/* Host cores for a front end's RANSAC / pose-fit pool when several ranks (one
 * process per GPU) share a node: this process's allowed CPUs ordered by NUMA
 * node are split among the local ranks, each rank taking its share of the node
 * its GPU sits on (gpu_node[r] = NUMA node of local rank r's GPU, or null to
 * split the whole ordered list by rank). Writes at most cap CPU ids to cpus and
 * their count to n; the sets of distinct local ranks are disjoint whenever the
 * node has at least one CPU per rank. svo_frontend_create pins its pool with
 * this plan (LOCAL_RANK / LOCAL_WORLD_SIZE from the environment, as
 * torch.distributed.run sets them) and sizes it to the set (at most 16). */
int svo_host_cpu_plan(int local_rank, int local_world, const int* gpu_node, int* cpus, int cap, int* n);
/* The CPUs a front end's pool threads are pinned to (empty: not pinned). */
int svo_frontend_host_cpus(svo_frontend* fe, int* cpus, int cap, int* n);
/* The HIP streams a front end runs on (LK, FAST, copies; hipStream_t as void*):
 * the context's, shared by every front end created on it, so a long-lived
 * process that creates and destroys front ends binds one fixed set of hardware
 * queues. */
int svo_frontend_streams(svo_frontend* fe, void** streams, int cap, int* n);
/* Self-test of the front end's host pool (no GPU): `jobs` jobs of changing sizes
 * with primes between them on `threads` threads; *bad = tasks run other than
 * exactly once, or after their job returned (0 when the pool is correct). */
int svo_pool_selftest(int threads, int jobs, int64_t* bad);

#ifdef __cplusplus
}
#endif
#endif /* SVO_GPU_H */
