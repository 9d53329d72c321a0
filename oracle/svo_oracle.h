/*
 * svo_oracle.h -- CPU restatement of the OpenCV algorithms on the ikryukov/svo
 * front-end hot path.
 *
 * *** TEST INFRASTRUCTURE ONLY. ***
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library, and only as the checker / CPU baseline -- never as the thing
 * measured or shipped. The product (svo_amd/, libsvo_gpu.so) never links it.
 *
 * PARITY STATUS: "parity unpinned" against the reference's own results.
 *   The reference (R: = /root/reference) has no tests, no fixtures and no golden
 *   vectors, and every line of its pixel arithmetic lives in OpenCV >= 4.0
 *   (R:CMakeLists.txt:9), which is absent from this image.
 *   The restatement below follows upstream OpenCV 4.x semantics function by
 *   function (file names cited per function). It is pinned only by analytic
 *   known-answer tests (tests/test_oracle_kat.py): pyrDown of constant/ramp
 *   images, hand-built FAST rings, LK on exact sub-pixel translations, RANSAC on
 *   exact correspondences + far outliers, bucket selection on hand-listed points.
 *
 * Reference call sites each oracle entry point restates:
 *   svo_oracle_bgr2gray       <- cv::cvtColor(COLOR_BGR2GRAY), R:include/async_image_loader.h:68-69
 *   svo_oracle_build_pyramid  <- cv::buildOpticalFlowPyramid inside
 *                                cv::calcOpticalFlowPyrLK, R:src/tracking.cpp:101,160
 *   svo_oracle_lk             <- cv::calcOpticalFlowPyrLK,  R:src/tracking.cpp:101-105,160-165
 *   svo_oracle_fast           <- cv::FastFeatureDetector::detect, R:src/tracking.cpp:54-57,82
 *   svo_oracle_orb_detect     <- cv::ORB::detect (use_orb: 1), R:src/tracking.cpp:33-50,82
 *   svo_oracle_mask_boxes     <- cv::rectangle(mask,...,FILLED), R:src/tracking.cpp:76-79
 *   svo_oracle_bucket         <- FeatureSet::bucketingFeatures, R:src/bucket.cpp:24-106
 *   svo_oracle_pnp_*          <- cv::solvePnPRansac(...,SOLVEPNP_SQPNP), R:src/tracking.cpp:191-196
 */
#ifndef SVO_ORACLE_H
#define SVO_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- ingest */

/* cv::cvtColor(COLOR_BGR2GRAY) on 8UC3 (R:include/async_image_loader.h:68-69):
 * gray is w*h, row stride w. */
void svo_oracle_bgr2gray(const uint8_t* bgr, int w, int h, int stride, uint8_t* gray);

/* ---------------------------------------------------------------- pyramid */

/* OpenCV modules/imgproc/src/pyramids.cpp pyrDown_ (8U): dst ((w+1)/2,(h+1)/2),
 * separable [1 4 6 4 1]^2, (s+128)>>8, BORDER_REFLECT_101. */
void svo_oracle_pyr_down(const uint8_t* src, int w, int h, int sstride,
                         uint8_t* dst, int dstride);

/* OpenCV modules/video/src/lkpyramid.cpp buildOpticalFlowPyramid (withDerivatives
 * = false). Returns the number of levels actually built minus one (the returned
 * maxLevel); writes level sizes into lw/lh (arrays of max_level+1). Levels are
 * written tightly packed (stride = width) into `out` back to back, level 0 first. */
int svo_oracle_pyramid_levels(int w, int h, int win_w, int win_h, int max_level,
                              int* lw, int* lh);
int svo_oracle_build_pyramid(const uint8_t* img, int w, int h, int stride,
                             int win_w, int win_h, int max_level, uint8_t* out);

/* lkpyramid.cpp calcSharrDeriv: int16 interleaved (Ix, Iy) per pixel. */
void svo_oracle_scharr(const uint8_t* src, int w, int h, int stride, int16_t* dst);

/* ---------------------------------------------------------------- LK */

/* How the LK normal-equation sums are accumulated.
 *  EXACT  : integer products summed exactly (int64), rounded to float once.
 *           This is what the HIP kernel does (order-independent, so a wave
 *           reduction reproduces it bit for bit).
 *  SCALAR : OpenCV's scalar loop, float accumulator (acctype=float, x86/aarch64).
 *  SSE    : OpenCV's CV_SIMD128 (x86) path summation order.
 * All three use identical integer sampling; they differ only in the rounding of
 * the A/b sums (relative ~1e-7), which the tests bound far below 0.1 px. */
enum { SVO_ORACLE_ACC_EXACT = 0, SVO_ORACLE_ACC_SCALAR = 1, SVO_ORACLE_ACC_SSE = 2 };
/* or-ed into acc_mode: iters_out receives (max_level + 1) x npts per-level counts (row = level) */
#define SVO_ORACLE_LEVEL_ITERS 0x100

#define SVO_ORACLE_LK_GET_MIN_EIGENVALS 8   /* cv::OPTFLOW_LK_GET_MIN_EIGENVALS */
#define SVO_ORACLE_LK_USE_INITIAL_FLOW  4   /* cv::OPTFLOW_USE_INITIAL_FLOW */
#define SVO_ORACLE_TERM_COUNT 1             /* cv::TermCriteria::COUNT */
#define SVO_ORACLE_TERM_EPS   2             /* cv::TermCriteria::EPS */

/* cv::calcOpticalFlowPyrLK on two 8U images (pyramids are built internally,
 * exactly as the reference's calls do). prev/next points are float (x,y) pairs.
 * err may be NULL. Returns the maxLevel used, or -1 on bad arguments. */
int svo_oracle_lk(const uint8_t* prev, const uint8_t* next, int w, int h, int stride,
                  const float* prev_xy, float* next_xy, uint8_t* status, float* err,
                  int npts, int win_w, int win_h, int max_level,
                  int crit_type, int max_count, double epsilon,
                  int flags, double min_eig_threshold, int acc_mode,
                  int* iters_out /* optional: GN iterations per point, summed over levels */);

/* ---------------------------------------------------------------- FAST */

/* features2d/src/fast.cpp FAST_t<16> + cornerScore<16> + KeyPointsFilter::
 * runByPixelsMask. mask may be NULL (W*H u8, row stride = w). Writes up to `cap`
 * keypoints as (x, y, response) float triples in OpenCV's emission order. Returns
 * the total number of keypoints (may exceed cap). */
int svo_oracle_fast(const uint8_t* img, int w, int h, int stride, int threshold,
                    int nonmax, const uint8_t* mask, float* kp_xyr, int cap);

/* FAST corner score map only (0 = not a corner), for kernel-level parity:
 * score[y*w+x] = cornerScore if (x,y) is a FAST-9 corner in the detection area,
 * else 0; corner[y*w+x] = 1 if it is a corner. */
void svo_oracle_fast_score(const uint8_t* img, int w, int h, int stride, int threshold,
                           uint8_t* score, uint8_t* corner);

/* R:src/tracking.cpp:76-79: W*H mask = 255, then cv::rectangle(mask, p-(h,h),
 * p+(h,h), 0, FILLED) for every point (Point2f -> Point via cvRound). */
void svo_oracle_mask_boxes(int w, int h, const float* pts_xy, int n, float half,
                           uint8_t* mask);

/* ---------------------------------------------------------------- ORB (orb.cpp) */

/* imgproc resize(src, dst, (dw, dh), 0, 0, INTER_LINEAR_EXACT) on 8UC1. */
void svo_oracle_resize_linear_exact(const uint8_t* src, int sw, int sh, int sstride, uint8_t* dst, int dw, int dh,
                                    int dstride);
/* ORB level geometry: sizes, float scales and nfeaturesPerLevel. */
void svo_oracle_orb_level_info(int w, int h, float scale_factor, int nlevels, int nfeatures, int* lw, int* lh,
                               float* lscale, int* nper);
/* cv::ORB::create(nfeatures, scale_factor, nlevels, edge_threshold, 0, 4,
 * harris_score ? HARRIS_SCORE : FAST_SCORE, patch_size, fast_threshold)
 * ->detect(img, kps, mask). Writes up to cap (x, y, response) triples and
 * octaves (may be NULL); returns the keypoint count. */
int svo_oracle_orb_detect(const uint8_t* img, int w, int h, int stride, const uint8_t* mask, int nfeatures,
                          float scale_factor, int nlevels, int edge_threshold, int patch_size, int fast_threshold,
                          int harris_score, float* kp_xyr, int* octave, int cap);

/* ---------------------------------------------------------------- bucket */

/* R:src/bucket.cpp:24-106 (compat: stride-nw aliasing, slot-0 overwrite).
 * Returns number of points written (<= cap; total returned via n_total). */
int svo_oracle_bucket(const float* xy, const int* ages, int n, int img_w, int img_h,
                      int bucket_size, int per_bucket, float* xy_out, int* ages_out,
                      int cap, int* n_total);

/* ---------------------------------------------------------------- PnP */

/* cv::RNG (core/include/opencv2/core/operations.hpp): MWC, state (uint64). */
uint32_t svo_oracle_rng_next(uint64_t* state);

/* cv::Rodrigues (vector -> matrix), calib3d/src/calibration.cpp. */
void svo_oracle_rodrigues(const double rvec[3], double R[9]);
/* matrix -> vector. */
void svo_oracle_rodrigues_inv(const double R[9], double rvec[3]);

/* PnPRansacCallback::computeError + findInliers for M hypotheses given as
 * (R row-major 9, t 3) doubles = 12 per hypothesis. obj is float xyz (OpenCV
 * converts the Point3d input to CV_32F), img float xy. K is the 3x3 camera
 * matrix (as double, from the reference's Matx33f). err (M*n floats) optional.
 * inlier mask: M*n bytes. counts: M ints. */
void svo_oracle_pnp_residuals(const float* obj_xyz, const float* img_xy, int n,
                              const double* hyp_Rt, int m, const double K[9],
                              float thresh2, float* err, uint8_t* mask, int* counts);

/* calib3d/src/epnp.cpp (EPnP on n >= 4 points, pixels + K). Returns 0 on ok. */
int svo_oracle_epnp(const float* obj_xyz, const float* img_xy, int n, const double K[9],
                    double R[9], double t[3]);

/* calib3d/src/ptsetreg.cpp RANSACUpdateNumIters. */
int svo_oracle_ransac_update_num_iters(double p, double ep, int model_points, int max_iters);

/* cv::solvePnPRansac(obj(Point3d), img(Point2f), K, zeros(1,4), rvec, tvec,
 * false, iters, reproj, confidence, inliers, SOLVEPNP_SQPNP) -- RANSAC stage
 * (EPnP minimal kernel, 5-point subsets, cv::RNG(-1)) exactly; the final
 * solvePnP(SQPNP) on the inliers by svo_oracle_sqpnp (sqpnp.c). Returns 1 on
 * success, 0 if RANSAC found no model, -1 on bad args (< 4 points).
 * inlier_mask: n bytes. n_hyp_out: hypotheses evaluated. */
int svo_oracle_solve_pnp_ransac(const double* obj_xyz_d, const float* img_xy, int n,
                                const double K[9], int iterations, float reproj_err,
                                double confidence, double rvec[3], double tvec[3],
                                uint8_t* inlier_mask, int* n_inliers, int* n_hyp_out);

/* calib3d/src/sqpnp.cpp PoseSolver::solve (sqpnp.c): pw n x 3 object points,
 * q n x 2 normalised image points (undistortPoints with K, zero distortion);
 * the first (smallest-error) solution. Returns 0 on ok, -1 when SQPnP asserts
 * (point variance, rank) or finds no solution with positive depth. */
int svo_oracle_sqpnp(const double* pw, const double* q, int n, double R[9], double t[3]);

/* Subset draw of RANSACPointSetRegistrator::getSubset (modelPoints 5, no
 * checkSubset): draws `k` distinct indices in [0,count). Returns 1 if found. */
int svo_oracle_get_subset(uint64_t* rng_state, int count, int k, int* idx);

/* Threads for the LK point loop (OpenMP, like OpenCV's parallel_for_). */
void svo_oracle_set_threads(int n);

/* cv::triangulatePoints + cv::convertPointsFromHomogeneous (triangulate.c). */
void svo_oracle_triangulate(const float P1[12], const float P2[12], const float* pts1, const float* pts2,
                            int n, float* xyzw, float* xyz);

#ifdef __cplusplus
}
#endif
#endif
