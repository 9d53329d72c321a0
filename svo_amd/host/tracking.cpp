// Tracking — R:src/tracking.cpp restated on top of the C ABI (include/svo_gpu.h).
// Each method keeps the reference's order of operations and parameters; each
// OpenCV call is replaced by its libsvo_gpu drop-in.
#include "svo/tracking.hpp"

#include <chrono>
#include <cmath>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <unordered_set>

#include "svo_gpu.h"

namespace svo {

namespace {

constexpr int kMaxLevel = Tracking::kImageLevels;  // maxLevel of both LK calls, R:src/tracking.cpp:104,163
// Both LK calls sum in OpenCV's own float order: the drop-in returns what
// cv::calcOpticalFlowPyrLK returns, bit for bit (the batched front end keeps the
// exact sums by default).
constexpr int kLkOrder = SVO_LK_OPENCV_ORDER;

[[noreturn]] void fail(svo_ctx* ctx, const char* what) {
    throw std::runtime_error(std::string(what) + ": " + (ctx ? svo_last_error(ctx) : "no context"));
}

// cv::Rodrigues (vector -> matrix), double.
void rodrigues(const double r[3], double R[9]) {
    const double th = std::sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    if (th < 2.220446049250313e-16) {
        for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0);
        return;
    }
    const double c = std::cos(th), s = std::sin(th), c1 = 1. - c;
    const double x = r[0] / th, y = r[1] / th, z = r[2] / th;
    const double rrt[9] = {x * x, x * y, x * z, x * y, y * y, y * z, x * z, y * z, z * z};
    const double rx[9] = {0, -z, y, z, 0, -x, -y, x, 0};
    for (int i = 0; i < 9; i++) R[i] = c * (i % 4 == 0) + c1 * rrt[i] + s * rx[i];
}

}  // namespace

void QueueImageSource::push(GrayImage left, GrayImage right) {
    std::lock_guard<std::mutex> g(mMutex);
    mQueue.emplace_back(std::move(left), std::move(right));
}

bool QueueImageSource::get(GrayImage& left, GrayImage& right) {
    std::lock_guard<std::mutex> g(mMutex);
    if (mQueue.empty()) return false;
    left = std::move(mQueue.front().first);
    right = std::move(mQueue.front().second);
    mQueue.pop_front();
    return true;
}

size_t QueueImageSource::size() const {
    std::lock_guard<std::mutex> g(mMutex);
    return mQueue.size();
}

void TrackingTrace::clear() { *this = TrackingTrace(); }

// R:src/tracking.cpp:22-58
Tracking::Tracking(const Config& config, Map& map, const std::vector<float>& c, ImageSource& source)
    : prevFrame(nullptr), currFrame(nullptr), lastFrameID(0), mImageLoader(source), mConfig(config), mMap(map),
      inlierRatio(0) {
    if (c.size() < 24) throw std::invalid_argument("Tracking: calib_data needs P0 and P1 (24 floats)");
    for (int i = 0; i < 12; i++) {
        mProjectionMatrixLeft[i] = c[i];
        mProjectionMatrixRight[i] = c[12 + i];
    }
    const int kidx[9] = {0, 1, 2, 4, 5, 6, 8, 9, 10};  // K(c[0], c[1], c[2], c[4], ...) as Matx33f
    for (int i = 0; i < 9; i++) K[i] = (double)c[kidx[i]];
    if (svo_ctx_create(config.device, &mGpu) != SVO_OK) {
        mGpu = nullptr;
        throw std::runtime_error("Tracking: no usable HIP device (libsvo_gpu)");
    }
}

Tracking::~Tracking() {
    // frames not handed to the Map yet
    if (currFrame && currFrame != prevFrame) delete currFrame;
    if (prevFrame) delete prevFrame;
    prevFrame = currFrame = nullptr;
    if (mGpu) svo_ctx_destroy(mGpu);
}

// R:src/tracking.cpp:61-72
StereoFrame* Tracking::nextFrame() {
    GrayImage imageLeft, imageRight;
    if (!mImageLoader.get(imageLeft, imageRight)) {
        if (mConfig.verbose && (int)lastFrameID != mConfig.end_frame)
            std::printf("-! Error reading frame #%zu\n", lastFrameID);
        return nullptr;
    }
    const bool isKeyFrame =
        (lastFrameID == 0) ||
        (!prevFrame->isKeyFrame() && prevFrame->countPts() < (size_t)mConfig.tracking.features_to_track);
    return new StereoFrame(lastFrameID++, isKeyFrame, std::move(imageLeft), std::move(imageRight));
}

// R:src/tracking.cpp:74-92
void Tracking::extractFeatures(StereoFrame* frame) {
    GrayImage& img = frame->leftImg();
    // mask to not detect same features again: svo_mask_boxes == cv::rectangle(FILLED) per feature
    const std::vector<Point2f> prevPts = prevFrame->leftPoints();
    std::vector<uint8_t> mask((size_t)img.cols() * img.rows());
    if (svo_mask_boxes(mGpu, img.cols(), img.rows(), reinterpret_cast<const float*>(prevPts.data()),
                       (int)prevPts.size(), 10.f, mask.data()) != SVO_OK)
        fail(mGpu, "svo_mask_boxes");

    svo_image* dimg = img.device(mGpu, kMaxLevel);
    std::vector<svo_keypoint> keypoints(1 << 15);
    int n = 0;
    for (;;) {
        if (mConfig.use_orb) {
            // R:src/tracking.cpp:33-50: ORB(nfeatures, scale_factor, pyr_levels,
            // edge_threshold = patch_size, first_level 0, WTA_K 4, HARRIS_SCORE,
            // patch_size, fast_treshold)
            svo_orb_params op{mConfig.orb_params.nfeatures, mConfig.orb_params.scale_factor,
                              mConfig.orb_params.pyr_levels, mConfig.orb_params.patch_size, 0, 4,
                              SVO_ORB_HARRIS_SCORE, mConfig.orb_params.patch_size,
                              mConfig.orb_params.fast_treshold};
            if (svo_orb_detect(mGpu, dimg, &op, mask.data(), keypoints.data(), nullptr, (int)keypoints.size(), &n) !=
                SVO_OK)
                fail(mGpu, "svo_orb_detect");
        } else if (svo_fast_detect(mGpu, dimg, mConfig.fast_params.threshold,
                                   mConfig.fast_params.nonMaxSuppression ? 1 : 0, mask.data(), keypoints.data(),
                                   (int)keypoints.size(), &n) != SVO_OK) {
            fail(mGpu, "svo_fast_detect");
        }
        if (n <= (int)keypoints.size()) break;
        keypoints.resize((size_t)n);
    }
    std::vector<Point2f> newPoints;  // cv::KeyPoint::convert
    newPoints.reserve((size_t)n);
    for (int i = 0; i < n; i++) newPoints.emplace_back(keypoints[i].x, keypoints[i].y);

    if (mTrace) {
        mTrace->mask_pts = prevPts;
        mTrace->kps = newPoints;
    }
    frame->setFeatures(Feature::FromPoints(newPoints), {});
    findLeftFeaturesInRight(frame);
}

// R:src/tracking.cpp:94-118
void Tracking::findLeftFeaturesInRight(StereoFrame* frame) const {
    std::vector<Feature::Ptr> newLeftFeatures, newRightFeatures;
    const std::vector<Point2f> leftPoints = frame->leftPoints();
    const size_t n = leftPoints.size();
    std::vector<Point2f> rightPoints(n);
    std::vector<uint8_t> status(n);
    std::vector<float> error(n);
    if (n > 0 &&
        svo_calc_optical_flow_pyr_lk(mGpu, frame->leftImg().device(mGpu, kMaxLevel),
                                     frame->rightImg().device(mGpu, kMaxLevel),
                                     reinterpret_cast<const float*>(leftPoints.data()), (int)n,
                                     reinterpret_cast<float*>(rightPoints.data()), status.data(), error.data(), 11,
                                     11, kMaxLevel, SVO_TERM_COUNT | SVO_TERM_EPS, 30, 0.001, kLkOrder, 1e-4) != SVO_OK)
        fail(mGpu, "svo_calc_optical_flow_pyr_lk (stereo)");

    newLeftFeatures.reserve(n);
    newRightFeatures.reserve(n);
    for (size_t i = 0; i < n; ++i) {
        if (status[i] &&
            (std::abs(rightPoints[i].y - frame->leftFeatures()[i]->pos.y) < mConfig.tracking.y_threshold)) {
            newLeftFeatures.push_back(frame->leftFeatures()[i]);
            newRightFeatures.push_back(Feature::Create(rightPoints[i], frame->leftFeatures()[i]->mapPoint));
        }
    }
    if (mTrace) {
        mTrace->stereo_right = rightPoints;
        mTrace->stereo_status = status;
    }
    // We will keep in left only features that was found in right
    frame->setFeatures(std::move(newLeftFeatures), std::move(newRightFeatures));
    if (mTrace) {
        mTrace->kept_left = frame->leftPoints();
        mTrace->kept_right = frame->rightPoints();
    }
}

// R:src/tracking.cpp:120-152
void Tracking::triangulateNewMapPoints(StereoFrame* frame) {
    const std::vector<Point2f> lp = frame->leftPoints(), rp = frame->rightPoints();
    std::vector<Point3f> pointsWorld(lp.size());
    if (!lp.empty() &&
        svo_triangulate_points(mGpu, mProjectionMatrixLeft, mProjectionMatrixRight,
                               reinterpret_cast<const float*>(lp.data()), reinterpret_cast<const float*>(rp.data()),
                               (int)lp.size(), nullptr, reinterpret_cast<float*>(pointsWorld.data())) != SVO_OK)
        fail(mGpu, "svo_triangulate_points");
    if (mTrace) mTrace->tri_xyz = pointsWorld;

    std::vector<Feature::Ptr> newLeftFeatures;
    newLeftFeatures.reserve(frame->countPts());
    for (size_t i = 0; i < pointsWorld.size(); ++i) {
        const auto& p_w = pointsWorld[i];
        if (p_w.z > 0) {
            const Point3d p = frame->pose() * Point3d{p_w.x, p_w.y, p_w.z};  // Transform point
            const auto& leftFeature = frame->leftFeatures()[i];
            auto mp = mMap.createMapPoint(p);
            mp->addObservation(frame->ID, leftFeature);  // Add observation from left img
            leftFeature->mapPoint = mp;
            newLeftFeatures.push_back(leftFeature);
        }
    }
    // Remove right features, we don't need them after triangulation
    frame->setFeatures(std::move(newLeftFeatures), {});
}

// R:src/tracking.cpp:154-179
void Tracking::trackFrames(StereoFrame* prev, StereoFrame* curr) {
    const std::vector<Point2f> prevPoints = prev->leftPoints();
    const size_t n = prevPoints.size();
    std::vector<Point2f> currPoints(n);
    std::vector<uint8_t> status(n);
    std::vector<float> error(n);
    if (n > 0 &&
        svo_calc_optical_flow_pyr_lk(mGpu, prev->leftImg().device(mGpu, kMaxLevel),
                                     curr->leftImg().device(mGpu, kMaxLevel),
                                     reinterpret_cast<const float*>(prevPoints.data()), (int)n,
                                     reinterpret_cast<float*>(currPoints.data()), status.data(), error.data(), 21, 21,
                                     kMaxLevel, SVO_TERM_COUNT | SVO_TERM_EPS, 50, 0.001, SVO_LK_GET_MIN_EIGENVALS | kLkOrder,
                                     1e-4) != SVO_OK)
        fail(mGpu, "svo_calc_optical_flow_pyr_lk (temporal)");

    std::vector<Feature::Ptr> newCurrFeatures;
    newCurrFeatures.reserve(n);
    for (size_t i = 0; i < n; ++i) {
        if (status[i]) {
            auto feat = Feature::Create(currPoints[i], prev->leftFeatures()[i]->mapPoint);
            feat->mapPoint->addObservation(curr->ID, feat);
            newCurrFeatures.push_back(feat);
        }
    }
    if (mTrace) {
        mTrace->lk_prev = prevPoints;
        mTrace->lk_next = currPoints;
        mTrace->lk_status = status;
    }
    curr->setFeatures(std::move(newCurrFeatures), {});
    // displayPoints (R:src/tracking.cpp:178) is UI: out of scope
}

// R:src/tracking.cpp:181-230
void Tracking::calculatePose(StereoFrame* frame) {
    std::vector<Point3d> worldPoints;
    worldPoints.reserve(frame->countPts());
    for (const auto& feature : frame->leftFeatures()) worldPoints.push_back(feature->mapPoint->mWorldPos);
    const std::vector<Point2f> imagePoints = frame->leftPoints();

    double rvec[3] = {0, 0, 0}, tvec[3] = {0, 0, 0};
    std::vector<int> inliersIdxs(worldPoints.size());
    int nin = 0;
    // cv::solvePnPRansac(world, left, K, zeros(1,4), rvec, tvec, false, 100, 8.0, 0.999, inliers, SQPNP);
    // < 4 points: OpenCV's CV_Assert throws; SVO_ERR_ARG here, thrown the same way
    const int rc = svo_solve_pnp_ransac(mGpu, reinterpret_cast<const double*>(worldPoints.data()),
                                        reinterpret_cast<const float*>(imagePoints.data()), (int)worldPoints.size(),
                                        K, 100, 8.0f, 0.999, rvec, tvec, inliersIdxs.data(), &nin);
    if (rc < 0) fail(mGpu, "svo_solve_pnp_ransac");
    if (rc == 0) {  // no model: OpenCV leaves rvec/tvec as given (zero) and the inlier list empty
        nin = 0;
        rvec[0] = rvec[1] = rvec[2] = tvec[0] = tvec[1] = tvec[2] = 0;
    }
    inliersIdxs.resize((size_t)nin);
    if (mTrace) {
        mTrace->pnp_obj = worldPoints;
        mTrace->pnp_img = imagePoints;
        mTrace->pnp_inliers = inliersIdxs;
        mTrace->pnp_ok = rc;
        for (int i = 0; i < 3; i++) {
            mTrace->rvec[i] = rvec[i];
            mTrace->tvec[i] = tvec[i];
        }
    }
    inlierRatio = static_cast<double>(inliersIdxs.size()) / (double)frame->countPts();

    double R[9];
    rodrigues(rvec, R);
    frame->pose() = SE3d(R, tvec).inverse();  // cv::Matx44d(...).inv()
    mRelativeMotion = frame->pose() * prevFrame->pose().inverse();

    // Remove outliers
    if (inliersIdxs.size() != frame->countPts()) {
        std::vector<Feature::Ptr> newLeftFeatures;
        newLeftFeatures.reserve(inliersIdxs.size());
        std::unordered_set<int> s(inliersIdxs.begin(), inliersIdxs.end());
        for (int i = 0; i < (int)frame->countPts(); ++i) {
            if (s.find(i) != s.end())
                newLeftFeatures.push_back(frame->leftFeatures()[i]);
            else
                frame->leftFeatures()[i]->isOutlier = true;
        }
        frame->setFeatures(std::move(newLeftFeatures), {});
    }
}

// R:src/tracking.cpp:233-235
bool Tracking::initialize() {
    if (mTrace) mTrace->clear();
    if (!(prevFrame = nextFrame())) return false;
    if (mTrace) {
        mTrace->frame_id = prevFrame->ID;
        mTrace->keyframe = true;
    }
    extractFeatures(prevFrame);
    triangulateNewMapPoints(prevFrame);
    return true;
}

// R:src/tracking.cpp:241-270 (one iteration of the main loop)
bool Tracking::processNext() {
    if (mTrace) mTrace->clear();
    if (!(currFrame = nextFrame())) return false;
    if (mTrace) {
        mTrace->frame_id = currFrame->ID;
        mTrace->keyframe = currFrame->isKeyFrame();
    }
    trackFrames(prevFrame, currFrame);
    calculatePose(currFrame);

    if (currFrame->isKeyFrame()) {
        StereoFrame temp(currFrame->ID, true, currFrame->leftImg(), currFrame->rightImg());
        temp.pose() = currFrame->pose();

        extractFeatures(&temp);
        triangulateNewMapPoints(&temp);

        currFrame->insertFeatures(temp.leftFeatures(), temp.rightFeatures());
    }

    mMap.addFrame(prevFrame);
    // the map keeps the frame (and its host pixels); its device pyramid is no longer needed
    prevFrame->leftImg().releaseDevice();
    prevFrame->rightImg().releaseDevice();
    prevFrame = currFrame;
    return true;
}

// R:src/tracking.cpp:232-276
void Tracking::startStereo() {
    if (!initialize()) return;
    double allTime = 0;
    for (;;) {
        const auto frameStart = std::chrono::steady_clock::now();
        StereoFrame* prev = prevFrame;
        if (!processNext()) break;
        const double frameTime =
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - frameStart).count();
        allTime += frameTime;
        if (mConfig.verbose)
            std::printf("%4zu | MPs: %5zu | Time: %.2lfms | Features: %zu | IR: %.2lf%% |%s\n", prev->ID,
                        mMap.mapPointsSize(), frameTime, prev->countPts(), inlierRatio * 100,
                        prev->isKeyFrame() ? " KF" : "");
    }
    if (mConfig.verbose)
        std::printf("All time: %lf\nAvg. frame time: %lf\n", allTime,
                    mConfig.end_frame ? allTime / mConfig.end_frame : 0.0);
}

}  // namespace svo
