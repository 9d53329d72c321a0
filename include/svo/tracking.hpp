// Tracking — mirror of R:include/tracking.h:19-58 / R:src/tracking.cpp on top of
// the C ABI (include/svo_gpu.h): the same methods, order of operations and
// parameters, with every OpenCV call replaced by its libsvo_gpu drop-in.
#pragma once

#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <vector>

#include "svo/frame.hpp"
#include "svo/map.hpp"
#include "svo/map_point.hpp"

namespace svo {

// R:include/config_reader.h:13-53 (fields the tracking path reads; YAML parsing
// is out of scope). device: HIP device of the tracker's context.
struct Config {
    std::string path, gt_path, calib_path;
    double fx = 0, fy = 0, cx = 0, cy = 0, bf = 0;
    int start_frame = 0, end_frame = 0;
    bool show_gt = false;
    bool use_orb = false;  // R:configs/config.yaml:20 ships 1; svo_orb_detect then replaces FAST
    struct {
        int nfeatures = 500;
        float scale_factor = 1.2f;
        int pyr_levels = 8;
        int patch_size = 31;
        int fast_treshold = 20;
    } orb_params;
    struct {
        int threshold = 20;
        bool nonMaxSuppression = true;
    } fast_params;
    struct {
        float y_threshold = 40;
        int features_to_track = 70;
    } tracking;
    int device = 0;
    bool verbose = true;  // the per-frame printf of startStereo
};

// Stereo image source (the reference's AsyncImageLoader::get contract,
// R:include/async_image_loader.h:49-56): false when no more frames.
class ImageSource {
public:
    virtual ~ImageSource() = default;
    virtual bool get(GrayImage& left, GrayImage& right) = 0;
};

// Frames pushed by the caller (thread-safe; get() does not block).
class QueueImageSource : public ImageSource {
public:
    void push(GrayImage left, GrayImage right);
    bool get(GrayImage& left, GrayImage& right) override;
    size_t size() const;

private:
    mutable std::mutex mMutex;
    std::deque<std::pair<GrayImage, GrayImage>> mQueue;
};

// What each stage of the last processed frame consumed and produced (for
// stage-by-stage parity checks; filled only when a trace is attached).
struct TrackingTrace {
    size_t frame_id = 0;
    bool keyframe = false;
    // trackFrames
    std::vector<Point2f> lk_prev, lk_next;
    std::vector<uint8_t> lk_status;
    // calculatePose
    std::vector<Point3d> pnp_obj;
    std::vector<Point2f> pnp_img;
    std::vector<int> pnp_inliers;
    int pnp_ok = 0;
    double rvec[3] = {0, 0, 0}, tvec[3] = {0, 0, 0};
    // extractFeatures / findLeftFeaturesInRight / triangulateNewMapPoints
    std::vector<Point2f> mask_pts, kps;
    std::vector<Point2f> stereo_right;
    std::vector<uint8_t> stereo_status;
    std::vector<Point2f> kept_left, kept_right;
    std::vector<Point3f> tri_xyz;
    void clear();
};

class Tracking {
public:
    // calib_data: P0 (left) then P1 (right), 3x4 row-major each (R:src/main.cpp:25-32).
    explicit Tracking(const Config& config, Map& map, const std::vector<float>& calib_data, ImageSource& source);
    ~Tracking();
    Tracking(const Tracking&) = delete;
    Tracking& operator=(const Tracking&) = delete;

    void startStereo();

    // pyrDown levels kept per device image: maxLevel of both LK calls (R:src/tracking.cpp:104,163)
    static constexpr int kImageLevels = 3;

    // startStereo split into its two parts, for callers that drive frames one
    // at a time: the first keyframe, then one loop iteration per call. Both
    // return false when the source has no frame.
    bool initialize();
    bool processNext();

    [[nodiscard]] StereoFrame* lastFrame() const { return prevFrame; }
    [[nodiscard]] double inlierRatioValue() const { return inlierRatio; }
    [[nodiscard]] const SE3d& relativeMotion() const { return mRelativeMotion; }
    [[nodiscard]] svo_ctx* context() const { return mGpu; }
    void setTrace(TrackingTrace* trace) { mTrace = trace; }

private:
    StereoFrame* nextFrame();
    void triangulateNewMapPoints(StereoFrame* frame);
    // static in the reference; a member here because it needs the GPU context
    void trackFrames(StereoFrame* prev, StereoFrame* curr);
    void calculatePose(StereoFrame* frame);
    void findLeftFeaturesInRight(StereoFrame* frame) const;
    void extractFeatures(StereoFrame* frame);

    StereoFrame *prevFrame, *currFrame;
    SE3d mRelativeMotion;

    size_t lastFrameID;
    ImageSource& mImageLoader;
    const Config& mConfig;
    Map& mMap;

    float mProjectionMatrixLeft[12], mProjectionMatrixRight[12];
    double K[9];  // Matx33f in the reference: float-rounded entries
    double inlierRatio;

    svo_ctx* mGpu = nullptr;
    TrackingTrace* mTrace = nullptr;
};

}  // namespace svo
