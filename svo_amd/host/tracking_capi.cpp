// C shim over the host Tracking mirror (include/svo_tracking.h).
#include <cstring>
#include <exception>
#include <memory>
#include <string>

#include "svo/tracking.hpp"
#include "svo_tracking.h"

struct svo_tracking {
    svo::Config config;
    svo::Map map;
    svo::QueueImageSource source;
    svo::TrackingTrace trace;
    std::unique_ptr<svo::Tracking> tracking;
    bool started = false;
    std::string err;
};

namespace {

template <class T>
int64_t copy_field(const std::vector<T>& v, void* dst, int64_t cap) {
    const int64_t bytes = (int64_t)(v.size() * sizeof(T));
    if (dst && cap > 0) std::memcpy(dst, v.data(), (size_t)(bytes < cap ? bytes : cap));
    return bytes;
}

}  // namespace

extern "C" {

int svo_tracking_create(const svo_tracking_config* cfg, const float calib[24], svo_tracking** out) {
    if (!cfg || !calib || !out) return -1;
    *out = nullptr;
    auto tr = std::make_unique<svo_tracking>();
    tr->config.fast_params.threshold = cfg->fast_threshold;
    tr->config.fast_params.nonMaxSuppression = cfg->fast_nonmax != 0;
    tr->config.tracking.y_threshold = cfg->y_threshold;
    tr->config.tracking.features_to_track = cfg->features_to_track;
    tr->config.device = cfg->device;
    tr->config.verbose = false;
    tr->config.use_orb = cfg->use_orb != 0;
    if (cfg->use_orb) {
        tr->config.orb_params.nfeatures = cfg->orb_nfeatures;
        tr->config.orb_params.scale_factor = cfg->orb_scale_factor;
        tr->config.orb_params.pyr_levels = cfg->orb_pyr_levels;
        tr->config.orb_params.patch_size = cfg->orb_patch_size;
        tr->config.orb_params.fast_treshold = cfg->orb_fast_threshold;
    }
    try {
        tr->tracking = std::make_unique<svo::Tracking>(tr->config, tr->map, std::vector<float>(calib, calib + 24),
                                                       tr->source);
    } catch (const std::exception&) {
        return -4;
    }
    tr->tracking->setTrace(&tr->trace);
    *out = tr.release();
    return 0;
}

void svo_tracking_destroy(svo_tracking* tr) {
    if (!tr) return;
    tr->tracking.reset();  // before the map: frames it still owns release their device images
    delete tr;
}

const char* svo_tracking_last_error(const svo_tracking* tr) { return tr ? tr->err.c_str() : "null tracking"; }

int svo_tracking_push_stereo(svo_tracking* tr, const uint8_t* left, const uint8_t* right, int w, int h,
                             int stride) {
    if (!tr || !left || !right || w <= 0 || h <= 0 || stride < w) return -1;
    tr->source.push(svo::GrayImage::copyFrom(left, w, h, stride), svo::GrayImage::copyFrom(right, w, h, stride));
    return 0;
}

int svo_tracking_push_stereo_bgr(svo_tracking* tr, const uint8_t* left, const uint8_t* right, int w, int h,
                                 int stride) {
    if (!tr || !left || !right || w <= 0 || h <= 0 || stride < 3 * w) return -1;
    try {
        svo_ctx* ctx = tr->tracking->context();
        const int lv = svo::Tracking::kImageLevels;
        tr->source.push(svo::GrayImage::fromBGR(ctx, left, w, h, stride, lv),
                        svo::GrayImage::fromBGR(ctx, right, w, h, stride, lv));
    } catch (const std::exception& e) {
        tr->err = e.what();
        return -2;
    }
    return 0;
}

int svo_tracking_step(svo_tracking* tr) {
    if (!tr) return -1;
    try {
        bool ok;
        if (!tr->started) {
            ok = tr->tracking->initialize();
            tr->started = ok;
        } else {
            ok = tr->tracking->processNext();
        }
        return ok ? 1 : 0;
    } catch (const std::exception& e) {
        tr->err = e.what();
        return -2;
    }
}

int svo_tracking_frame_info(const svo_tracking* tr, int64_t* frame_id, int* is_keyframe, int64_t* n_features,
                            int64_t* n_map_points, double* inlier_ratio, double pose[12]) {
    if (!tr || !tr->tracking) return -1;
    svo::StereoFrame* f = tr->tracking->lastFrame();
    if (!f) return -1;
    if (frame_id) *frame_id = (int64_t)f->ID;
    if (is_keyframe) *is_keyframe = f->isKeyFrame() ? 1 : 0;
    if (n_features) *n_features = (int64_t)f->countPts();
    if (n_map_points) *n_map_points = (int64_t)tr->map.mapPointsSize();
    if (inlier_ratio) *inlier_ratio = tr->tracking->inlierRatioValue();
    if (pose) {
        std::memcpy(pose, f->pose().R, sizeof(double) * 9);
        std::memcpy(pose + 9, f->pose().t, sizeof(double) * 3);
    }
    return 0;
}

int svo_tracking_features(const svo_tracking* tr, float* xy, double* world, int64_t* mp_ids, int cap, int* n) {
    if (!tr || !tr->tracking || cap < 0) return -1;
    svo::StereoFrame* f = tr->tracking->lastFrame();
    if (!f) return -1;
    const auto& fs = f->leftFeatures();
    if (n) *n = (int)fs.size();
    for (size_t i = 0; i < fs.size() && (int)i < cap; i++) {
        if (xy) {
            xy[2 * i] = fs[i]->pos.x;
            xy[2 * i + 1] = fs[i]->pos.y;
        }
        const svo::MapPoint* mp = fs[i]->mapPoint;
        if (world) {
            world[3 * i] = mp ? mp->mWorldPos.x : 0;
            world[3 * i + 1] = mp ? mp->mWorldPos.y : 0;
            world[3 * i + 2] = mp ? mp->mWorldPos.z : 0;
        }
        if (mp_ids) mp_ids[i] = mp ? (int64_t)mp->ID : -1;
    }
    return 0;
}

int64_t svo_tracking_trace(const svo_tracking* tr, const char* field, void* dst, int64_t cap) {
    if (!tr || !field) return -1;
    const svo::TrackingTrace& t = tr->trace;
    const std::string f(field);
    if (f == "lk_prev") return copy_field(t.lk_prev, dst, cap);
    if (f == "lk_next") return copy_field(t.lk_next, dst, cap);
    if (f == "lk_status") return copy_field(t.lk_status, dst, cap);
    if (f == "pnp_obj") return copy_field(t.pnp_obj, dst, cap);
    if (f == "pnp_img") return copy_field(t.pnp_img, dst, cap);
    if (f == "pnp_inliers") return copy_field(t.pnp_inliers, dst, cap);
    if (f == "pnp_pose") {
        std::vector<double> v(t.rvec, t.rvec + 3);
        v.insert(v.end(), t.tvec, t.tvec + 3);
        v.push_back((double)t.pnp_ok);
        return copy_field(v, dst, cap);
    }
    if (f == "mask_pts") return copy_field(t.mask_pts, dst, cap);
    if (f == "kps") return copy_field(t.kps, dst, cap);
    if (f == "stereo_right") return copy_field(t.stereo_right, dst, cap);
    if (f == "stereo_status") return copy_field(t.stereo_status, dst, cap);
    if (f == "kept_left") return copy_field(t.kept_left, dst, cap);
    if (f == "kept_right") return copy_field(t.kept_right, dst, cap);
    if (f == "tri_xyz") return copy_field(t.tri_xyz, dst, cap);
    return -1;
}

}  // extern "C"
