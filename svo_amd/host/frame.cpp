// Feature, Frame/StereoFrame and Map of the host API mirror:
// R:src/feature.cpp:6-28, R:src/frame.cpp:11-50, R:src/map.cpp:51-81.
#include <mutex>

#include "svo/feature.hpp"
#include "svo/frame.hpp"
#include "svo/map.hpp"
#include "svo/map_point.hpp"

namespace svo {

Feature::Ptr Feature::Create(const Point2f& p, MapPoint* mp) { return std::make_shared<Feature>(p, mp); }

std::vector<Feature::Ptr> Feature::FromPoints(const std::vector<Point2f>& pts) {
    std::vector<Feature::Ptr> result;
    result.reserve(pts.size());
    for (const auto& p : pts) result.emplace_back(std::make_shared<Feature>(p));
    return result;
}

Feature::Feature(const Point2f& p) : pos(p), mapPoint(nullptr), isOutlier(false) {}
Feature::Feature(const Point2f& p, MapPoint* mp) : pos(p), mapPoint(mp), isOutlier(false) {}

Frame::Frame(size_t frameID, bool is_kf) : ID(frameID), mIsKeyFrame(is_kf), mCameraPose() {}

StereoFrame::StereoFrame(size_t frameID, bool is_kf, GrayImage left, GrayImage right)
    : Frame(frameID, is_kf), mLeftImg(std::move(left)), mRightImg(std::move(right)) {}

void StereoFrame::setFeatures(std::vector<Feature::Ptr>&& left, std::vector<Feature::Ptr>&& right) {
    mLeftFeatures = std::move(left);
    mRightFeatures = std::move(right);
}

void StereoFrame::insertFeatures(const std::vector<Feature::Ptr>& left, const std::vector<Feature::Ptr>& right) {
    mLeftFeatures.insert(mLeftFeatures.end(), left.begin(), left.end());
    mRightFeatures.insert(mRightFeatures.end(), right.begin(), right.end());
}

std::vector<Point2f> StereoFrame::leftPoints() const {
    std::vector<Point2f> res;
    res.reserve(mLeftFeatures.size());
    for (const auto& f : mLeftFeatures) res.push_back(f->pos);
    return res;
}

std::vector<Point2f> StereoFrame::rightPoints() const {
    std::vector<Point2f> res;
    res.reserve(mRightFeatures.size());
    for (const auto& f : mRightFeatures) res.push_back(f->pos);
    return res;
}

Map::~Map() {
    for (auto* f : mAllFrames) delete f;
    for (auto* mp : mMapPoints) delete mp;
}

void Map::addFrame(Frame* frame) {
    std::unique_lock lock(mMapMutex);
    mAllFrames.push_back(frame);
    if (frame->isKeyFrame()) mKeyFrames.insert({frame->ID, frame});
}

MapPoint* Map::createMapPoint(const Point3d& position) {
    std::unique_lock lock(mMapMutex);
    mMapPoints.push_back(new MapPoint(mMapPoints.size(), position));
    return mMapPoints.back();
}

size_t Map::mapPointsSize() const {
    std::shared_lock lock(mMapMutex);
    return mMapPoints.size();
}

size_t Map::framesSize() const {
    std::shared_lock lock(mMapMutex);
    return mAllFrames.size();
}

}  // namespace svo
