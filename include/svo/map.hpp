// Map — the parts of R:include/map.h / R:src/map.cpp the tracking path uses
// (frame and map-point ownership). The viewer thread, drawer and ground-truth
// parsing are UI and out of scope.
#pragma once

#include <shared_mutex>
#include <unordered_map>
#include <vector>

#include "svo/types.hpp"

namespace svo {

class Frame;
class MapPoint;

class Map {
public:
    Map() = default;
    ~Map();
    Map(const Map&) = delete;
    Map& operator=(const Map&) = delete;

    void addFrame(Frame* frame);
    MapPoint* createMapPoint(const Point3d& position);
    [[nodiscard]] size_t mapPointsSize() const;
    [[nodiscard]] size_t framesSize() const;

private:
    std::vector<Frame*> mAllFrames;
    std::unordered_map<size_t, Frame*> mKeyFrames;
    std::vector<MapPoint*> mMapPoints;
    mutable std::shared_mutex mMapMutex;
};

}  // namespace svo
