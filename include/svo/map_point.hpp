// MapPoint — mirror of R:include/map_point.h.
#pragma once

#include <unordered_map>

#include "svo/feature.hpp"

namespace svo {

class MapPoint {
    friend class Map;

public:
    const size_t ID;

    inline void addObservation(size_t frame_id, const Feature::Ptr& obs) { mObservations.insert({frame_id, obs}); }

private:
    inline MapPoint(size_t id, const Point3d& worldPos) : ID(id), mWorldPos(worldPos) {}

public:
    Point3d mWorldPos;
    std::unordered_map<size_t, Feature::Ptr> mObservations;
};

}  // namespace svo
