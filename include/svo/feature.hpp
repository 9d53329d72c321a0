// Feature — mirror of R:include/feature.h:15-27 / R:src/feature.cpp:6-28.
#pragma once

#include <memory>
#include <vector>

#include "svo/types.hpp"

namespace svo {

class MapPoint;

struct Feature {
    using Ptr = std::shared_ptr<Feature>;

    static Feature::Ptr Create(const Point2f& p, MapPoint* mp);
    static std::vector<Feature::Ptr> FromPoints(const std::vector<Point2f>& pts);

    explicit Feature(const Point2f& p);
    Feature(const Point2f& p, MapPoint* mp);

    Point2f pos;
    MapPoint* mapPoint;
    bool isOutlier;
};

}  // namespace svo
