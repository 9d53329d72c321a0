// Frame / StereoFrame — mirror of R:include/frame.h:13-49, R:src/frame.cpp:11-50.
#pragma once

#include <vector>

#include "svo/feature.hpp"
#include "svo/types.hpp"

namespace svo {

class Frame {
public:
    size_t ID;

    explicit Frame(size_t frameID, bool is_kf);
    virtual ~Frame() = default;

    [[nodiscard]] inline bool isKeyFrame() const { return mIsKeyFrame; }
    [[nodiscard]] inline SE3d& pose() { return mCameraPose; }

private:
    bool mIsKeyFrame;
    SE3d mCameraPose;
};

class StereoFrame : public Frame {
public:
    StereoFrame(size_t frameID, bool is_kf, GrayImage left, GrayImage right);

    void setFeatures(std::vector<Feature::Ptr>&& left, std::vector<Feature::Ptr>&& right);
    void insertFeatures(const std::vector<Feature::Ptr>& left, const std::vector<Feature::Ptr>& right);

    [[nodiscard]] inline size_t countPts() const { return mLeftFeatures.size(); }

    [[nodiscard]] inline GrayImage& leftImg() { return mLeftImg; }
    [[nodiscard]] inline GrayImage& rightImg() { return mRightImg; }

    [[nodiscard]] inline const std::vector<Feature::Ptr>& leftFeatures() const { return mLeftFeatures; }
    [[nodiscard]] inline const std::vector<Feature::Ptr>& rightFeatures() const { return mRightFeatures; }

    [[nodiscard]] std::vector<Point2f> leftPoints() const;
    [[nodiscard]] std::vector<Point2f> rightPoints() const;

private:
    GrayImage mLeftImg, mRightImg;
    std::vector<Feature::Ptr> mLeftFeatures, mRightFeatures;
};

}  // namespace svo
