// Plain value types of the host API mirror (stand-ins for the cv:: / Sophus
// types the reference's Frame/Feature/Tracking use; layout-compatible where it
// matters: Point2f is two floats like cv::Point2f, Point3d three doubles).
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>
#include <vector>

struct svo_ctx;
struct svo_image;

namespace svo {

struct Point2f {
    float x = 0.f, y = 0.f;
    Point2f() = default;
    Point2f(float x_, float y_) : x(x_), y(y_) {}
    Point2f operator-(const Point2f& o) const { return {x - o.x, y - o.y}; }
    Point2f operator+(const Point2f& o) const { return {x + o.x, y + o.y}; }
};

struct Point3f {
    float x = 0.f, y = 0.f, z = 0.f;
};

struct Point3d {
    double x = 0, y = 0, z = 0;
    Point3d() = default;
    Point3d(double x_, double y_, double z_) : x(x_), y(y_), z(z_) {}
};

// Rigid transform p -> R p + t (Sophus::SE3d stand-in, R row-major).
struct SE3d {
    double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    double t[3] = {0, 0, 0};
    SE3d() = default;
    SE3d(const double* R_, const double* t_);
    SE3d operator*(const SE3d& o) const;
    Point3d operator*(const Point3d& p) const;
    SE3d inverse() const;
};

// Reference-counted 8-bit single-channel image (the cv::Mat CV_8UC1 the
// reference passes around). Copies share the pixels and the device pyramid,
// which is uploaded and built on first use by a GPU call.
class GrayImage {
public:
    GrayImage() = default;
    GrayImage(int w, int h);
    static GrayImage copyFrom(const uint8_t* data, int w, int h, int stride);
    // The loader's imread + cvtColor(COLOR_BGR2GRAY) (R:include/async_image_loader.h:63-69)
    // done on the device: the grey image is born device-resident (svo_image_upload_bgr,
    // pyramid of max_level levels) and its host pixels are downloaded on first data().
    static GrayImage fromBGR(svo_ctx* ctx, const uint8_t* bgr, int w, int h, int stride, int max_level);

    int cols() const { return b_ ? b_->w : 0; }
    int rows() const { return b_ ? b_->h : 0; }
    bool empty() const { return !b_ || b_->w == 0; }
    uint8_t* data() { return b_ ? b_->host() : nullptr; }
    const uint8_t* data() const { return b_ ? b_->host() : nullptr; }

    // Device image with >= max_level pyrDown levels (uploaded once per image).
    svo_image* device(svo_ctx* ctx, int max_level) const;
    // Frees the device copy (pixels stay on the host).
    void releaseDevice() const;

private:
    struct Body {
        std::vector<uint8_t> px;
        bool px_valid = true;  // false while only the device copy holds the pixels
        int w = 0, h = 0;
        svo_ctx* ctx = nullptr;
        svo_image* dev = nullptr;
        int levels = -1;
        uint8_t* host();
        ~Body();
    };
    std::shared_ptr<Body> b_;
};

}  // namespace svo
