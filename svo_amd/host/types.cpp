// SE3d and GrayImage of the host API mirror (include/svo/types.hpp).
#include <cstring>
#include <stdexcept>
#include <string>

#include "svo/types.hpp"
#include "svo_gpu.h"

namespace svo {

SE3d::SE3d(const double* R_, const double* t_) {
    std::memcpy(R, R_, sizeof(R));
    std::memcpy(t, t_, sizeof(t));
}

SE3d SE3d::operator*(const SE3d& o) const {
    SE3d r;
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++)
            r.R[3 * i + j] = R[3 * i] * o.R[j] + R[3 * i + 1] * o.R[3 + j] + R[3 * i + 2] * o.R[6 + j];
        r.t[i] = R[3 * i] * o.t[0] + R[3 * i + 1] * o.t[1] + R[3 * i + 2] * o.t[2] + t[i];
    }
    return r;
}

Point3d SE3d::operator*(const Point3d& p) const {
    return {R[0] * p.x + R[1] * p.y + R[2] * p.z + t[0], R[3] * p.x + R[4] * p.y + R[5] * p.z + t[1],
            R[6] * p.x + R[7] * p.y + R[8] * p.z + t[2]};
}

SE3d SE3d::inverse() const {
    SE3d r;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) r.R[3 * i + j] = R[3 * j + i];
    for (int i = 0; i < 3; i++) r.t[i] = -(r.R[3 * i] * t[0] + r.R[3 * i + 1] * t[1] + r.R[3 * i + 2] * t[2]);
    return r;
}

GrayImage::Body::~Body() {
    if (dev) svo_image_destroy(ctx, dev);
}

GrayImage::GrayImage(int w, int h) : b_(std::make_shared<Body>()) {
    if (w < 0 || h < 0) throw std::invalid_argument("GrayImage: negative size");
    b_->w = w;
    b_->h = h;
    b_->px.assign((size_t)w * h, 0);
}

GrayImage GrayImage::copyFrom(const uint8_t* data, int w, int h, int stride) {
    GrayImage im(w, h);
    for (int y = 0; y < h; y++) std::memcpy(im.b_->px.data() + (size_t)y * w, data + (size_t)y * stride, (size_t)w);
    return im;
}

GrayImage GrayImage::fromBGR(svo_ctx* ctx, const uint8_t* bgr, int w, int h, int stride, int max_level) {
    if (!ctx || !bgr || w <= 0 || h <= 0 || stride < 3 * w) throw std::invalid_argument("GrayImage::fromBGR");
    GrayImage im;
    im.b_ = std::make_shared<Body>();
    Body& b = *im.b_;
    b.w = w;
    b.h = h;
    b.px_valid = false;
    svo_image* d = nullptr;
    int rc = svo_image_create(ctx, w, h, max_level, &d);
    if (rc == SVO_OK) rc = svo_image_upload_bgr(ctx, d, bgr, stride);
    if (rc != SVO_OK) {
        if (d) svo_image_destroy(ctx, d);
        throw std::runtime_error(std::string("svo_image_upload_bgr: ") + svo_last_error(ctx));
    }
    b.dev = d;
    b.ctx = ctx;
    b.levels = max_level;
    return im;
}

uint8_t* GrayImage::Body::host() {
    if (!px_valid) {
        px.resize((size_t)w * h);
        if (!dev || svo_image_download_level(ctx, dev, 0, px.data(), w) != SVO_OK)
            throw std::runtime_error("GrayImage: device pixels unavailable");
        px_valid = true;
    }
    return px.data();
}

svo_image* GrayImage::device(svo_ctx* ctx, int max_level) const {
    if (empty()) throw std::invalid_argument("GrayImage::device: empty image");
    Body& b = *b_;
    if (b.dev && (b.ctx != ctx || b.levels < max_level)) {
        b.host();  // keep the pixels of a device-born image before dropping the device copy
        releaseDevice();
    }
    if (!b.dev) {
        svo_image* im = nullptr;
        int rc = svo_image_create(ctx, b.w, b.h, max_level, &im);
        if (rc == SVO_OK) rc = svo_image_upload(ctx, im, b.host(), b.w);
        if (rc != SVO_OK) {
            if (im) svo_image_destroy(ctx, im);
            throw std::runtime_error(std::string("svo_image_upload: ") + svo_last_error(ctx));
        }
        b.dev = im;
        b.ctx = ctx;
        b.levels = max_level;
    }
    return b.dev;
}

void GrayImage::releaseDevice() const {
    if (b_ && b_->dev) {
        svo_image_destroy(b_->ctx, b_->dev);
        b_->dev = nullptr;
        b_->levels = -1;
    }
}

}  // namespace svo
