/* TEST INFRASTRUCTURE ONLY (see svo_oracle.h): cv::ORB::detect restated.
 *
 * The reference's default detector (use_orb: 1, R:configs/config.yaml:20-27;
 * R:src/tracking.cpp:33-50 builds cv::ORB::create(nfeatures, scaleFactor,
 * nlevels, edgeThreshold = patch_size, 0, 4, HARRIS_SCORE, patchSize,
 * fastThreshold); :82 detect(img, keypoints, mask)). OpenCV 4.x files restated:
 *   features2d/src/orb.cpp     ORB_Impl::detectAndCompute (keypoints only),
 *                              computeKeyPoints, HarrisResponses, getScale
 *   imgproc/src/resize.cpp     resize(..., INTER_LINEAR_EXACT) ->
 *                              resize_bitExact<uchar, interpolationLinear>
 *                              (interpolationLinear::getCoeffs, hlineResizeCn,
 *                              vlineSet / vlineResize, ufixedpoint16/32)
 *   imgproc/src/thresh.cpp     threshold(254, THRESH_TOZERO) on the masks
 *   features2d/src/keypoint.cpp KeyPointsFilter::runByImageBorder, retainBest
 *   features2d/src/fast.cpp    FAST via svo_oracle_fast (fast.c)
 * C++ because retainBest's output order is defined by std::nth_element /
 * std::partition, which this file calls exactly as keypoint.cpp does.
 * PARITY: unpinned against OpenCV itself (absent here); KATs in
 * tests/test_orb.py pin the resize and the level schedule analytically. */
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "svo_oracle.h"

namespace {

/* resize_bitExact<uchar, interpolationLinear<uchar>> for one channel. */
struct LinearAxis {
    std::vector<int> ofs;
    std::vector<uint16_t> c0, c1;  /* ufixedpoint16 raw (8 fractional bits) */
    int dmin = 0, dmax = 0;        /* getMinMax: [dmin, dmax) interpolates */
};

LinearAxis linear_axis(int ssize, int dsize) {
    LinearAxis a;
    a.ofs.assign(dsize, 0);
    a.c0.assign(dsize, 0);
    a.c1.assign(dsize, 0);
    const double inv_scale = (double)dsize / (double)ssize; /* cv::resize: dsize.width / ssize.width */
    const double scale = 1.0 / inv_scale;                   /* softdouble::one() / softdouble(inv_scale) */
    int minofst = 0, maxofst = dsize;
    for (int val = 0; val < dsize; val++) {
        double fval = scale * ((double)val + 0.5) - 0.5;
        int ival = (int)std::floor(fval);
        if (ival >= 0 && ssize > 1) {
            if (ival < ssize - 1) {
                a.ofs[val] = ival;
                /* ufixedpoint16(softdouble): cvRound(v * 256), round-half-even */
                a.c1[val] = (uint16_t)std::nearbyint((fval - (double)ival) * 256.0);
                a.c0[val] = (uint16_t)(256 - a.c1[val]);
            } else {
                a.ofs[val] = ssize - 1;
                maxofst = std::min(maxofst, val);
            }
        } else {
            minofst = std::max(minofst, val + 1);
        }
    }
    a.dmin = minofst;
    a.dmax = maxofst;
    return a;
}

/* hlineResizeCn<uchar, ufixedpoint16, 2, true, 1>: one source row -> dw
 * ufixedpoint16 values. */
void hline(const uint8_t* src, const LinearAxis& ax, int dw, uint16_t* dst) {
    int i = 0;
    const uint16_t left = (uint16_t)(src[0] << 8);
    for (; i < ax.dmin && i < dw; i++) dst[i] = left;
    for (; i < ax.dmax; i++) {
        const uint8_t* px = src + ax.ofs[i];
        dst[i] = (uint16_t)(ax.c0[i] * px[0] + ax.c1[i] * px[1]);
    }
    const uint16_t right = (uint16_t)(src[ax.ofs[dw - 1]] << 8);
    for (; i < dw; i++) dst[i] = right;
}

/* ufixedpoint16 -> uchar (vlineSet): (v + 128) >> 8 */
inline uint8_t fx16_to_u8(uint32_t v) { return (uint8_t)((v + 128u) >> 8); }
/* ufixedpoint32 -> uchar: (v + 2^15) >> 16 */
inline uint8_t fx32_to_u8(uint32_t v) { return (uint8_t)((v + 32768u) >> 16); }

void resize_linear_exact(const uint8_t* src, int sw, int sh, int sstride, uint8_t* dst, int dw, int dh,
                         int dstride) {
    const LinearAxis ax = linear_axis(sw, dw), ay = linear_axis(sh, dh);
    std::vector<uint16_t> r0(dw), r1(dw);
    for (int dy = 0; dy < dh; dy++) {
        uint8_t* d = dst + (size_t)dy * dstride;
        if (dy < ay.dmin || dy >= ay.dmax) {
            /* rows above / below the source: the first / last source row */
            const int sy = dy < ay.dmin ? 0 : sh - 1;
            hline(src + (size_t)sy * sstride, ax, dw, r0.data());
            for (int x = 0; x < dw; x++) d[x] = fx16_to_u8(r0[x]);
            continue;
        }
        const int iy = ay.ofs[dy];
        hline(src + (size_t)iy * sstride, ax, dw, r0.data());
        hline(src + (size_t)(iy + 1) * sstride, ax, dw, r1.data());
        for (int x = 0; x < dw; x++)
            d[x] = fx32_to_u8((uint32_t)r0[x] * ay.c0[dy] + (uint32_t)r1[x] * ay.c1[dy]);
    }
}

struct Kp {
    float x, y, size, angle, response;
    int octave, class_id;
};

void retain_best(std::vector<Kp>& k, int n_points) {
    if (n_points >= 0 && k.size() > (size_t)n_points) {
        if (n_points == 0) {
            k.clear();
            return;
        }
        std::nth_element(k.begin(), k.begin() + n_points - 1, k.end(),
                         [](const Kp& a, const Kp& b) { return a.response > b.response; });
        const float amb = k[n_points - 1].response;
        auto ne = std::partition(k.begin() + n_points, k.end(), [amb](const Kp& p) { return p.response >= amb; });
        k.resize(ne - k.begin());
    }
}

float harris(const uint8_t* img, int stride, int x0, int y0) {
    const int block = 7, r = block / 2;
    const float scale = 1.f / ((1 << 2) * block * 255.f);
    const float scale_sq_sq = scale * scale * scale * scale;
    const float harris_k = 0.04f;
    const uint8_t* ptr0 = img + (long)(y0 - r) * stride + (x0 - r);
    int a = 0, b = 0, c = 0;
    for (int i = 0; i < block; i++)
        for (int j = 0; j < block; j++) {
            const uint8_t* ptr = ptr0 + i * stride + j;
            const int Ix = (ptr[1] - ptr[-1]) * 2 + (ptr[-stride + 1] - ptr[-stride - 1]) +
                           (ptr[stride + 1] - ptr[stride - 1]);
            const int Iy = (ptr[stride] - ptr[-stride]) * 2 + (ptr[stride - 1] - ptr[-stride - 1]) +
                           (ptr[stride + 1] - ptr[-stride + 1]);
            a += Ix * Ix;
            b += Iy * Iy;
            c += Ix * Iy;
        }
    return ((float)a * b - (float)c * c - harris_k * ((float)a + b) * ((float)a + b)) * scale_sq_sq;
}

}  // namespace

extern "C" {

void svo_oracle_resize_linear_exact(const uint8_t* src, int sw, int sh, int sstride, uint8_t* dst, int dw, int dh,
                                    int dstride) {
    resize_linear_exact(src, sw, sh, sstride, dst, dw, dh, dstride);
}

void svo_oracle_orb_level_info(int w, int h, float scale_factor, int nlevels, int nfeatures, int* lw, int* lh,
                               float* lscale, int* nper) {
    const double sf = (double)scale_factor; /* ORB_Impl keeps scaleFactor as double */
    for (int l = 0; l < nlevels; l++) {
        const float s = (float)std::pow(sf, (double)l); /* getScale(level, 0, scaleFactor) */
        lscale[l] = s;
        lw[l] = (int)std::nearbyint((float)w / s); /* cvRound(image.cols / scale) */
        lh[l] = (int)std::nearbyint((float)h / s);
    }
    const float factor = (float)(1.0 / sf);
    float nd = nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nlevels));
    int sum = 0;
    for (int l = 0; l < nlevels - 1; l++) {
        nper[l] = (int)std::nearbyint(nd);
        sum += nper[l];
        nd *= factor;
    }
    nper[nlevels - 1] = std::max(nfeatures - sum, 0);
}

int svo_oracle_orb_detect(const uint8_t* img, int w, int h, int stride, const uint8_t* mask, int nfeatures,
                          float scale_factor, int nlevels, int edge_threshold, int patch_size, int fast_threshold,
                          int harris_score, float* kp_xyr, int* octave, int cap) {
    if (nlevels < 1 || nlevels > 16 || edge_threshold < 4) return -1; /* Harris reads 4 px around */
    std::vector<int> lw(nlevels), lh(nlevels), nper(nlevels);
    std::vector<float> lscale(nlevels);
    svo_oracle_orb_level_info(w, h, scale_factor, nlevels, nfeatures, lw.data(), lh.data(), lscale.data(),
                              nper.data());
    /* image and mask pyramids, tightly packed per level */
    std::vector<std::vector<uint8_t>> im(nlevels), mk(nlevels);
    im[0].resize((size_t)w * h);
    for (int y = 0; y < h; y++) std::memcpy(&im[0][(size_t)y * w], img + (size_t)y * stride, w);
    if (mask) mk[0].assign(mask, mask + (size_t)w * h);
    for (int l = 1; l < nlevels; l++) {
        im[l].resize((size_t)lw[l] * lh[l]);
        resize_linear_exact(im[l - 1].data(), lw[l - 1], lh[l - 1], lw[l - 1], im[l].data(), lw[l], lh[l], lw[l]);
        if (mask) {
            mk[l].resize((size_t)lw[l] * lh[l]);
            resize_linear_exact(mk[l - 1].data(), lw[l - 1], lh[l - 1], lw[l - 1], mk[l].data(), lw[l], lh[l],
                                lw[l]);
            for (auto& v : mk[l]) v = v > 254 ? v : 0; /* THRESH_TOZERO */
        }
    }
    std::vector<Kp> all;
    std::vector<int> counters(nlevels);
    for (int l = 0; l < nlevels; l++) {
        const int capf = lw[l] * lh[l];
        std::vector<float> f((size_t)capf * 3 + 3);
        int n = svo_oracle_fast(im[l].data(), lw[l], lh[l], lw[l], fast_threshold, 1, mask ? mk[l].data() : nullptr,
                                f.data(), capf);
        std::vector<Kp> k;
        for (int i = 0; i < n; i++) k.push_back(Kp{f[3 * i], f[3 * i + 1], 7.f, -1.f, f[3 * i + 2], 0, -1});
        /* runByImageBorder(keypoints, img.size(), edgeThreshold) */
        if (edge_threshold > 0) {
            if (lh[l] <= edge_threshold * 2 || lw[l] <= edge_threshold * 2) {
                k.clear();
            } else {
                const float x0 = (float)edge_threshold, y0 = (float)edge_threshold;
                const float x1 = (float)(lw[l] - edge_threshold), y1 = (float)(lh[l] - edge_threshold);
                k.erase(std::remove_if(k.begin(), k.end(),
                                       [&](const Kp& p) { return !(p.x >= x0 && p.y >= y0 && p.x < x1 && p.y < y1); }),
                        k.end());
            }
        }
        retain_best(k, harris_score ? 2 * nper[l] : nper[l]);
        counters[l] = (int)k.size();
        for (auto& p : k) {
            p.octave = l;
            p.size = patch_size * lscale[l];
            all.push_back(p);
        }
    }
    if (harris_score) {
        for (auto& p : all)
            p.response = harris(im[p.octave].data(), lw[p.octave], (int)std::nearbyint(p.x), (int)std::nearbyint(p.y));
        std::vector<Kp> sel;
        size_t off = 0;
        for (int l = 0; l < nlevels; l++) {
            std::vector<Kp> k(all.begin() + off, all.begin() + off + counters[l]);
            off += counters[l];
            retain_best(k, nper[l]);
            sel.insert(sel.end(), k.begin(), k.end());
        }
        all.swap(sel);
    }
    const int n = (int)all.size();
    for (int i = 0; i < n && i < cap; i++) {
        const float s = lscale[all[i].octave];
        kp_xyr[3 * i] = all[i].x * s;
        kp_xyr[3 * i + 1] = all[i].y * s;
        kp_xyr[3 * i + 2] = all[i].response;
        if (octave) octave[i] = all[i].octave;
    }
    return n;
}

}  // extern "C"
