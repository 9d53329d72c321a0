// Deterministic synthetic input for tests and bench only: a
// canvas of random rectangles (box-blurred) seen by a pinhole camera that only
// rotates, so frame-to-frame motion is the homography K R K^-1 and a map point
// at ANY depth along a canvas ray reprojects exactly (no stereo needed to make
// consistent 3D points). The reference reads KITTI PNGs instead
// (R:include/async_image_loader.h:57-69); KITTI is not available here.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>

#include "svo_synth.h"

namespace {
constexpr int SVO_OK = 0, SVO_ERR_ARG = -1;  // the values of svo_gpu.h's codes
}

namespace {

inline uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
inline uint64_t hash3(uint64_t seed, uint64_t a, uint64_t b) {
    uint64_t s = seed ^ (a * 0x9E3779B97F4A7C15ULL) ^ (b * 0xC2B2AE3D27D4EB4FULL);
    return splitmix(s);
}

// rows [0, h) in contiguous bands on up to 16 host threads (deterministic: each
// pixel depends on its own coordinates only)
template <class F>
void for_rows(int h, F f) {
    const int nt = std::max(1, std::min({16, (int)std::thread::hardware_concurrency(), h / 16}));
    if (nt == 1) {
        f(0, h);
        return;
    }
    std::vector<std::thread> th;
    for (int i = 0; i < nt; i++) th.emplace_back(f, (int)((int64_t)h * i / nt), (int)((int64_t)h * (i + 1) / nt));
    for (auto& t : th) t.join();
}

}  // namespace

extern "C" int svo_synth_canvas(uint64_t seed, int cw, int ch, int n_rect, uint8_t* canvas) {
    if (cw <= 0 || ch <= 0 || !canvas || n_rect < 0) return SVO_ERR_ARG;
    std::vector<uint8_t> tmp((size_t)cw * ch, 128);
    uint64_t s = seed * 2 + 1;
    for (int r = 0; r < n_rect; r++) {
        int x = (int)(splitmix(s) % (uint64_t)cw), y = (int)(splitmix(s) % (uint64_t)ch);
        int w = 4 + (int)(splitmix(s) % 61), h = 4 + (int)(splitmix(s) % 61);
        uint8_t v = (uint8_t)(splitmix(s) & 0xFF);
        for (int yy = y; yy < y + h && yy < ch; yy++)
            std::memset(&tmp[(size_t)yy * cw + x], v, (size_t)((x + w <= cw ? w : cw - x)));
    }
    // 3x3 box blur, replicate border
    for (int y = 0; y < ch; y++)
        for (int x = 0; x < cw; x++) {
            int acc = 0;
            for (int dy = -1; dy <= 1; dy++) {
                int yy = y + dy < 0 ? 0 : y + dy >= ch ? ch - 1 : y + dy;
                for (int dx = -1; dx <= 1; dx++) {
                    int xx = x + dx < 0 ? 0 : x + dx >= cw ? cw - 1 : x + dx;
                    acc += tmp[(size_t)yy * cw + xx];
                }
            }
            canvas[(size_t)y * cw + x] = (uint8_t)((acc + 4) / 9);
        }
    return SVO_OK;
}

extern "C" int svo_synth_frame(const uint8_t* canvas, int cw, int ch, int margin_x, int margin_y,
                               const double R[9], const double K[9], uint64_t noise_seed, int noise,
                               uint8_t* frame, int w, int h) {
    if (!canvas || !R || !K || !frame || w <= 0 || h <= 0) return SVO_ERR_ARG;
    const double fx = K[0], fy = K[4], cx = K[2], cy = K[5];
    for_rows(h, [&](int y0, int y1) {
    for (int y = y0; y < y1; y++)
        for (int x = 0; x < w; x++) {
            // camera ray, rotated to the world (canvas) frame: R^T K^-1 p
            const double dx = (x - cx) / fx, dy = (y - cy) / fy;
            const double wx = R[0] * dx + R[3] * dy + R[6];
            const double wy = R[1] * dx + R[4] * dy + R[7];
            const double wz = R[2] * dx + R[5] * dy + R[8];
            double u = fx * wx / wz + cx + margin_x, v = fy * wy / wz + cy + margin_y;
            if (!(wz > 0)) u = v = -1;
            u = u < 0 ? 0 : u > cw - 1.001 ? cw - 1.001 : u;
            v = v < 0 ? 0 : v > ch - 1.001 ? ch - 1.001 : v;
            const int iu = (int)u, iv = (int)v;
            const double a = u - iu, b = v - iv;
            const uint8_t* c0 = canvas + (size_t)iv * cw + iu;
            const uint8_t* c1 = c0 + cw;
            double val = (1 - a) * (1 - b) * c0[0] + a * (1 - b) * c0[1] + (1 - a) * b * c1[0] + a * b * c1[1];
            if (noise > 0) val += (int)(hash3(noise_seed, (uint64_t)x, (uint64_t)y) % (uint64_t)(2 * noise + 1)) - noise;
            int iv8 = (int)std::floor(val + 0.5);
            frame[(size_t)y * w + x] = (uint8_t)(iv8 < 0 ? 0 : iv8 > 255 ? 255 : iv8);
        }
    });
    return SVO_OK;
}

// Right image of a rectified stereo rig (baseline along camera x, fx*b = bf):
// the canvas points now sit at the depth field rho(cu, cv) (world z, the same
// field the map points use), so the right view of right pixel (xr, y) is the
// left view of the pixel xl solving xl = xr + bf / z(xl, y), with z the
// camera-frame depth of the surface point seen at left pixel (xl, y).
// Fixed-point iteration (a contraction: |d(bf/z)/dx| << 1 for this field),
// stopped once the step is below 1e-7 px.
extern "C" int svo_synth_frame_right(const uint8_t* canvas, int cw, int ch, int margin_x, int margin_y,
                                     const double R[9], const double K[9], double bf, int depth_seed,
                                     uint64_t noise_seed, int noise, uint8_t* frame, int w, int h) {
    if (!canvas || !R || !K || !frame || w <= 0 || h <= 0) return SVO_ERR_ARG;
    const double fx = K[0], fy = K[4], cx = K[2], cy = K[5];
    const double seed = (double)depth_seed;
    for_rows(h, [&](int y0, int y1) {
    for (int y = y0; y < y1; y++) {
        double xprev = 0.0;  // the previous pixel's solution: a warm start for this one
        for (int x = 0; x < w; x++) {
            double xl = x == 0 ? 0.0 : xprev + 1.0, u = -1, v = -1;
            for (int it = 0; it < 12; it++) {
                const double dx = (xl - cx) / fx, dy = (y - cy) / fy;
                const double wx = R[0] * dx + R[3] * dy + R[6];
                const double wy = R[1] * dx + R[4] * dy + R[7];
                const double wz = R[2] * dx + R[5] * dy + R[8];
                if (!(wz > 0)) break;
                const double cu = fx * wx / wz + cx, cv = fy * wy / wz + cy;
                const double rho = 12.0 + 5.0 * std::sin(cu / 97.0 + seed) + 4.0 * std::cos(cv / 61.0 - 0.5 * seed);
                u = cu + margin_x;
                v = cv + margin_y;
                const double xn = x + bf * wz / rho;  // camera-frame depth of the surface point = rho / wz
                const bool done = std::fabs(xn - xl) < 1e-7;
                xl = xn;
                if (done) break;
            }
            xprev = xl;
            u = u < 0 ? 0 : u > cw - 1.001 ? cw - 1.001 : u;
            v = v < 0 ? 0 : v > ch - 1.001 ? ch - 1.001 : v;
            const int iu = (int)u, iv = (int)v;
            const double a = u - iu, b = v - iv;
            const uint8_t* c0 = canvas + (size_t)iv * cw + iu;
            const uint8_t* c1 = c0 + cw;
            double val = (1 - a) * (1 - b) * c0[0] + a * (1 - b) * c0[1] + (1 - a) * b * c1[0] + a * b * c1[1];
            if (noise > 0) val += (int)(hash3(noise_seed, (uint64_t)x, (uint64_t)y) % (uint64_t)(2 * noise + 1)) - noise;
            int iv8 = (int)std::floor(val + 0.5);
            frame[(size_t)y * w + x] = (uint8_t)(iv8 < 0 ? 0 : iv8 > 255 ? 255 : iv8);
        }
    }
    });
    return SVO_OK;
}

// svo_synth_view (include/svo_synth.h): a general camera (R, C) over the depth-field
// surface X(cu, cv) = (((cu - cx) / fx) rho, ((cv - cy) / fy) rho, rho), rho =
// rho(cu, cv) (the surface the rotation-only views and the right view use), plus
// rectangular occluders in world planes z = const.
extern "C" int svo_synth_view(const uint8_t* canvas, int cw, int ch, int margin_x, int margin_y, const double R[9],
                              const double C[3], const double K[9], int depth_seed, const double* occ, int n_occ,
                              const uint8_t* occ_tex, int tw, int th, uint64_t noise_seed, int noise, uint8_t* frame,
                              int w, int h) {
    if (!canvas || !R || !C || !K || !frame || w <= 0 || h <= 0 || n_occ < 0 || (n_occ > 0 && (!occ || !occ_tex)) ||
        (n_occ > 0 && (tw < 2 || th < 2)))
        return SVO_ERR_ARG;
    const double fx = K[0], fy = K[4], cx = K[2], cy = K[5];
    const double seed = (double)depth_seed;
    auto bilinear = [](const uint8_t* img, int iw, int ih, double u, double v) {
        u = u < 0 ? 0 : u > iw - 1.001 ? iw - 1.001 : u;
        v = v < 0 ? 0 : v > ih - 1.001 ? ih - 1.001 : v;
        const int iu = (int)u, iv = (int)v;
        const double a = u - iu, b = v - iv;
        const uint8_t* c0 = img + (size_t)iv * iw + iu;
        const uint8_t* c1 = c0 + iw;
        return (1 - a) * (1 - b) * c0[0] + a * (1 - b) * c0[1] + (1 - a) * b * c1[0] + a * b * c1[1];
    };
    for_rows(h, [&](int y0, int y1) {
        for (int y = y0; y < y1; y++) {
            double lam_prev = -1.0;  // the previous pixel's ray parameter: a warm start
            for (int x = 0; x < w; x++) {
                // world ray d = R^T K^-1 p from C
                const double dx = (x - cx) / fx, dy = (y - cy) / fy;
                const double d0 = R[0] * dx + R[3] * dy + R[6];
                const double d1 = R[1] * dx + R[4] * dy + R[7];
                const double d2 = R[2] * dx + R[5] * dy + R[8];
                double val = 128.0;
                double lam = -1.0;
                if (d2 > 0) {
                    // f(lam) = X_z - rho(cu, cv), X = C + lam d: f < 0 at rho's minimum
                    // 3, > 0 at its maximum 21 -> a bracket; Newton steps inside it
                    double lo = (3.0 - C[2]) / d2, hi = (21.0 - C[2]) / d2;
                    lam = lam_prev > lo && lam_prev < hi ? lam_prev : 0.5 * (lo + hi);
                    double cu = 0, cv = 0;
                    for (int it = 0; it < 60; it++) {
                        const double X0 = C[0] + lam * d0, X1 = C[1] + lam * d1, X2 = C[2] + lam * d2;
                        cu = fx * X0 / X2 + cx;
                        cv = fy * X1 / X2 + cy;
                        const double rho = 12.0 + 5.0 * std::sin(cu / 97.0 + seed) + 4.0 * std::cos(cv / 61.0 - 0.5 * seed);
                        const double f = X2 - rho;
                        if (std::fabs(f) < 1e-10) break;
                        if (f < 0) lo = lam; else hi = lam;
                        const double dcu = fx * (d0 * X2 - X0 * d2) / (X2 * X2);
                        const double dcv = fy * (d1 * X2 - X1 * d2) / (X2 * X2);
                        const double drho = 5.0 * std::cos(cu / 97.0 + seed) / 97.0 * dcu -
                                            4.0 * std::sin(cv / 61.0 - 0.5 * seed) / 61.0 * dcv;
                        const double fp = d2 - drho;
                        double nl = fp > 0 ? lam - f / fp : 0.5 * (lo + hi);
                        if (!(nl > lo && nl < hi)) nl = 0.5 * (lo + hi);
                        if (hi - lo < 1e-13) break;
                        lam = nl;
                    }
                    val = bilinear(canvas, cw, ch, cu + margin_x, cv + margin_y);
                    // the nearest occluder in front of the surface point
                    double best = lam;
                    for (int k = 0; k < n_occ; k++) {
                        const double* o = occ + 5 * k;
                        const double lo_ = (o[4] - C[2]) / d2;
                        if (!(lo_ > 0 && lo_ < best)) continue;
                        const double X0 = C[0] + lo_ * d0, X1 = C[1] + lo_ * d1;
                        if (X0 < o[0] || X0 > o[2] || X1 < o[1] || X1 > o[3]) continue;
                        best = lo_;
                        val = bilinear(occ_tex, tw, th, (X0 - o[0]) / (o[2] - o[0]) * (tw - 1),
                                       (X1 - o[1]) / (o[3] - o[1]) * (th - 1));
                    }
                }
                lam_prev = lam;
                if (noise > 0)
                    val += (int)(hash3(noise_seed, (uint64_t)x, (uint64_t)y) % (uint64_t)(2 * noise + 1)) - noise;
                const int iv8 = (int)std::floor(val + 0.5);
                frame[(size_t)y * w + x] = (uint8_t)(iv8 < 0 ? 0 : iv8 > 255 ? 255 : iv8);
            }
        }
    });
    return SVO_OK;
}
