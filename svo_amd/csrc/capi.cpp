// C ABI of libsvo_gpu.so: context, device images, and the host-pointer entry
// points that mirror the reference's OpenCV calls (see include/svo_gpu.h for
// the reference file:line each one replaces).
#include <algorithm>
#include <cstdlib>
#include <cstdarg>
#include <cstring>
#include <vector>

#include "common.hpp"
#include "epnp.hpp"
#include "epnp_ql.hpp"
#include "pose.hpp"

namespace svo {

int set_error(svo_ctx* ctx, int code, const char* fmt, ...) {
    if (ctx) {
        char buf[1024];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof(buf), fmt, ap);
        va_end(ap);
        ctx->err = buf;
    }
    return code;
}

void* scratch(svo_ctx* ctx, int slot, size_t bytes) {
    svo_scratch& s = ctx->s[slot];
    if (s.bytes >= bytes && s.p) return s.p;
    if (s.p) {
        (void)hipStreamSynchronize(ctx->stream);
        (void)hipFree(s.p);
        s.p = nullptr;
        s.bytes = 0;
    }
    size_t want = bytes < 4096 ? 4096 : bytes + bytes / 4;
    if (hipMalloc(&s.p, want) != hipSuccess) {
        s.p = nullptr;
        return nullptr;
    }
    s.bytes = want;
    return s.p;
}

void* pinned(svo_ctx* ctx, size_t bytes) {
    if (ctx->pinned_bytes >= bytes && ctx->pinned) return ctx->pinned;
    if (ctx->pinned) {
        (void)hipStreamSynchronize(ctx->stream);
        (void)hipHostFree(ctx->pinned);
        ctx->pinned = nullptr;
        ctx->pinned_bytes = 0;
    }
    size_t want = bytes < 65536 ? 65536 : bytes + bytes / 4;
    if (hipHostMalloc(&ctx->pinned, want, hipHostMallocDefault) != hipSuccess) {
        ctx->pinned = nullptr;
        return nullptr;
    }
    ctx->pinned_bytes = want;
    return ctx->pinned;
}

int ingest_bgr(svo_ctx* ctx, const uint8_t* bgr, int stride, int w, int h, uint8_t* level0, int pitch) {
    const int bp = (3 * w + 63) & ~63;
    const size_t bytes = (size_t)bp * h;
    const int i = ctx->ingest_next;
    ctx->ingest_next ^= 1;
    if (!ctx->ingest_ev[i]) SVO_HIP(ctx, hipEventCreateWithFlags(&ctx->ingest_ev[i], hipEventDisableTiming));
    else SVO_HIP(ctx, hipEventSynchronize(ctx->ingest_ev[i]));  // buffer i's previous H2D is done
    if (ctx->ingest_bytes[i] < bytes) {
        if (ctx->ingest_host[i]) (void)hipHostFree(ctx->ingest_host[i]);
        ctx->ingest_host[i] = nullptr;
        ctx->ingest_bytes[i] = 0;
        SVO_HIP(ctx, hipHostMalloc(&ctx->ingest_host[i], bytes, hipHostMallocDefault));
        ctx->ingest_bytes[i] = bytes;
    }
    uint8_t* hb = (uint8_t*)ctx->ingest_host[i];
    for (int y = 0; y < h; y++) std::memcpy(hb + (size_t)y * bp, bgr + (size_t)y * stride, (size_t)3 * w);
    uint8_t* dev = (uint8_t*)scratch(ctx, 8 + i, bytes);
    if (!dev) return set_error(ctx, SVO_ERR_HIP, "ingest: scratch alloc failed");
    SVO_HIP(ctx, hipMemcpyAsync(dev, hb, bytes, hipMemcpyHostToDevice, ctx->stream));
    SVO_HIP(ctx, hipEventRecord(ctx->ingest_ev[i], ctx->stream));
    SVO_HIP(ctx, launch_bgr_to_gray(dev, bp, level0, pitch, w, h, ctx->stream));
    return SVO_OK;
}

// Upload one pyramid descriptor to device scratch slot 3's head (single-image calls).
static PyrDesc* stage_desc(svo_ctx* ctx, const svo_image* img, void* dst) {
    PyrDesc* h = (PyrDesc*)pinned(ctx, sizeof(PyrDesc));
    if (!h || hipStreamSynchronize(ctx->stream) != hipSuccess) return nullptr;
    *h = img->desc;
    if (hipMemcpyAsync(dst, h, sizeof(PyrDesc), hipMemcpyHostToDevice, ctx->stream) != hipSuccess) return nullptr;
    return (PyrDesc*)dst;
}

}  // namespace svo

using namespace svo;

namespace svo {
int download_deriv_level(svo_ctx* ctx, const DerivDesc& dd, int level, int w, int h, int16_t* ix, int16_t* iy,
                         int stride) {
    std::vector<uint32_t> v((size_t)w * h);
    SVO_HIP(ctx, hipMemcpy2D(v.data(), (size_t)w * 4, dd.data[level], (size_t)dd.pitch[level] * 4, (size_t)w * 4, h,
                             hipMemcpyDeviceToHost));
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            const uint32_t p = v[(size_t)y * w + x];
            if (ix) ix[(size_t)y * stride + x] = (int16_t)(p & 0xFFFFu);
            if (iy) iy[(size_t)y * stride + x] = (int16_t)(p >> 16);
        }
    return SVO_OK;
}
}  // namespace svo

extern "C" {

const char* svo_version(void) { return "svo_gpu gfx950 hip " SVO_HIP_VERSION_STR; }

int svo_ctx_create(int device, svo_ctx** out) {
    if (!out) return SVO_ERR_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return SVO_ERR_NODEVICE;
    if (device < 0 || device >= ndev) return SVO_ERR_ARG;
    if (hipSetDevice(device) != hipSuccess) return SVO_ERR_HIP;
    // spin-wait host synchronisation: the front end syncs a few times per frame
    // and a sleeping wake-up costs tens of microseconds (fails harmlessly if the
    // device was already initialised with other flags)
    (void)hipSetDeviceFlags(hipDeviceScheduleSpin);
    svo_ctx* c = new svo_ctx();
    c->device = device;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return SVO_ERR_HIP;
    }
    *out = c;
    return SVO_OK;
}

void svo_ctx_destroy(svo_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    for (auto& s : ctx->s)
        if (s.p) (void)hipFree(s.p);
    if (ctx->pinned) (void)hipHostFree(ctx->pinned);
    for (int i = 0; i < 2; i++) {
        if (ctx->ingest_host[i]) (void)hipHostFree(ctx->ingest_host[i]);
        if (ctx->ingest_ev[i]) (void)hipEventDestroy(ctx->ingest_ev[i]);
    }
    for (hipStream_t st : {ctx->fe_lk, ctx->fe_fast, ctx->fe_copy, ctx->fe_up})
        if (st) {
            (void)hipStreamSynchronize(st);
            (void)hipStreamDestroy(st);
        }
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

const char* svo_last_error(const svo_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int svo_ctx_synchronize(svo_ctx* ctx) {
    if (!ctx) return SVO_ERR_ARG;
    SVO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return SVO_OK;
}

// ------------------------------------------------------------------ images
int svo_image_create(svo_ctx* ctx, int w, int h, int max_levels, svo_image** out) {
    if (!ctx || !out || w <= 0 || h <= 0 || max_levels < 0)
        return set_error(ctx, SVO_ERR_ARG, "svo_image_create: bad arguments");
    if (max_levels > kMaxLevels - 1) max_levels = kMaxLevels - 1;
    (void)hipSetDevice(ctx->device);
    svo_image* im = new svo_image();
    im->w = w;
    im->h = h;
    im->nlevels = max_levels + 1;
    size_t off[kMaxLevels];
    size_t total = 0;
    int lw = w, lh = h;
    for (int l = 0; l < im->nlevels; l++) {
        // + 4: the border writer's last dword of a row may pass column w + kPyrPad - 1
        int pitch = (lw + 2 * kPyrPad + 4 + 63) & ~63;
        off[l] = total + (size_t)kPyrPad * pitch + kPyrPad;
        total += (size_t)pitch * (lh + 2 * kPyrPad);
        total = (total + 255) & ~(size_t)255;
        im->desc.lv[l].w = lw;
        im->desc.lv[l].h = lh;
        im->desc.lv[l].pitch = pitch;
        lw = (lw + 1) / 2;
        lh = (lh + 1) / 2;
    }
    total += 256;  // over-read slack: the LK stager loads whole aligned dwords past a row's end
    if (hipMalloc(&im->base, total) != hipSuccess) {
        delete im;
        return set_error(ctx, SVO_ERR_HIP, "svo_image_create: hipMalloc(%zu) failed", total);
    }
    im->bytes = total;
    for (int l = 0; l < im->nlevels; l++) im->desc.lv[l].data = im->base + off[l];
    im->desc.nlevels = im->nlevels;
    *out = im;
    return SVO_OK;
}

void svo_image_destroy(svo_ctx* ctx, svo_image* img) {
    if (!img) return;
    if (ctx) (void)hipStreamSynchronize(ctx->stream);
    if (img->base) (void)hipFree(img->base);
    delete img;
}

int svo_image_build_pyramid(svo_ctx* ctx, svo_image* img) {
    if (!ctx || !img) return SVO_ERR_ARG;
    SVO_HIP(ctx, launch_pyramid(img, 1, ctx->stream));
    return SVO_OK;
}

int svo_image_upload(svo_ctx* ctx, svo_image* img, const uint8_t* gray, int stride) {
    if (!ctx || !img || !gray || stride < img->w)
        return set_error(ctx, SVO_ERR_ARG, "svo_image_upload: bad arguments");
    const ImgLevel& L = img->desc.lv[0];
    SVO_HIP(ctx, hipMemcpy2DAsync(const_cast<uint8_t*>(L.data), L.pitch, gray, stride, L.w, L.h,
                                  hipMemcpyHostToDevice, ctx->stream));
    return svo_image_build_pyramid(ctx, img);
}

int svo_image_upload_bgr(svo_ctx* ctx, svo_image* img, const uint8_t* bgr, int stride) {
    if (!ctx || !img || !bgr || stride < 3 * img->w)
        return set_error(ctx, SVO_ERR_ARG, "svo_image_upload_bgr: bad arguments");
    const ImgLevel& L = img->desc.lv[0];
    int rc = ingest_bgr(ctx, bgr, stride, L.w, L.h, const_cast<uint8_t*>(L.data), L.pitch);
    if (rc) return rc;
    return svo_image_build_pyramid(ctx, img);
}

int svo_image_level_size(const svo_image* img, int level, int* w, int* h) {
    if (!img || level < 0 || level >= img->nlevels) return SVO_ERR_ARG;
    if (w) *w = img->desc.lv[level].w;
    if (h) *h = img->desc.lv[level].h;
    return SVO_OK;
}

int svo_image_download_level(svo_ctx* ctx, const svo_image* img, int level, uint8_t* dst, int stride) {
    if (!ctx || !img || !dst || level < 0 || level >= img->nlevels)
        return set_error(ctx, SVO_ERR_ARG, "svo_image_download_level: bad arguments");
    const ImgLevel& L = img->desc.lv[level];
    if (stride < L.w) return set_error(ctx, SVO_ERR_ARG, "svo_image_download_level: stride");
    SVO_HIP(ctx, hipMemcpy2DAsync(dst, stride, L.data, L.pitch, L.w, L.h, hipMemcpyDeviceToHost,
                                  ctx->stream));
    SVO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return SVO_OK;
}


int svo_image_scharr_level(svo_ctx* ctx, const svo_image* img, int level, int16_t* ix, int16_t* iy, int stride) {
    if (!ctx || !img || level < 0 || level >= img->nlevels)
        return set_error(ctx, SVO_ERR_ARG, "svo_image_scharr_level: bad arguments");
    const ImgLevel& L = img->desc.lv[level];
    if (stride < L.w) return set_error(ctx, SVO_ERR_ARG, "svo_image_scharr_level: stride");
    const int nl = level + 1;
    size_t doff[kMaxLevels];
    int dpitch[kMaxLevels];
    const size_t dbytes = deriv_layout(img->w, img->h, nl, doff, dpitch);
    char* d = (char*)scratch(ctx, 8, dbytes + 1024);
    if (!d) return set_error(ctx, SVO_ERR_HIP, "scratch alloc");
    struct Staged {
        PyrDesc pd;
        DerivDesc dd;
    };
    Staged* hs = (Staged*)pinned(ctx, sizeof(Staged));
    if (!hs) return set_error(ctx, SVO_ERR_HIP, "pinned alloc");
    SVO_HIP(ctx, hipStreamSynchronize(ctx->stream));  // pinned staging is reused
    char* dbase = d + 512;
    hs->pd = img->desc;
    for (int l = 0; l < kMaxLevels; l++) {
        hs->dd.data[l] = l < nl ? (uint32_t*)(dbase + doff[l]) : nullptr;
        hs->dd.pitch[l] = l < nl ? dpitch[l] : 0;
    }
    PyrDesc* ddesc = (PyrDesc*)d;
    DerivDesc* dder = (DerivDesc*)(d + 256);
    static_assert(sizeof(PyrDesc) <= 256 && sizeof(DerivDesc) <= 256, "staging slots");
    SVO_HIP(ctx, hipMemcpyAsync(ddesc, &hs->pd, sizeof(PyrDesc), hipMemcpyHostToDevice, ctx->stream));
    SVO_HIP(ctx, hipMemcpyAsync(dder, &hs->dd, sizeof(DerivDesc), hipMemcpyHostToDevice, ctx->stream));
    SVO_HIP(ctx, hipMemsetAsync(dbase, 0, dbytes, ctx->stream));
    SVO_HIP(ctx, launch_scharr(ddesc, dder, 1, img->w, img->h, nl, ctx->stream));
    SVO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return download_deriv_level(ctx, hs->dd, level, L.w, L.h, ix, iy, stride);
}

// ------------------------------------------------------------------ FAST
int svo_fast_score_map(svo_ctx* ctx, const svo_image* img, int threshold, uint8_t* score,
                       uint8_t* corner) {
    if (!ctx || !img) return SVO_ERR_ARG;
    threshold = threshold < 0 ? 0 : threshold > 255 ? 255 : threshold;
    const ImgLevel& L = img->desc.lv[0];
    size_t npx = (size_t)L.w * L.h;
    uint16_t* cs = (uint16_t*)scratch(ctx, 0, npx * 2 + 1024);
    if (!cs) return set_error(ctx, SVO_ERR_HIP, "scratch alloc");
    PyrDesc* dd = stage_desc(ctx, img, (char*)cs + ((npx * 2 + 255) & ~(size_t)255));
    if (!dd) return set_error(ctx, SVO_ERR_HIP, "desc staging");
    FastBatch b{dd, cs, nullptr, nullptr, nullptr, nullptr, npx, 0};
    SVO_HIP(ctx, launch_fast_score(b, 1, L.w, L.h, threshold, 1, ctx->stream));
    std::vector<uint16_t> h(npx);
    SVO_HIP(ctx, hipMemcpyAsync(h.data(), cs, npx * 2, hipMemcpyDeviceToHost, ctx->stream));
    SVO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    for (size_t i = 0; i < npx; i++) {
        if (score) score[i] = (uint8_t)(h[i] & 0xFF);
        if (corner) corner[i] = (uint8_t)(h[i] >> 8);
    }
    return SVO_OK;
}

int svo_fast_detect(svo_ctx* ctx, const svo_image* img, int threshold, int nonmax,
                    const uint8_t* mask, svo_keypoint* out, int cap, int* n_out) {
    if (!ctx || !img || (!out && cap > 0) || cap < 0)
        return set_error(ctx, SVO_ERR_ARG, "svo_fast_detect: bad arguments");
    threshold = threshold < 0 ? 0 : threshold > 255 ? 255 : threshold;
    const ImgLevel& L = img->desc.lv[0];
    const size_t npx = (size_t)L.w * L.h;
    const int nseg = (L.w + 63) / 64;
    const int kcap = cap > 0 ? cap : 1;
    const size_t bbytes = sizeof(unsigned long long) * (size_t)L.h * nseg;
    char* d = (char*)scratch(ctx, 0, bbytes + sizeof(int) * 2 * ((size_t)L.h + 64) + 1024);
    uint8_t* dmask = mask ? (uint8_t*)scratch(ctx, 2, npx) : nullptr;
    svo_keypoint* dout = (svo_keypoint*)scratch(ctx, 3, sizeof(svo_keypoint) * (size_t)kcap + 64);
    if (!d || (mask && !dmask) || !dout) return set_error(ctx, SVO_ERR_HIP, "scratch alloc");
    int* dn = (int*)((char*)dout + sizeof(svo_keypoint) * (size_t)kcap);
    PyrDesc* dd = stage_desc(ctx, img, d);
    if (!dd) return set_error(ctx, SVO_ERR_HIP, "desc staging");
    unsigned long long* bits = (unsigned long long*)(d + 256);
    int* rowcnt = (int*)((char*)bits + ((bbytes + 255) & ~(size_t)255));
    int* rowoff = rowcnt + L.h + 64;
    if (mask) SVO_HIP(ctx, hipMemcpyAsync(dmask, mask, npx, hipMemcpyHostToDevice, ctx->stream));
    FastDetBatch b{dd, dmask, bits, rowcnt, rowoff, dout, dn, npx, nseg, cap};
    b.padded = true;  // an svo_image level
    SVO_HIP(ctx, launch_fast_detect(b, 1, L.w, L.h, threshold, nonmax ? 1 : 0, ctx->stream));
    int n = 0;
    SVO_HIP(ctx, hipMemcpyAsync(&n, dn, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    SVO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    int nc = n < cap ? n : cap;
    if (nc > 0)
        SVO_HIP(ctx, hipMemcpy(out, dout, sizeof(svo_keypoint) * (size_t)nc, hipMemcpyDeviceToHost));
    if (n_out) *n_out = n;
    return SVO_OK;
}

int svo_mask_boxes(svo_ctx* ctx, int w, int h, const float* pts_xy, int n, float half, uint8_t* mask) {
    if (!ctx || w <= 0 || h <= 0 || !mask || n < 0 || (n > 0 && !pts_xy))
        return set_error(ctx, SVO_ERR_ARG, "svo_mask_boxes: bad arguments");
    size_t npx = (size_t)w * h;
    uint8_t* dmask = (uint8_t*)scratch(ctx, 2, npx);
    float* dpts = (float*)scratch(ctx, 4, sizeof(float) * 2 * (size_t)(n > 0 ? n : 1));
    if (!dmask || !dpts) return set_error(ctx, SVO_ERR_HIP, "scratch alloc");
    if (n > 0) SVO_HIP(ctx, hipMemcpyAsync(dpts, pts_xy, sizeof(float) * 2 * n, hipMemcpyHostToDevice, ctx->stream));
    SVO_HIP(ctx, launch_mask_boxes(w, h, dpts, nullptr, n, n, 1, half, dmask, ctx->stream));
    SVO_HIP(ctx, hipMemcpyAsync(mask, dmask, npx, hipMemcpyDeviceToHost, ctx->stream));
    SVO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return SVO_OK;
}

// ------------------------------------------------------------------ bucket
int svo_bucket_features(svo_ctx* ctx, const float* xy, const int* ages, int n, int img_w, int img_h,
                        int bucket_size, int per_bucket, float* xy_out, int* ages_out, int cap,
                        int* n_out) {
    if (!ctx || n < 0 || (n > 0 && !xy) || img_w <= 0 || img_h <= 0 || bucket_size <= 0 ||
        per_bucket <= 0 || cap < 0 || (cap > 0 && !xy_out))
        return set_error(ctx, SVO_ERR_ARG, "svo_bucket_features: bad arguments");
    const int nh = img_h / bucket_size, nw = img_w / bucket_size;
    if (nw <= 0) return set_error(ctx, SVO_ERR_ARG, "svo_bucket_features: bucket wider than image");
    (void)nh;
    size_t scr_ints = bucket_scratch_ints(img_w, img_h, bucket_size, per_bucket, n);
    int* scr = (int*)scratch(ctx, 5, sizeof(int) * scr_ints);
    int ncap = cap > 0 ? cap : 1;
    char* io = (char*)scratch(ctx, 6, sizeof(float) * 2 * ((size_t)n + ncap) + sizeof(int) * ((size_t)n + ncap) + 256);
    if (!scr || !io) return set_error(ctx, SVO_ERR_HIP, "scratch alloc");
    float* dxy = (float*)io;
    int* dages = (int*)(dxy + 2 * (size_t)n);
    float* dxy_out = (float*)(dages + n);
    int* dages_out = (int*)(dxy_out + 2 * (size_t)ncap);
    int* dn = dages_out + ncap;
    if (n > 0) {
        SVO_HIP(ctx, hipMemcpyAsync(dxy, xy, sizeof(float) * 2 * n, hipMemcpyHostToDevice, ctx->stream));
        if (ages) SVO_HIP(ctx, hipMemcpyAsync(dages, ages, sizeof(int) * n, hipMemcpyHostToDevice, ctx->stream));
    }
    BucketBatch bb{dxy, 2, n, nullptr, n, ages ? dages : nullptr, dxy_out, dages_out, cap, dn, scr, scr_ints};
    SVO_HIP(ctx, launch_bucket(bb, 1, img_w, img_h, bucket_size, per_bucket, ctx->stream));
    int tot = 0;
    SVO_HIP(ctx, hipMemcpyAsync(&tot, dn, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    SVO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    int nc = tot < cap ? tot : cap;
    if (nc > 0) {
        SVO_HIP(ctx, hipMemcpy(xy_out, dxy_out, sizeof(float) * 2 * nc, hipMemcpyDeviceToHost));
        if (ages_out) SVO_HIP(ctx, hipMemcpy(ages_out, dages_out, sizeof(int) * nc, hipMemcpyDeviceToHost));
    }
    if (n_out) *n_out = tot;
    return SVO_OK;
}

// ------------------------------------------------------------------ LK
int svo_calc_optical_flow_pyr_lk(svo_ctx* ctx, const svo_image* prev, const svo_image* next,
                                 const float* prev_xy, int n, float* next_xy, uint8_t* status,
                                 float* err, int win_w, int win_h, int max_level, int crit_type,
                                 int max_count, double epsilon, int flags,
                                 double min_eig_threshold) {
    if (!ctx || !prev || !next) return SVO_ERR_ARG;
    ctx->lk_iters = 0;
    if (n == 0) return SVO_OK;  // OpenCV releases the outputs and returns
    if (n < 0 || !prev_xy || !next_xy || !status || max_level < 0 || win_w <= 2 || win_h <= 2)
        return set_error(ctx, SVO_ERR_ARG, "calcOpticalFlowPyrLK: bad arguments (CV_Assert)");
    if (prev->w != next->w || prev->h != next->h)
        return set_error(ctx, SVO_ERR_ARG, "calcOpticalFlowPyrLK: image sizes differ");
    if (!lk_supported(win_w, win_h))
        return set_error(ctx, SVO_ERR_CAPACITY, "calcOpticalFlowPyrLK: window %dx%d unsupported", win_w, win_h);
    // criteria clamping as SparsePyrLKOpticalFlowImpl::calc
    if ((crit_type & SVO_TERM_COUNT) == 0) max_count = 30;
    else max_count = max_count < 0 ? 0 : max_count > 100 ? 100 : max_count;
    if ((crit_type & SVO_TERM_EPS) == 0) epsilon = 0.01;
    else epsilon = epsilon < 0. ? 0. : epsilon > 10. ? 10. : epsilon;
    int ml = lk_levels_for_window(prev->w, prev->h, win_w, win_h, max_level);
    if (ml > prev->nlevels - 1 || ml > next->nlevels - 1)
        return set_error(ctx, SVO_ERR_CAPACITY, "calcOpticalFlowPyrLK: pyramid has %d levels, %d needed",
                         prev->nlevels < next->nlevels ? prev->nlevels : next->nlevels, ml + 1);
    LKParams p;
    p.win_w = win_w;
    p.win_h = win_h;
    p.max_level = ml;
    p.max_count = max_count;
    p.eps2 = epsilon * epsilon;
    p.flags = flags & ~SVO_LK_OPENCV_ORDER;
    p.cv_order = (flags & SVO_LK_OPENCV_ORDER) ? 1 : 0;
    p.min_eig = (float)min_eig_threshold;
    p.want_err = err ? 1 : 0;
    lk_apply_env(p);
    // derivative pyramid of prev (calcSharrDeriv per level), then LK
    size_t doff[kMaxLevels];
    int dpitch[kMaxLevels];
    const size_t dbytes = deriv_layout(prev->w, prev->h, ml + 1, doff, dpitch);
    size_t bytes = (size_t)n * (8 + 8 + 1 + 4 + 4) + 2 * sizeof(PyrDesc) + sizeof(DerivDesc) + dbytes + 2048;
    char* d = (char*)scratch(ctx, 7, bytes);
    if (!d) return set_error(ctx, SVO_ERR_HIP, "scratch alloc");
    PyrDesc* ddesc = (PyrDesc*)d;
    DerivDesc* dder = (DerivDesc*)(d + 2 * sizeof(PyrDesc));
    char* dbase = (char*)(((uintptr_t)(d + 2 * sizeof(PyrDesc) + sizeof(DerivDesc)) + 255) & ~(uintptr_t)255);
    d = dbase + ((dbytes + 255) & ~(size_t)255);
    float* dprev = (float*)d;
    float* dnext = dprev + 2 * (size_t)n;
    float* derr = dnext + 2 * (size_t)n;
    int* diters = (int*)(derr + n);
    uint8_t* dst = (uint8_t*)(diters + n);
    SVO_HIP(ctx, hipMemcpyAsync(dprev, prev_xy, sizeof(float) * 2 * n, hipMemcpyHostToDevice, ctx->stream));
    if (flags & SVO_LK_USE_INITIAL_FLOW)
        SVO_HIP(ctx, hipMemcpyAsync(dnext, next_xy, sizeof(float) * 2 * n, hipMemcpyHostToDevice, ctx->stream));
    struct Staged {
        PyrDesc pd[2];
        DerivDesc dd;
    };
    Staged* hs = (Staged*)pinned(ctx, sizeof(Staged));
    if (!hs) return set_error(ctx, SVO_ERR_HIP, "pinned alloc");
    SVO_HIP(ctx, hipStreamSynchronize(ctx->stream));  // pinned staging is reused
    hs->pd[0] = prev->desc;
    hs->pd[1] = next->desc;
    for (int l = 0; l < kMaxLevels; l++) {
        hs->dd.data[l] = l <= ml ? (uint32_t*)(dbase + doff[l]) : nullptr;
        hs->dd.pitch[l] = l <= ml ? dpitch[l] : 0;
    }
    SVO_HIP(ctx, hipMemcpyAsync(ddesc, hs, sizeof(Staged), hipMemcpyHostToDevice, ctx->stream));
    SVO_HIP(ctx, hipMemsetAsync(dbase, 0, dbytes, ctx->stream));  // the zero borders
    SVO_HIP(ctx, launch_scharr(ddesc, dder, 1, prev->w, prev->h, ml + 1, ctx->stream));
    LKBatch b{ddesc, ddesc + 1, dder, dprev, dnext, dst, err ? derr : nullptr, diters, nullptr, n, n};
    SVO_HIP(ctx, launch_lk(b, 1, n, p, ctx->stream));
    std::vector<int> it(n);
    SVO_HIP(ctx, hipMemcpyAsync(next_xy, dnext, sizeof(float) * 2 * n, hipMemcpyDeviceToHost, ctx->stream));
    SVO_HIP(ctx, hipMemcpyAsync(status, dst, n, hipMemcpyDeviceToHost, ctx->stream));
    if (err) SVO_HIP(ctx, hipMemcpyAsync(err, derr, sizeof(float) * n, hipMemcpyDeviceToHost, ctx->stream));
    SVO_HIP(ctx, hipMemcpyAsync(it.data(), diters, sizeof(int) * n, hipMemcpyDeviceToHost, ctx->stream));
    SVO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    int64_t s = 0;
    for (int v : it) s += v;
    ctx->lk_iters = s;
    return SVO_OK;
}

int64_t svo_lk_last_iterations(const svo_ctx* ctx) { return ctx ? ctx->lk_iters : 0; }

// ------------------------------------------------------------------ PnP residuals
int svo_pnp_residuals(svo_ctx* ctx, const float* obj_xyz, const float* img_xy, int n,
                      const double* hyp_Rt, int m, const double K[9], float thresh2, float* err,
                      uint8_t* mask, int* counts) {
    if (!ctx || n < 0 || m < 0 || (n > 0 && (!obj_xyz || !img_xy)) || (m > 0 && !hyp_Rt) || !K)
        return set_error(ctx, SVO_ERR_ARG, "svo_pnp_residuals: bad arguments");
    if (n == 0 || m == 0) {
        if (counts)
            for (int i = 0; i < m; i++) counts[i] = 0;
        return SVO_OK;
    }
    const int words = (n + 31) / 32;
    size_t bytes = sizeof(float) * 5 * (size_t)n + sizeof(double) * 12 * (size_t)m +
                   (err ? sizeof(float) * (size_t)n * m : 0) + sizeof(uint32_t) * (size_t)words * m +
                   sizeof(int) * (size_t)m + 1024;
    char* d = (char*)scratch(ctx, 7, bytes);
    if (!d) return set_error(ctx, SVO_ERR_HIP, "scratch alloc");
    double* dh = (double*)d;
    float* dobj = (float*)(dh + 12 * (size_t)m);
    float* dimg = dobj + 3 * (size_t)n;
    int* dcnt = (int*)(dimg + 2 * (size_t)n);
    uint32_t* dbits = (uint32_t*)(dcnt + m);
    float* derr = err ? (float*)(dbits + (size_t)words * m) : nullptr;
    SVO_HIP(ctx, hipMemcpyAsync(dh, hyp_Rt, sizeof(double) * 12 * m, hipMemcpyHostToDevice, ctx->stream));
    SVO_HIP(ctx, hipMemcpyAsync(dobj, obj_xyz, sizeof(float) * 3 * n, hipMemcpyHostToDevice, ctx->stream));
    SVO_HIP(ctx, hipMemcpyAsync(dimg, img_xy, sizeof(float) * 2 * n, hipMemcpyHostToDevice, ctx->stream));
    PnpBatch b{dobj, dimg, nullptr, n, n, dh, m, derr, dbits, words, dcnt};
    SVO_HIP(ctx, launch_pnp_residuals(b, 1, n, K[0], K[4], K[2], K[5], thresh2, ctx->stream));
    std::vector<uint32_t> bits((size_t)words * m);
    SVO_HIP(ctx, hipMemcpyAsync(bits.data(), dbits, sizeof(uint32_t) * bits.size(), hipMemcpyDeviceToHost, ctx->stream));
    if (counts) SVO_HIP(ctx, hipMemcpyAsync(counts, dcnt, sizeof(int) * m, hipMemcpyDeviceToHost, ctx->stream));
    if (err) SVO_HIP(ctx, hipMemcpyAsync(err, derr, sizeof(float) * (size_t)n * m, hipMemcpyDeviceToHost, ctx->stream));
    SVO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (mask)
        for (int h = 0; h < m; h++)
            for (int i = 0; i < n; i++) mask[(size_t)h * n + i] = (bits[(size_t)h * words + (i >> 5)] >> (i & 31)) & 1;
    return SVO_OK;
}

int svo_epnp_subsets(svo_ctx* ctx, const float* subsets, int m, const double K[9], int device, double* Rt,
                     int* ok) {
    if ((!ctx && (device == 1 || device == 6)) || device < 0 || device > 6 || m < 0 ||
        (m > 0 && (!subsets || !Rt || !ok)) || !K)
        return set_error(ctx, SVO_ERR_ARG, "svo_epnp_subsets: bad arguments");
    // 0: the front end's solver as dispatched; 3 / 4 / 5: forced scalar / AVX2 / AVX-512
    const int isa = device == 3 ? kEpnpScalar : device == 4 ? kEpnpAvx2 : device == 5 ? kEpnpAvx512 : kEpnpAuto;
    if (device >= 3 && device <= 5 && !epnp_isa_supported(isa))
        return set_error(ctx, SVO_ERR_NODEVICE, "svo_epnp_subsets: instruction set not on this CPU");
    if (m == 0) return SVO_OK;
    if (device == 2) {  // the device solver's host twin (epnp_ql.hpp)
        for (int j = 0; j < m; j++) {
            const float* sp = subsets + 25 * (size_t)j;
            double R[9], t[3];
            ok[j] = epnp_pixels_ql(sp, sp + 15, nullptr, 5, K, R, t) ? 1 : 0;
            std::memcpy(Rt + 12 * (size_t)j, R, sizeof(R));
            std::memcpy(Rt + 12 * (size_t)j + 9, t, sizeof(t));
        }
        return SVO_OK;
    }
    if (device == 0 || (device >= 3 && device <= 5)) {  // the front end's host solver, kEpnpLanes at a time
        for (int j0 = 0; j0 < m; j0 += kEpnpLanes) {
            const int c = std::min(kEpnpLanes, m - j0);
            const float *o[kEpnpLanes], *im[kEpnpLanes];
            const int* id[kEpnpLanes];
            double R[kEpnpLanes][9], t[kEpnpLanes][3];
            bool v[kEpnpLanes];
            for (int q = 0; q < c; q++) {
                o[q] = subsets + 25 * (size_t)(j0 + q);
                im[q] = o[q] + 15;
                id[q] = nullptr;
            }
            epnp_pixels_batch(c, o, im, id, K, R, t, v, isa);
            for (int q = 0; q < c; q++) {
                ok[j0 + q] = v[q] ? 1 : 0;
                std::memcpy(Rt + 12 * (size_t)(j0 + q), R[q], sizeof(R[q]));
                std::memcpy(Rt + 12 * (size_t)(j0 + q) + 9, t[q], sizeof(t[q]));
            }
        }
        return SVO_OK;
    }
    const size_t bytes = sizeof(double) * (9 + 12 * (size_t)m) + sizeof(float) * 25 * (size_t)m + sizeof(int) * m + 1024;
    char* d = (char*)scratch(ctx, 9, bytes);
    if (!d) return set_error(ctx, SVO_ERR_HIP, "scratch alloc");
    double* dK = (double*)d;
    double* dRt = dK + 9;
    float* dsub = (float*)(dRt + 12 * (size_t)m);
    int* dok = (int*)(dsub + 25 * (size_t)m);
    SVO_HIP(ctx, hipMemcpyAsync(dK, K, sizeof(double) * 9, hipMemcpyHostToDevice, ctx->stream));
    SVO_HIP(ctx, hipMemcpyAsync(dsub, subsets, sizeof(float) * 25 * (size_t)m, hipMemcpyHostToDevice, ctx->stream));
    // 1: a wave per subset (the QL variant); 6: a lane per subset (the front end's solver)
    SVO_HIP(ctx, device == 6 ? launch_epnp_lanes(dsub, m, dK, dRt, dok, ctx->stream)
                             : launch_epnp_wave(dsub, m, dK, dRt, dok, ctx->stream));
    SVO_HIP(ctx, hipMemcpyAsync(Rt, dRt, sizeof(double) * 12 * (size_t)m, hipMemcpyDeviceToHost, ctx->stream));
    SVO_HIP(ctx, hipMemcpyAsync(ok, dok, sizeof(int) * (size_t)m, hipMemcpyDeviceToHost, ctx->stream));
    SVO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return SVO_OK;
}

int svo_triangulate_points(svo_ctx* ctx, const float P1[12], const float P2[12], const float* pts1,
                           const float* pts2, int n, float* xyzw, float* xyz) {
    if (!ctx || !P1 || !P2 || n < 0 || (n > 0 && (!pts1 || !pts2)))
        return set_error(ctx, SVO_ERR_ARG, "svo_triangulate_points: bad arguments");
    if (n == 0) return SVO_OK;
    const size_t bytes = sizeof(float) * (24 + 4 * (size_t)n + 7 * (size_t)n) + 1024;
    float* d = (float*)scratch(ctx, 6, bytes);
    if (!d) return set_error(ctx, SVO_ERR_HIP, "scratch alloc");
    float* dP = d;
    float* dp1 = dP + 24;
    float* dp2 = dp1 + 2 * (size_t)n;
    float* dh = dp2 + 2 * (size_t)n;
    float* dx = dh + 4 * (size_t)n;
    SVO_HIP(ctx, hipMemcpyAsync(dP, P1, sizeof(float) * 12, hipMemcpyHostToDevice, ctx->stream));
    SVO_HIP(ctx, hipMemcpyAsync(dP + 12, P2, sizeof(float) * 12, hipMemcpyHostToDevice, ctx->stream));
    SVO_HIP(ctx, hipMemcpyAsync(dp1, pts1, sizeof(float) * 2 * n, hipMemcpyHostToDevice, ctx->stream));
    SVO_HIP(ctx, hipMemcpyAsync(dp2, pts2, sizeof(float) * 2 * n, hipMemcpyHostToDevice, ctx->stream));
    SVO_HIP(ctx, launch_triangulate(dP, dp1, dp2, n, dh, dx, ctx->stream));
    if (xyzw) SVO_HIP(ctx, hipMemcpyAsync(xyzw, dh, sizeof(float) * 4 * n, hipMemcpyDeviceToHost, ctx->stream));
    if (xyz) SVO_HIP(ctx, hipMemcpyAsync(xyz, dx, sizeof(float) * 3 * n, hipMemcpyDeviceToHost, ctx->stream));
    SVO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return SVO_OK;
}

// Page-locked host memory for frames streamed with svo_frontend_queue_frames
// (the reference's loader thread would decode into it: an H2D from pageable
// memory is staged through a driver bounce buffer at a fraction of the rate).
int svo_pinned_alloc(size_t bytes, void** out) {
    if (!out || bytes == 0) return SVO_ERR_ARG;
    *out = nullptr;
    if (hipHostMalloc(out, bytes, hipHostMallocDefault) != hipSuccess) {
        *out = nullptr;
        return SVO_ERR_HIP;
    }
    return SVO_OK;
}

void svo_pinned_free(void* p) {
    if (p) (void)hipHostFree(p);
}

}  // extern "C"
