// svo_orb_detect: cv::ORB::detect for the reference's ORB configuration
// (R:src/tracking.cpp:33-50 creates ORB(nfeatures, scaleFactor, nlevels,
// edgeThreshold = patch_size, firstLevel 0, WTA_K 4, HARRIS_SCORE, patchSize,
// fastThreshold); R:src/tracking.cpp:82 calls detect(img, keypoints, mask) and
// :85 keeps only the positions). Restates features2d/src/orb.cpp
// ORB_Impl::detectAndCompute (keypoints only) + computeKeyPoints:
//
//   level sizes      sz_l = (cvRound(W / s_l), cvRound(H / s_l)),
//                    s_l = (float)pow(scaleFactor, l)
//   image pyramid    level l = resize(level l-1, sz_l, INTER_LINEAR_EXACT)   GPU
//   mask pyramid     same resize, then threshold(254, TOZERO)                GPU
//   per level        FAST(fastThreshold, NMS) with the level mask           GPU
//                    runByImageBorder(edgeThreshold)                        host
//                    retainBest(2 n_l) by FAST response (HARRIS) or n_l     host
//   HARRIS           HarrisResponses(block 7, k 0.04) of every kept point    GPU
//                    retainBest(n_l) per level by Harris response           host
//   output           level order, pt *= s_l
//
// The per-level selection is KeyPointsFilter::retainBest (features2d
// keypoint.cpp): std::nth_element by response, then std::partition of the
// tail by >= the boundary response. Its output ORDER is whatever the C++
// standard library's introselect leaves, so it runs on the host with the same
// algorithms (a few thousand records per level) rather than being re-derived
// on the GPU. n_l: nfeatures (1 - 1/f) / (1 - (1/f)^nlevels) rounded per level,
// the rest to the last level. Keypoint angles (ICAngle) are not computed: the
// reference converts keypoints to points (KeyPoint::convert) right away.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "common.hpp"

namespace svo {

hipError_t launch_orb_resize(const uint8_t* src, int spitch, const uint8_t* smask, int sw, uint8_t* dst, int dpitch,
                             uint8_t* dmask, int dw, int dh, const int* xofs, const uint32_t* xc, const int* yofs,
                             const uint32_t* yc, hipStream_t st);
hipError_t launch_orb_harris(const PyrDesc& levels, int nlevels, const svo_keypoint* kps, const int* n, int cap,
                             int max_n, float* resp, hipStream_t st);

namespace {

// interpolationLinear<uchar>::getCoeffs (resize.cpp), per destination index:
// source offset and the 8-bit fixed-point pair c0 | c1 << 16.
void linear_exact_coeffs(int ssize, int dsize, std::vector<int>& ofs, std::vector<uint32_t>& cf) {
    ofs.resize(dsize);
    cf.resize(dsize);
    const double inv_scale = (double)dsize / ssize;
    const double scale = 1.0 / inv_scale;
    for (int v = 0; v < dsize; v++) {
        const double fval = scale * ((double)v + 0.5) - 0.5;
        const int ival = (int)std::floor(fval);
        if (ival >= 0 && ssize > 1) {
            if (ival < ssize - 1) {
                const int c1 = (int)std::nearbyint((fval - ival) * 256.0);  // ufixedpoint16(softdouble)
                ofs[v] = ival;
                cf[v] = (uint32_t)(256 - c1) | ((uint32_t)c1 << 16);
            } else {  // right of the source: the last sample
                ofs[v] = ssize - 1;
                cf[v] = 256u;
            }
        } else {  // left of the source: the first sample
            ofs[v] = 0;
            cf[v] = 256u;
        }
    }
}

struct OrbKp {  // layout irrelevant to the selection order; mirrors cv::KeyPoint's fields
    float x, y, size, angle, response;
    int octave, class_id;
};

// features2d keypoint.cpp KeyPointsFilter::retainBest
void retain_best(std::vector<OrbKp>& kps, int n_points) {
    if (n_points < 0 || kps.size() <= (size_t)n_points) return;
    if (n_points == 0) {
        kps.clear();
        return;
    }
    std::nth_element(kps.begin(), kps.begin() + n_points - 1, kps.end(),
                     [](const OrbKp& a, const OrbKp& b) { return a.response > b.response; });
    const float amb = kps[n_points - 1].response;
    auto end = std::partition(kps.begin() + n_points, kps.end(), [amb](const OrbKp& k) { return k.response >= amb; });
    kps.resize(end - kps.begin());
}

}  // namespace

// ORB_Impl::computeKeyPoints' nfeaturesPerLevel.
void orb_features_per_level(int nfeatures, double scale_factor, int nlevels, int* out) {
    const float factor = (float)(1.0 / scale_factor);
    float nd = nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nlevels));
    int sum = 0;
    for (int l = 0; l < nlevels - 1; l++) {
        out[l] = (int)std::nearbyint(nd);  // cvRound(float)
        sum += out[l];
        nd *= factor;
    }
    out[nlevels - 1] = std::max(nfeatures - sum, 0);
}

}  // namespace svo

using namespace svo;

extern "C" int svo_orb_detect(svo_ctx* ctx, const svo_image* img, const svo_orb_params* prm, const uint8_t* mask,
                              svo_keypoint* out, int* octave, int cap, int* n_out) {
    if (!ctx || !img || !prm || (!out && cap > 0) || cap < 0)
        return set_error(ctx, SVO_ERR_ARG, "svo_orb_detect: bad arguments");
    const int nlev = prm->nlevels;
    if (nlev < 1 || nlev > kMaxLevels || prm->nfeatures < 0 || !(prm->scale_factor > 1.f) || prm->first_level != 0 ||
        prm->edge_threshold < 4 || prm->patch_size < 2 ||
        (prm->score_type != SVO_ORB_HARRIS_SCORE && prm->score_type != SVO_ORB_FAST_SCORE))
        return set_error(ctx, SVO_ERR_ARG, "svo_orb_detect: unsupported parameters");
    hipStream_t st = ctx->stream;
    const ImgLevel& L0 = img->desc.lv[0];
    const int W = L0.w, H = L0.h;
    const double sf = (double)prm->scale_factor;
    // level geometry (orb.cpp: getScale, layer sizes)
    int lw[kMaxLevels], lh[kMaxLevels], pitch[kMaxLevels], kcap[kMaxLevels], nf[kMaxLevels];
    float lscale[kMaxLevels];
    size_t img_off[kMaxLevels], mask_off[kMaxLevels];
    size_t ibytes = 0, mbytes = 0;
    int maxcap = 0, maxh = 0, maxnseg = 0;
    for (int l = 0; l < nlev; l++) {
        lscale[l] = (float)std::pow(sf, (double)l);
        lw[l] = (int)std::nearbyint((float)W / lscale[l]);
        lh[l] = (int)std::nearbyint((float)H / lscale[l]);
        if (lw[l] < 1 || lh[l] < 1) return set_error(ctx, SVO_ERR_ARG, "svo_orb_detect: image too small");
        pitch[l] = (lw[l] + 63) & ~63;
        img_off[l] = ibytes;
        ibytes += (size_t)pitch[l] * lh[l] + 256;
        ibytes = (ibytes + 255) & ~(size_t)255;
        mask_off[l] = mbytes;
        mbytes += ((size_t)lw[l] * lh[l] + 255) & ~(size_t)255;
        kcap[l] = ((lw[l] + 1) / 2) * ((lh[l] + 1) / 2) + 16;  // NMS maxima: at most one per 2x2 block
        maxcap = std::max(maxcap, kcap[l]);
        maxh = std::max(maxh, lh[l]);
        maxnseg = std::max(maxnseg, (lw[l] + 63) / 64);
    }
    orb_features_per_level(prm->nfeatures, sf, nlev, nf);
    // workspace: level images (level 0 is the caller's image), masks, FAST
    // scratch, keypoints [nlev][maxcap], Harris responses, coefficient tables
    std::vector<int> xo, yo;
    std::vector<uint32_t> xc, yc;
    size_t tab_words = 0;
    for (int l = 1; l < nlev; l++) tab_words += 2 * (size_t)(lw[l] + lh[l]);
    const size_t bits_bytes = sizeof(unsigned long long) * (size_t)maxh * maxnseg;
    size_t off = 0;
    auto take = [&off](size_t b) {
        size_t o = off;
        off = (off + b + 255) & ~(size_t)255;
        return o;
    };
    const size_t o_img = take(ibytes), o_mask = take(mbytes), o_bits = take(bits_bytes),
                 o_rc = take(sizeof(int) * 2 * ((size_t)maxh + 64)),
                 o_kp = take(sizeof(svo_keypoint) * (size_t)nlev * maxcap), o_n = take(sizeof(int) * kMaxLevels),
                 o_resp = take(sizeof(float) * (size_t)nlev * maxcap), o_tab = take(sizeof(uint32_t) * tab_words),
                 o_desc = take(sizeof(PyrDesc) * (kMaxLevels + 1));
    char* ws = (char*)scratch(ctx, 10, off);
    if (!ws) return set_error(ctx, SVO_ERR_HIP, "svo_orb_detect: workspace alloc failed");
    uint8_t* dimg = (uint8_t*)(ws + o_img);
    uint8_t* dmask = mask ? (uint8_t*)(ws + o_mask) : nullptr;
    svo_keypoint* dkp = (svo_keypoint*)(ws + o_kp);
    int* dn = (int*)(ws + o_n);
    float* dresp = (float*)(ws + o_resp);
    // levels as pyramid descriptors (level 0 = the caller's image)
    PyrDesc lev{};
    lev.nlevels = nlev;
    for (int l = 0; l < nlev; l++)
        lev.lv[l] = l == 0 ? L0 : ImgLevel{dimg + img_off[l], lw[l], lh[l], pitch[l]};
    // host staging: tables, per-level descriptors (lv[0] = that level)
    std::vector<uint32_t> tabs(tab_words + 1);
    size_t tw = 0;
    std::vector<size_t> tab_at(kMaxLevels, 0);
    for (int l = 1; l < nlev; l++) {
        linear_exact_coeffs(lw[l - 1], lw[l], xo, xc);
        linear_exact_coeffs(lh[l - 1], lh[l], yo, yc);
        tab_at[l] = tw;
        std::memcpy(&tabs[tw], xo.data(), sizeof(int) * lw[l]);
        tw += lw[l];
        std::memcpy(&tabs[tw], xc.data(), sizeof(uint32_t) * lw[l]);
        tw += lw[l];
        std::memcpy(&tabs[tw], yo.data(), sizeof(int) * lh[l]);
        tw += lh[l];
        std::memcpy(&tabs[tw], yc.data(), sizeof(uint32_t) * lh[l]);
        tw += lh[l];
    }
    const size_t stage_bytes = sizeof(uint32_t) * tab_words + sizeof(PyrDesc) * kMaxLevels;
    char* hst = (char*)pinned(ctx, stage_bytes + 64);
    if (!hst) return set_error(ctx, SVO_ERR_HIP, "svo_orb_detect: pinned alloc failed");
    SVO_HIP(ctx, hipStreamSynchronize(st));  // the pinned buffer may still feed an earlier copy
    std::memcpy(hst, tabs.data(), sizeof(uint32_t) * tab_words);
    PyrDesc* hdesc = (PyrDesc*)(hst + sizeof(uint32_t) * tab_words);
    for (int l = 0; l < nlev; l++) {
        PyrDesc d{};
        d.nlevels = 1;
        d.lv[0] = lev.lv[l];
        std::memcpy(&hdesc[l], &d, sizeof(d));
    }
    uint32_t* dtab = (uint32_t*)(ws + o_tab);
    PyrDesc* ddesc = (PyrDesc*)(ws + o_desc);
    if (tab_words) SVO_HIP(ctx, hipMemcpyAsync(dtab, hst, sizeof(uint32_t) * tab_words, hipMemcpyHostToDevice, st));
    SVO_HIP(ctx, hipMemcpyAsync(ddesc, hdesc, sizeof(PyrDesc) * nlev, hipMemcpyHostToDevice, st));
    if (mask) SVO_HIP(ctx, hipMemcpyAsync(dmask, mask, (size_t)W * H, hipMemcpyHostToDevice, st));
    // scale pyramid (each level from the previous one, as orb.cpp does)
    for (int l = 1; l < nlev; l++) {
        const uint32_t* t = dtab + tab_at[l];
        SVO_HIP(ctx, launch_orb_resize(lev.lv[l - 1].data, lev.lv[l - 1].pitch, dmask ? dmask + mask_off[l - 1] : nullptr,
                                       lw[l - 1], const_cast<uint8_t*>(lev.lv[l].data), pitch[l],
                                       dmask ? dmask + mask_off[l] : nullptr, lw[l], lh[l], (const int*)t,
                                       t + lw[l], (const int*)(t + 2 * lw[l]), t + 2 * lw[l] + lh[l], st));
    }
    // FAST(fastThreshold, NMS) + the level mask, per level
    unsigned long long* bits = (unsigned long long*)(ws + o_bits);
    int* rowcnt = (int*)(ws + o_rc);
    int* rowoff = rowcnt + maxh + 64;
    const int thr = std::min(std::max(prm->fast_threshold, 0), 255);
    for (int l = 0; l < nlev; l++) {
        FastDetBatch b{ddesc + l, dmask ? dmask + mask_off[l] : nullptr, bits, rowcnt, rowoff,
                       dkp + (size_t)l * maxcap, dn + l, (size_t)lw[l] * lh[l], (lw[l] + 63) / 64, kcap[l]};
        SVO_HIP(ctx, launch_fast_detect(b, 1, lw[l], lh[l], thr, 1, st));
    }
    int hn[kMaxLevels] = {0};
    SVO_HIP(ctx, hipMemcpyAsync(hn, dn, sizeof(int) * nlev, hipMemcpyDeviceToHost, st));
    SVO_HIP(ctx, hipStreamSynchronize(st));
    int max_n = 0;
    for (int l = 0; l < nlev; l++) {
        if (hn[l] > kcap[l]) return set_error(ctx, SVO_ERR_CAPACITY, "svo_orb_detect: FAST overflow");
        max_n = std::max(max_n, hn[l]);
    }
    const bool harris = prm->score_type == SVO_ORB_HARRIS_SCORE;
    if (harris) SVO_HIP(ctx, launch_orb_harris(lev, nlev, dkp, dn, maxcap, max_n, dresp, st));
    std::vector<svo_keypoint> hk((size_t)nlev * maxcap);
    std::vector<float> hr(harris ? (size_t)nlev * maxcap : 0);
    for (int l = 0; l < nlev; l++) {
        if (!hn[l]) continue;
        SVO_HIP(ctx, hipMemcpyAsync(&hk[(size_t)l * maxcap], dkp + (size_t)l * maxcap, sizeof(svo_keypoint) * hn[l],
                                    hipMemcpyDeviceToHost, st));
        if (harris)
            SVO_HIP(ctx, hipMemcpyAsync(&hr[(size_t)l * maxcap], dresp + (size_t)l * maxcap, sizeof(float) * hn[l],
                                        hipMemcpyDeviceToHost, st));
    }
    SVO_HIP(ctx, hipStreamSynchronize(st));
    // host selection, level by level (computeKeyPoints)
    const int edge = prm->edge_threshold;
    std::vector<OrbKp> all, lvl;
    std::vector<int> counters(nlev, 0);
    std::vector<float> all_harris;
    for (int l = 0; l < nlev; l++) {
        lvl.clear();
        // runByImageBorder: keep edge <= x < w - edge (same for y); none if the level is too small
        if (!(lh[l] <= edge * 2 || lw[l] <= edge * 2)) {
            for (int i = 0; i < hn[l]; i++) {
                const svo_keypoint& k = hk[(size_t)l * maxcap + i];
                if (k.x >= (float)edge && k.y >= (float)edge && k.x < (float)(lw[l] - edge) &&
                    k.y < (float)(lh[l] - edge))
                    lvl.push_back(OrbKp{k.x, k.y, 7.f, -1.f, k.response, l,
                                        harris ? (int)i : -1});  // class_id carries the GPU index
            }
        }
        retain_best(lvl, harris ? 2 * nf[l] : nf[l]);
        counters[l] = (int)lvl.size();
        for (auto& k : lvl) {
            k.size = prm->patch_size * lscale[l];
            all.push_back(k);
        }
    }
    if (harris) {
        std::vector<OrbKp> sel;
        size_t o = 0;
        for (int l = 0; l < nlev; l++) {
            lvl.assign(all.begin() + o, all.begin() + o + counters[l]);
            o += counters[l];
            for (auto& k : lvl) {
                k.response = hr[(size_t)l * maxcap + k.class_id];
                k.class_id = -1;
            }
            retain_best(lvl, nf[l]);
            sel.insert(sel.end(), lvl.begin(), lvl.end());
        }
        all.swap(sel);
    }
    const int n = (int)all.size();
    for (int i = 0; i < n && i < cap; i++) {
        const float s = lscale[all[i].octave];
        out[i].x = all[i].x * s;
        out[i].y = all[i].y * s;
        out[i].response = all[i].response;
        if (octave) octave[i] = all[i].octave;
    }
    if (n_out) *n_out = n;
    return SVO_OK;
}
