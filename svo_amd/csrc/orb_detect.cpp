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
#include <string>
#include <vector>

#include "common.hpp"
#include "orb.hpp"

namespace svo {

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


bool orb_geometry(int W, int H, const svo_orb_params& p, OrbGeometry& g, const char** err) {
    const int nlev = p.nlevels;
    if (nlev < 1 || nlev > kMaxLevels || p.nfeatures < 0 || !(p.scale_factor > 1.f) || p.first_level != 0 ||
        p.edge_threshold < 4 || p.patch_size < 2 ||
        (p.score_type != SVO_ORB_HARRIS_SCORE && p.score_type != SVO_ORB_FAST_SCORE)) {
        *err = "unsupported parameters";
        return false;
    }
    const double sf = (double)p.scale_factor;
    g.nlev = nlev;
    g.maxcap = g.maxh = g.maxnseg = 0;
    for (int l = 0; l < nlev; l++) {  // orb.cpp: getScale, layer sizes
        g.lscale[l] = (float)std::pow(sf, (double)l);
        g.lw[l] = (int)std::nearbyint((float)W / g.lscale[l]);
        g.lh[l] = (int)std::nearbyint((float)H / g.lscale[l]);
        if (g.lw[l] < 1 || g.lh[l] < 1) {
            *err = "image too small";
            return false;
        }
        g.pitch[l] = (g.lw[l] + 63) & ~63;
        g.kcap[l] = ((g.lw[l] + 1) / 2) * ((g.lh[l] + 1) / 2) + 16;  // NMS maxima: at most one per 2x2 block
        g.maxcap = std::max(g.maxcap, g.kcap[l]);
        g.maxh = std::max(g.maxh, g.lh[l]);
        g.maxnseg = std::max(g.maxnseg, (g.lw[l] + 63) / 64);
    }
    orb_features_per_level(p.nfeatures, sf, nlev, g.nf);
    std::vector<int> xo, yo;
    std::vector<uint32_t> xc, yc;
    g.tabs.clear();
    for (int l = 1; l < nlev; l++) {
        linear_exact_coeffs(g.lw[l - 1], g.lw[l], xo, xc);
        linear_exact_coeffs(g.lh[l - 1], g.lh[l], yo, yc);
        g.tab_at[l] = g.tabs.size();
        g.tabs.insert(g.tabs.end(), xo.begin(), xo.end());
        g.tabs.insert(g.tabs.end(), xc.begin(), xc.end());
        g.tabs.insert(g.tabs.end(), yo.begin(), yo.end());
        g.tabs.insert(g.tabs.end(), yc.begin(), yc.end());
    }
    return true;
}

int orb_select(const OrbGeometry& g, const svo_orb_params& p, const svo_keypoint* const* kps,
               const float* const* resp, const int* n, svo_keypoint* out, int* octave, int cap) {
    const int nlev = g.nlev, edge = p.edge_threshold;
    const bool harris = p.score_type == SVO_ORB_HARRIS_SCORE;
    std::vector<OrbKp> all, lvl;
    std::vector<int> counters(nlev, 0);
    for (int l = 0; l < nlev; l++) {
        lvl.clear();
        // runByImageBorder: keep edge <= x < w - edge (same for y); none if the level is too small
        if (!(g.lh[l] <= edge * 2 || g.lw[l] <= edge * 2)) {
            for (int i = 0; i < n[l]; i++) {
                const svo_keypoint& k = kps[l][i];
                if (k.x >= (float)edge && k.y >= (float)edge && k.x < (float)(g.lw[l] - edge) &&
                    k.y < (float)(g.lh[l] - edge))
                    lvl.push_back(OrbKp{k.x, k.y, 7.f, -1.f, k.response, l,
                                        harris ? (int)i : -1});  // class_id carries the GPU index
            }
        }
        retain_best(lvl, harris ? 2 * g.nf[l] : g.nf[l]);
        counters[l] = (int)lvl.size();
        for (auto& k : lvl) {
            k.size = p.patch_size * g.lscale[l];
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
                k.response = resp[l][k.class_id];
                k.class_id = -1;
            }
            retain_best(lvl, g.nf[l]);
            sel.insert(sel.end(), lvl.begin(), lvl.end());
        }
        all.swap(sel);
    }
    const int total = (int)all.size();
    for (int i = 0; i < total && i < cap; i++) {
        const float sc = g.lscale[all[i].octave];
        out[i].x = all[i].x * sc;
        out[i].y = all[i].y * sc;
        out[i].response = all[i].response;
        if (octave) octave[i] = all[i].octave;
    }
    return total;
}

struct OrbBatch {
    int S = 0, W = 0, H = 0;
    svo_orb_params p{};
    OrbGeometry g;
    void* mem = nullptr;                      // device: everything below
    uint8_t* img = nullptr;                   // levels 1.. of every sequence: [s][img_off[l]]
    size_t img_off[kMaxLevels] = {0}, img_seq = 0;
    uint8_t* mask = nullptr;                  // [l][s][lw * lh]
    size_t mask_off[kMaxLevels] = {0};
    unsigned long long* bits = nullptr;       // FAST scratch of one level: [s][maxh][maxnseg]
    int *rowcnt = nullptr, *rowoff = nullptr; // [s][maxh]
    svo_keypoint* kps = nullptr;              // [l][s][maxcap]
    float* resp = nullptr;                    // [l][s][maxcap]
    int* n = nullptr;                         // [l][s]
    uint32_t* tabs = nullptr;
    PyrDesc* desc = nullptr;                  // [l][s]: lv[0] = level l of sequence s
    std::vector<PyrDesc> hdesc;
    std::vector<int> hn;
    std::vector<svo_keypoint> hk, hsel;
    std::vector<float> hr;
    std::vector<int> hcnt;
};

OrbBatch* orb_batch_create(int S, int W, int H, const svo_orb_params& p) {
    auto* ob = new OrbBatch();
    ob->S = S;
    ob->W = W;
    ob->H = H;
    ob->p = p;
    const char* err = nullptr;
    if (S <= 0 || !orb_geometry(W, H, p, ob->g, &err)) {
        delete ob;
        return nullptr;
    }
    const OrbGeometry& g = ob->g;
    size_t off = 0;
    auto take = [&off](size_t b) {
        const size_t o = off;
        off = (off + b + 255) & ~(size_t)255;
        return o;
    };
    size_t img_seq = 0;
    for (int l = 1; l < g.nlev; l++) {
        ob->img_off[l] = img_seq;
        img_seq = (img_seq + (size_t)g.pitch[l] * g.lh[l] + 256 + 255) & ~(size_t)255;
    }
    ob->img_seq = img_seq;
    size_t mask_bytes = 0;
    for (int l = 0; l < g.nlev; l++) {
        ob->mask_off[l] = mask_bytes;
        mask_bytes += ((size_t)S * g.lw[l] * g.lh[l] + 255) & ~(size_t)255;
    }
    const size_t LS = (size_t)g.nlev * S;
    const size_t o_img = take(img_seq * S), o_mask = take(mask_bytes),
                 o_bits = take(sizeof(unsigned long long) * S * (size_t)g.maxh * g.maxnseg),
                 o_rc = take(sizeof(int) * S * (size_t)g.maxh), o_ro = take(sizeof(int) * S * (size_t)g.maxh),
                 o_kp = take(sizeof(svo_keypoint) * LS * g.maxcap), o_resp = take(sizeof(float) * LS * g.maxcap),
                 o_n = take(sizeof(int) * LS), o_tab = take(sizeof(uint32_t) * (g.tabs.size() + 1)),
                 o_desc = take(sizeof(PyrDesc) * LS);
    if (hipMalloc(&ob->mem, off) != hipSuccess) {
        delete ob;
        return nullptr;
    }
    char* b = (char*)ob->mem;
    ob->img = (uint8_t*)(b + o_img);
    ob->mask = (uint8_t*)(b + o_mask);
    ob->bits = (unsigned long long*)(b + o_bits);
    ob->rowcnt = (int*)(b + o_rc);
    ob->rowoff = (int*)(b + o_ro);
    ob->kps = (svo_keypoint*)(b + o_kp);
    ob->resp = (float*)(b + o_resp);
    ob->n = (int*)(b + o_n);
    ob->tabs = (uint32_t*)(b + o_tab);
    ob->desc = (PyrDesc*)(b + o_desc);
    if (!g.tabs.empty() &&
        hipMemcpy(ob->tabs, g.tabs.data(), sizeof(uint32_t) * g.tabs.size(), hipMemcpyHostToDevice) != hipSuccess) {
        orb_batch_destroy(ob);
        return nullptr;
    }
    ob->hdesc.assign(LS, PyrDesc{});
    for (int l = 1; l < g.nlev; l++)
        for (int s = 0; s < S; s++) {
            PyrDesc& d = ob->hdesc[(size_t)l * S + s];
            d.nlevels = 1;
            d.lv[0] = ImgLevel{ob->img + (size_t)s * img_seq + ob->img_off[l], g.lw[l], g.lh[l], g.pitch[l]};
        }
    return ob;
}

void orb_batch_destroy(OrbBatch* ob) {
    if (!ob) return;
    if (ob->mem) (void)hipFree(ob->mem);
    delete ob;
}

hipError_t orb_batch_detect(OrbBatch* ob, const ImgLevel* lv0, const float* box_pts, const int* box_counts,
                            int box_stride, int box_max, float half, svo_keypoint* out, int* nout, int cap_out,
                            hipStream_t st, const std::function<void(int, const std::function<void(int)>&)>& par,
                            int* overflow) {
#define ORB_HIP(x)                          \
    do {                                    \
        const hipError_t e_ = (x);          \
        if (e_ != hipSuccess) return e_;    \
    } while (0)
    const OrbGeometry& g = ob->g;
    const int S = ob->S, nlev = g.nlev;
    const size_t LS = (size_t)nlev * S;
    for (int s = 0; s < S; s++) {
        PyrDesc& d = ob->hdesc[s];
        d.nlevels = 1;
        d.lv[0] = lv0[s];
    }
    ORB_HIP(hipMemcpyAsync(ob->desc, ob->hdesc.data(), sizeof(PyrDesc) * LS, hipMemcpyHostToDevice, st));
    uint8_t* m0 = box_pts ? ob->mask + ob->mask_off[0] : nullptr;
    if (m0) {  // the reference's mask: 255 with a filled box around each previous feature
        ORB_HIP(hipMemsetAsync(m0, 255, (size_t)S * g.lw[0] * g.lh[0], st));
        ORB_HIP(launch_mask_boxes(g.lw[0], g.lh[0], box_pts, box_counts, box_max, box_stride, S, half, m0, st));
    }
    // scale pyramid and mask pyramid, each level from the previous one (orb.cpp)
    for (int l = 1; l < nlev; l++) {
        const uint32_t* t = ob->tabs + g.tab_at[l];
        ORB_HIP(launch_orb_resize_batched(ob->desc + (size_t)(l - 1) * S, ob->desc + (size_t)l * S,
                                          m0 ? ob->mask + ob->mask_off[l - 1] : nullptr,
                                          (size_t)g.lw[l - 1] * g.lh[l - 1], g.lw[l - 1],
                                          m0 ? ob->mask + ob->mask_off[l] : nullptr, (size_t)g.lw[l] * g.lh[l],
                                          g.lw[l], g.lh[l], S, (const int*)t, t + g.lw[l],
                                          (const int*)(t + 2 * g.lw[l]), t + 2 * g.lw[l] + g.lh[l], st));
    }
    // FAST(fastThreshold, NMS) + the level mask, per level, every sequence at once
    const int thr = std::min(std::max(ob->p.fast_threshold, 0), 255);
    for (int l = 0; l < nlev; l++) {
        FastDetBatch b{ob->desc + (size_t)l * S, m0 ? ob->mask + ob->mask_off[l] : nullptr, ob->bits, ob->rowcnt,
                       ob->rowoff, ob->kps + (size_t)l * S * g.maxcap, ob->n + (size_t)l * S,
                       (size_t)g.lw[l] * g.lh[l], (g.lw[l] + 63) / 64, g.maxcap};
        ORB_HIP(launch_fast_detect(b, S, g.lw[l], g.lh[l], thr, 1, st));
    }
    ob->hn.assign(LS, 0);
    ORB_HIP(hipMemcpyAsync(ob->hn.data(), ob->n, sizeof(int) * LS, hipMemcpyDeviceToHost, st));
    ORB_HIP(hipStreamSynchronize(st));
    int max_n = 0, lmax[kMaxLevels] = {0};
    for (int l = 0; l < nlev; l++)
        for (int s = 0; s < S; s++) {
            const int v = ob->hn[(size_t)l * S + s];
            if (v > g.kcap[l]) return hipErrorInvalidValue;  // cannot happen: NMS keeps <= 1 per 2x2
            lmax[l] = std::max(lmax[l], v);
            max_n = std::max(max_n, v);
        }
    const bool harris = ob->p.score_type == SVO_ORB_HARRIS_SCORE;
    if (harris) ORB_HIP(launch_orb_harris_batched(ob->desc, nlev, S, ob->kps, ob->n, g.maxcap, max_n, ob->resp, st));
    // the keypoints (and responses) of every (level, sequence), lmax[l] per row
    size_t hoff[kMaxLevels], htot = 0;
    for (int l = 0; l < nlev; l++) {
        hoff[l] = htot;
        htot += (size_t)S * lmax[l];
    }
    ob->hk.resize(htot + 1);
    ob->hr.resize(harris ? htot + 1 : 0);
    for (int l = 0; l < nlev; l++) {
        if (!lmax[l]) continue;
        ORB_HIP(hipMemcpy2DAsync(ob->hk.data() + hoff[l], sizeof(svo_keypoint) * lmax[l],
                                 ob->kps + (size_t)l * S * g.maxcap, sizeof(svo_keypoint) * g.maxcap,
                                 sizeof(svo_keypoint) * lmax[l], S, hipMemcpyDeviceToHost, st));
        if (harris)
            ORB_HIP(hipMemcpy2DAsync(ob->hr.data() + hoff[l], sizeof(float) * lmax[l],
                                     ob->resp + (size_t)l * S * g.maxcap, sizeof(float) * g.maxcap,
                                     sizeof(float) * lmax[l], S, hipMemcpyDeviceToHost, st));
    }
    ORB_HIP(hipStreamSynchronize(st));
    // host selection per sequence
    ob->hsel.resize((size_t)S * cap_out + 1);
    ob->hcnt.assign(S, 0);
    par(S, [&](int s) {
        const svo_keypoint* kp[kMaxLevels];
        const float* rp[kMaxLevels];
        int nn[kMaxLevels];
        for (int l = 0; l < nlev; l++) {
            kp[l] = ob->hk.data() + hoff[l] + (size_t)s * lmax[l];
            rp[l] = harris ? ob->hr.data() + hoff[l] + (size_t)s * lmax[l] : nullptr;
            nn[l] = ob->hn[(size_t)l * S + s];
        }
        const int tot = orb_select(g, ob->p, kp, rp, nn, ob->hsel.data() + (size_t)s * cap_out, nullptr, cap_out);
        ob->hcnt[s] = std::min(tot, cap_out);
        if (overflow) overflow[s] = std::max(tot - cap_out, 0);
    });
    int maxsel = 0;
    for (int s = 0; s < S; s++) maxsel = std::max(maxsel, ob->hcnt[s]);
    if (maxsel)
        ORB_HIP(hipMemcpy2DAsync(out, sizeof(svo_keypoint) * cap_out, ob->hsel.data(), sizeof(svo_keypoint) * cap_out,
                                 sizeof(svo_keypoint) * maxsel, S, hipMemcpyHostToDevice, st));
    ORB_HIP(hipMemcpyAsync(nout, ob->hcnt.data(), sizeof(int) * S, hipMemcpyHostToDevice, st));
    // the host vectors feed copies still in flight: wait for them
    ORB_HIP(hipStreamSynchronize(st));
    return hipSuccess;
#undef ORB_HIP
}

}  // namespace svo

using namespace svo;

extern "C" int svo_orb_detect(svo_ctx* ctx, const svo_image* img, const svo_orb_params* prm, const uint8_t* mask,
                              svo_keypoint* out, int* octave, int cap, int* n_out) {
    if (!ctx || !img || !prm || (!out && cap > 0) || cap < 0)
        return set_error(ctx, SVO_ERR_ARG, "svo_orb_detect: bad arguments");
    hipStream_t st = ctx->stream;
    const ImgLevel& L0 = img->desc.lv[0];
    const int W = L0.w, H = L0.h;
    OrbGeometry g;
    const char* why = nullptr;
    if (!orb_geometry(W, H, *prm, g, &why))
        return set_error(ctx, SVO_ERR_ARG, "svo_orb_detect: %s", why);
    const int nlev = g.nlev;
    size_t img_off[kMaxLevels], mask_off[kMaxLevels];
    size_t ibytes = 0, mbytes = 0;
    for (int l = 0; l < nlev; l++) {
        img_off[l] = ibytes;
        ibytes += (size_t)g.pitch[l] * g.lh[l] + 256;
        ibytes = (ibytes + 255) & ~(size_t)255;
        mask_off[l] = mbytes;
        mbytes += ((size_t)g.lw[l] * g.lh[l] + 255) & ~(size_t)255;
    }
    const int maxcap = g.maxcap, maxh = g.maxh, maxnseg = g.maxnseg;
    // workspace: level images (level 0 is the caller's image), masks, FAST
    // scratch, keypoints [nlev][maxcap], Harris responses, coefficient tables
    const size_t tab_words = g.tabs.size();
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
        lev.lv[l] = l == 0 ? L0 : ImgLevel{dimg + img_off[l], g.lw[l], g.lh[l], g.pitch[l]};
    // host staging: tables, per-level descriptors (lv[0] = that level)
    const size_t stage_bytes = sizeof(uint32_t) * tab_words + sizeof(PyrDesc) * kMaxLevels;
    char* hst = (char*)pinned(ctx, stage_bytes + 64);
    if (!hst) return set_error(ctx, SVO_ERR_HIP, "svo_orb_detect: pinned alloc failed");
    SVO_HIP(ctx, hipStreamSynchronize(st));  // the pinned buffer may still feed an earlier copy
    if (tab_words) std::memcpy(hst, g.tabs.data(), sizeof(uint32_t) * tab_words);
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
        const uint32_t* t = dtab + g.tab_at[l];
        SVO_HIP(ctx, launch_orb_resize(lev.lv[l - 1].data, lev.lv[l - 1].pitch, dmask ? dmask + mask_off[l - 1] : nullptr,
                                       g.lw[l - 1], const_cast<uint8_t*>(lev.lv[l].data), g.pitch[l],
                                       dmask ? dmask + mask_off[l] : nullptr, g.lw[l], g.lh[l], (const int*)t,
                                       t + g.lw[l], (const int*)(t + 2 * g.lw[l]), t + 2 * g.lw[l] + g.lh[l], st));
    }
    // FAST(fastThreshold, NMS) + the level mask, per level
    unsigned long long* bits = (unsigned long long*)(ws + o_bits);
    int* rowcnt = (int*)(ws + o_rc);
    int* rowoff = rowcnt + maxh + 64;
    const int thr = std::min(std::max(prm->fast_threshold, 0), 255);
    for (int l = 0; l < nlev; l++) {
        FastDetBatch b{ddesc + l, dmask ? dmask + mask_off[l] : nullptr, bits, rowcnt, rowoff,
                       dkp + (size_t)l * maxcap, dn + l, (size_t)g.lw[l] * g.lh[l], (g.lw[l] + 63) / 64, g.kcap[l]};
        SVO_HIP(ctx, launch_fast_detect(b, 1, g.lw[l], g.lh[l], thr, 1, st));
    }
    int hn[kMaxLevels] = {0};
    SVO_HIP(ctx, hipMemcpyAsync(hn, dn, sizeof(int) * nlev, hipMemcpyDeviceToHost, st));
    SVO_HIP(ctx, hipStreamSynchronize(st));
    int max_n = 0;
    for (int l = 0; l < nlev; l++) {
        if (hn[l] > g.kcap[l]) return set_error(ctx, SVO_ERR_CAPACITY, "svo_orb_detect: FAST overflow");
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
    const svo_keypoint* kp[kMaxLevels];
    const float* rp[kMaxLevels];
    for (int l = 0; l < nlev; l++) {
        kp[l] = &hk[(size_t)l * maxcap];
        rp[l] = harris ? &hr[(size_t)l * maxcap] : nullptr;
    }
    const int n = orb_select(g, *prm, kp, rp, hn, out, octave, cap);
    if (n_out) *n_out = n;
    return SVO_OK;
}
