// Grayscale pyramid build (pyrDown chain) for gfx950.
//
// Replaces the pyramid OpenCV builds inside every cv::calcOpticalFlowPyrLK call
// at R:src/tracking.cpp:101-105 and :160-165 (lkpyramid.cpp buildOpticalFlowPyramid
// -> pyramids.cpp pyrDown_): dst = ((w+1)/2, (h+1)/2), separable [1 4 6 4 1]^2,
// (sum + 128) >> 8, BORDER_REFLECT_101. Bit-exact (integer arithmetic).
//
// Unlike the reference, which rebuilds both pyramids on every LK call, a frame's
// pyramid is built once, kept in HBM and shared by the temporal and stereo LK
// calls. HBM roofline: reads w*h, writes w*h/4 bytes per level.
#include <algorithm>
#include <cstdlib>
#include <utility>

#include "common.hpp"
#include "xcd_tile.hpp"

namespace svo {

__device__ __forceinline__ int refl101(int p, int len) {
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        p = p < 0 ? -p : 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

// The REFLECT_101 border (kPyrPad pixels each side) of one level, written by the
// block that owns the border pixels' sources: every border pixel (px, py) is a
// copy of pixel (refl(px), refl(py)) of the level, and the blocks of a launch
// partition the level's pixels into owned rectangles [ox0, ox1) x [oy0, oy1), so
// each border pixel has exactly one writer, which already holds its value
// (val(sx, sy): a staged copy). Only blocks owning pixels within kPyrPad + 1 of
// an edge do any work.
//
// Border coordinates of one axis whose sources lie in [o0, o1): for a level
// longer than the border (one reflection) two runs, p = -s for s in [lo, lo + nlo)
// and p = 2 len - 2 - s for s in [hi, hi + nhi); a shorter level reflects
// several times and every one of the 2 kPyrPad border coordinates is tested.
struct BorderSpan {
    int lo, nlo, hi, nhi;
    bool many;
    __device__ int count() const { return many ? 2 * kPyrPad : nlo + nhi; }
    // k-th border coordinate (p) and its source (s); false: not sourced here (many)
    __device__ bool at(int k, int len, int o0, int o1, int& p, int& s) const {
        if (many) {
            p = k < kPyrPad ? k - kPyrPad : len + (k - kPyrPad);
            s = refl101(p, len);
            return s >= o0 && s < o1;
        }
        if (k < nlo) {
            s = lo + k;
            p = -s;
        } else {
            s = hi + (k - nlo);
            p = 2 * len - 2 - s;
        }
        return true;
    }
};
__device__ __forceinline__ BorderSpan border_span(int len, int o0, int o1) {
    BorderSpan b;
    b.many = len <= kPyrPad;
    b.lo = max(o0, 1);
    b.nlo = max(0, min(o1, kPyrPad + 1) - b.lo);
    b.hi = max(o0, len - 1 - kPyrPad);
    b.nhi = max(0, min(o1, len - 1) - b.hi);
    return b;
}

// rowp(sy): the staged copy of pixel (ox0, sy), 4-byte aligned (the top / bottom
// band rows go out as dwords), or nullptr (bytes through val). The side bands go
// out byte by byte: a dword form (aligned groups, four reflected sources each)
// measured slower (KITTI level 0: 48.7 vs 46.7 us).
template <class F, class G>
__device__ __forceinline__ void pad_owned(uint8_t* __restrict__ d, int w, int h, int pitch, int ox0, int ox1, int oy0,
                                          int oy1, F val, G rowp) {
    const int tid = threadIdx.x, nt = blockDim.x;
    const BorderSpan bx = border_span(w, ox0, ox1), by = border_span(h, oy0, oy1);
    const int ncx = bx.count(), ncy = by.count();
    // left / right bands of the owned rows
    if (ncx > 0) {
        const int n = (oy1 - oy0) * ncx;
        for (int k = tid; k < n; k += nt) {
            const int r = k / ncx, j = k - r * ncx;
            int px, sx;
            if (bx.at(j, w, ox0, ox1, px, sx)) d[(ptrdiff_t)(oy0 + r) * pitch + px] = val(sx, oy0 + r);
        }
    }
    if (ncy == 0) return;
    // top / bottom rows whose source rows are owned: the owned columns ...
    const int ow = ox1 - ox0, nq = (ow + 3) >> 2;
    for (int k = tid; k < ncy * nq; k += nt) {
        const int r = k / nq, q = k - r * nq;
        int py, sy;
        if (!by.at(r, h, oy0, oy1, py, sy)) continue;
        uint8_t* drow = d + (ptrdiff_t)py * pitch + ox0 + 4 * q;
        const uint8_t* srow = rowp(sy);
        if (srow && 4 * q + 4 <= ow) {
            *reinterpret_cast<uint32_t*>(drow) = *reinterpret_cast<const uint32_t*>(srow + 4 * q);
        } else {
            for (int m = 0; m < 4 && 4 * q + m < ow; m++) drow[m] = val(ox0 + 4 * q + m, sy);
        }
    }
    // ... and the border columns sourced here (corners)
    if (ncx > 0) {
        for (int k = tid; k < ncy * ncx; k += nt) {
            const int r = k / ncx, j = k - r * ncx;
            int py, sy, px, sx;
            if (!by.at(r, h, oy0, oy1, py, sy) || !bx.at(j, w, ox0, ox1, px, sx)) continue;
            d[(ptrdiff_t)py * pitch + px] = val(sx, sy);
        }
    }
}

constexpr int PD_TX = 64;   // output tile width
constexpr int PD_TY = 16;   // output tile height
constexpr int PD_IW = 2 * PD_TX + 4;  // 132 input columns
constexpr int PD_IH = 2 * PD_TY + 4;  // 36 input rows

// pad_src: also write the source level's border pixels whose sources this block
// owns (the level-l pixels [2x0, 2x0 + 128) x [2y0, 2y0 + 32) under its tile)
__device__ __forceinline__ void pyr_down_tile(const uint8_t* __restrict__ src, int sw, int sh,
                                              int sp, uint8_t* __restrict__ dst, int dw, int dh,
                                              int dp, bool pad_src = false) {
    __shared__ uint8_t T[PD_IH][PD_IW + 4];
    __shared__ int H[PD_IH][PD_TX + 1];
    const int x0 = blockIdx.x * PD_TX, y0 = blockIdx.y * PD_TY;
    const int sx0 = 2 * x0 - 2, sy0 = 2 * y0 - 2;
    const int tid = threadIdx.x;
    const bool interior = sx0 >= 0 && sy0 >= 0 && sx0 + PD_IW <= sw && sy0 + PD_IH <= sh;
    if (interior) {
        for (int k = tid; k < PD_IH * PD_IW; k += 256) {
            int r = k / PD_IW, c = k - r * PD_IW;
            T[r][c] = src[(size_t)(sy0 + r) * sp + (sx0 + c)];
        }
    } else {
        for (int k = tid; k < PD_IH * PD_IW; k += 256) {
            int r = k / PD_IW, c = k - r * PD_IW;
            T[r][c] = src[(size_t)refl101(sy0 + r, sh) * sp + refl101(sx0 + c, sw)];
        }
    }
    __syncthreads();
    for (int k = tid; k < PD_IH * PD_TX; k += 256) {
        int r = k >> 6, c = k & 63;
        const uint8_t* t = &T[r][2 * c];
        H[r][c] = t[0] + 4 * t[1] + 6 * t[2] + 4 * t[3] + t[4];
    }
    __syncthreads();
    // (after the last barrier: no wait for these stores)
    if (pad_src)
        pad_owned(const_cast<uint8_t*>(src), sw, sh, sp, 2 * x0, min(2 * x0 + 2 * PD_TX, sw), 2 * y0,
                  min(2 * y0 + 2 * PD_TY, sh), [&](int x, int y) { return T[y - sy0][x - sx0]; },
                  [](int) { return (const uint8_t*)nullptr; });  // (T's column 2x0 is not dword-aligned)
    const int c = tid & 63;
    const int x = x0 + c;
    if (x >= dw) return;
#pragma unroll
    for (int i = 0; i < PD_TY / 4; i++) {
        int r = (tid >> 6) * (PD_TY / 4) + i;
        int y = y0 + r;
        if (y < dh) {
            int s = H[2 * r][c] + 4 * H[2 * r + 1][c] + 6 * H[2 * r + 2][c] + 4 * H[2 * r + 3][c] +
                    H[2 * r + 4][c];
            dst[(size_t)y * dp + x] = (uint8_t)((s + 128) >> 8);
        }
    }
}

__global__ __launch_bounds__(256) void pyr_down_kernel(const uint8_t* __restrict__ src, int sw,
                                                       int sh, int sp, uint8_t* __restrict__ dst,
                                                       int dw, int dh, int dp) {
    pyr_down_tile(src, sw, sh, sp, dst, dw, dh, dp);
}

// Batched form: blockIdx.z = sequence, level l of descs[z] from level l-1
// (pad_src: and level l-1's border, pad_owned).
__global__ __launch_bounds__(256) void pyr_down_batched_kernel(const PyrDesc* __restrict__ descs,
                                                               int level, int pad_src) {
    const PyrDesc& P = descs[blockIdx.z];
    const ImgLevel& s = P.lv[level - 1];
    const ImgLevel& d = P.lv[level];
    if ((int)blockIdx.x * PD_TX >= d.w || (int)blockIdx.y * PD_TY >= d.h) return;
    // same body as pyr_down_kernel (inlined call keeps one copy of the math)
    pyr_down_tile(s.data, s.w, s.h, s.pitch, const_cast<uint8_t*>(d.data), d.w, d.h, d.pitch, pad_src != 0);
}

// REFLECT_101 border (kPyrPad pixels each side) of one level, written from the
// level's interior one aligned dword (4 pixels) per thread: the top and bottom
// bands over the full padded width, then the left and right bands of the
// interior rows (the right band starts at the dword holding column w, so it may
// rewrite a few interior pixels with their own values). One dword per thread
// (the grid covers level 0's dwords; smaller levels' surplus blocks exit), so
// the whole border costs one memory round trip.
__device__ __forceinline__ int refl_pad(int p, int len, bool single) {
    // levels larger than the padding reflect once (p in [-kPyrPad, len + kPyrPad))
    if (single) return p < 0 ? -p : (p >= len ? 2 * len - 2 - p : p);
    return refl101(p, len);
}
constexpr int PAD_SIDE = kPyrPad / 4 + 1;  // dwords per row and side (right side: alignment)
__host__ __device__ constexpr int pad_dwords(int w, int h) {
    return 2 * kPyrPad * ((w + 2 * kPyrPad + 3) / 4) + 2 * PAD_SIDE * h;
}
__device__ __forceinline__ void pad_level(const ImgLevel& L, int k) {
    const int w = L.w, h = L.h, dw = (w + 2 * kPyrPad + 3) / 4;
    const int n_tb = 2 * kPyrPad * dw;
    if (k >= n_tb + 2 * PAD_SIDE * h) return;
    uint8_t* __restrict__ d = const_cast<uint8_t*>(L.data);
    int x0, y;
    if (k < n_tb) {
        const int r = k / dw, c = k - r * dw;
        y = r < kPyrPad ? r - kPyrPad : h + (r - kPyrPad);
        x0 = 4 * c - kPyrPad;
    } else {
        const int k2 = k - n_tb, r = k2 / (2 * PAD_SIDE), c = k2 - r * (2 * PAD_SIDE);
        y = r;
        x0 = c < PAD_SIDE ? -kPyrPad + 4 * c : (w & ~3) + 4 * (c - PAD_SIDE);
        if (c < PAD_SIDE && x0 >= 0) return;  // left side: PAD_SIDE - 1 dwords suffice
    }
    const bool single = w > kPyrPad && h > kPyrPad;
    const uint8_t* srow = d + (ptrdiff_t)refl_pad(y, h, single) * L.pitch;
    unsigned v = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) v |= (unsigned)srow[refl_pad(x0 + i, w, single)] << (8 * i);
    *reinterpret_cast<unsigned*>(d + (ptrdiff_t)y * L.pitch + x0) = v;
}

__global__ __launch_bounds__(256) void pad_batched_kernel(const PyrDesc* __restrict__ descs) {
    pad_level(descs[blockIdx.z].lv[blockIdx.y], blockIdx.x * 256 + threadIdx.x);
}
__global__ __launch_bounds__(256) void pad_kernel(PyrDesc d) { pad_level(d.lv[blockIdx.y], blockIdx.x * 256 + threadIdx.x); }

hipError_t launch_pyramid_pad(const PyrDesc* d_descs, int nseq, int w, int h, int nlevels, hipStream_t st) {
    const int blocks = (pad_dwords(w, h) + 255) / 256;  // level 0 has the most
    hipLaunchKernelGGL(pad_batched_kernel, dim3(blocks, nlevels, nseq), dim3(256), 0, st, d_descs);
    return hipGetLastError();
}

// one launch per level + the border pass (nlevels beyond the fused chain's LDS)
static hipError_t pyramid_levels(const PyrDesc* d_descs, int nseq, int w, int h, int nlevels, hipStream_t st) {
    int lw = w, lh = h;
    for (int l = 1; l < nlevels; l++) {
        lw = (lw + 1) / 2;
        lh = (lh + 1) / 2;
        dim3 grid((lw + PD_TX - 1) / PD_TX, (lh + PD_TY - 1) / PD_TY, nseq);
        hipLaunchKernelGGL(pyr_down_batched_kernel, grid, dim3(256), 0, st, d_descs, l, 0);
    }
    return launch_pyramid_pad(d_descs, nseq, w, h, nlevels, st);
}

hipError_t launch_pyramid(const svo_image* img, int first_level, hipStream_t st) {
    for (int l = first_level < 1 ? 1 : first_level; l < img->nlevels; l++) {
        const ImgLevel& s = img->desc.lv[l - 1];
        const ImgLevel& d = img->desc.lv[l];
        dim3 grid((d.w + PD_TX - 1) / PD_TX, (d.h + PD_TY - 1) / PD_TY);
        hipLaunchKernelGGL(pyr_down_kernel, grid, dim3(256), 0, st, s.data, s.w, s.h, s.pitch,
                           const_cast<uint8_t*>(d.data), d.w, d.h, d.pitch);
    }
    hipLaunchKernelGGL(pad_kernel, dim3((pad_dwords(img->w, img->h) + 255) / 256, img->nlevels), dim3(256), 0, st,
                       img->desc);
    return hipGetLastError();
}

}  // namespace svo

// ---------------------------------------------------------------------------
// Fused pyrDown + Scharr: one pass over level l writes level l+1 of the image
// pyramid and level l of the derivative pyramid (scharr.hip's packed layout).
// A block owns a 64x16 tile of level l+1, i.e. the 128x32 pixels of level l
// under it; the staged 136x36 level-l tile (dword loads; REFLECT_101 at the
// borders, which both operators use) feeds both outputs, so level l is read
// once instead of twice. Bit-exact integer arithmetic as the separate kernels.
namespace svo {

namespace {

constexpr int FS_IW = 2 * PD_TX + 8;  // 136 staged columns: sx0 - 2 .. sx0 + 133 (dword aligned)
constexpr int FS_IH = PD_IH;          // 36 rows

// Scharr of a 4 x 4 pixel block, packed: a row's 6 columns k = 0 .. 5 (the block's
// columns -1 .. 4: byte 3 of dword a0, the 4 bytes of a1, byte 0 of a2) as the
// 16-bit column pairs (k0, k2), (k2, k4), (k1, k3), (k3, k5). Output columns
// m = 0, 2 and m = 1, 3 are then one packed lane each, and the 16-bit wrap-around
// arithmetic leaves the stored low 16 bits of ix 2^kDerShift, iy 2^kDerShift
// unchanged (|values| <= 16320).
typedef short s16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void scharr_pairs(unsigned a0, unsigned a1, unsigned a2, s16x2 (&pr)[4]) {
    pr[0] = __builtin_bit_cast(s16x2, __builtin_amdgcn_perm(a1, a0, 0x0c050c03u));  // a0.b3, a1.b1
    pr[1] = __builtin_bit_cast(s16x2, (a1 >> 8) & 0x00FF00FFu);                     // a1.b1, a1.b3
    pr[2] = __builtin_bit_cast(s16x2, a1 & 0x00FF00FFu);                            // a1.b0, a1.b2
    pr[3] = __builtin_bit_cast(s16x2, __builtin_amdgcn_perm(a2, a1, 0x0c040c02u));  // a1.b2, a2.b0
}

// one output row of the block from its top / middle / bottom rows' pairs:
// o[m] = (iy(m) << 16) | (ix(m) & 0xFFFF), both x 2^kDerShift
__device__ __forceinline__ void scharr_row(const s16x2 (&t)[4], const s16x2 (&mi)[4], const s16x2 (&b)[4],
                                           unsigned (&o)[4]) {
    constexpr short C3 = 3 << kDerShift, C10 = 10 << kDerShift;
    // vertical smoothing vs = 3 t + 10 m + 3 b and difference d = b - t per pair
    s16x2 vs[4], dd[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        vs[k] = (t[k] + b[k]) * C3 + mi[k] * C10;
        dd[k] = b[k] - t[k];
    }
    // ix(m) = vs(m + 2) - vs(m); iy(m) = 3 d(m) + 10 d(m + 1) + 3 d(m + 2)
    const unsigned ue = __builtin_bit_cast(unsigned, (s16x2)(vs[1] - vs[0]));
    const unsigned uo = __builtin_bit_cast(unsigned, (s16x2)(vs[3] - vs[2]));
    const unsigned ve = __builtin_bit_cast(unsigned, (s16x2)((dd[0] + dd[1]) * C3 + dd[2] * C10));
    const unsigned vo = __builtin_bit_cast(unsigned, (s16x2)((dd[2] + dd[3]) * C3 + dd[1] * C10));
    o[0] = __builtin_amdgcn_perm(ve, ue, 0x05040100u);
    o[1] = __builtin_amdgcn_perm(vo, uo, 0x05040100u);
    o[2] = __builtin_amdgcn_perm(ve, ue, 0x07060302u);
    o[3] = __builtin_amdgcn_perm(vo, uo, 0x07060302u);
}

// NT: the derivative and level stores as non-temporal (streaming) stores; SCH:
// false = pyrDown (+ the source level's border) only, the right frames' pyramid
// (the dword staging and packed row pass of this kernel, against the byte loads
// of pyr_down_batched_kernel)
// XT: tiles in XCD order (xcd_tile.hpp)
template <bool NT, bool SCH = true, bool XT = false>
__global__ __launch_bounds__(256) void pyr_scharr_kernel(const PyrDesc* __restrict__ descs,
                                                         const DerivDesc* __restrict__ ders, int level, int pad_src) {
    const XcdTile tile = XT ? xcd_tile() : XcdTile{(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z};
    const PyrDesc& P = descs[tile.z];
    const ImgLevel& s = P.lv[level];
    const ImgLevel& d = P.lv[level + 1];
    const int x0 = tile.x * PD_TX, y0 = tile.y * PD_TY;
    const int sx0 = 2 * x0 - 2, sy0 = 2 * y0 - 2;
    const int xa = sx0 - 2;  // multiple of 4 (x0 is a multiple of 64)
    __shared__ __attribute__((aligned(16))) uint8_t T[FS_IH][FS_IW + 8];  // rows 16-byte aligned (b128 reads)
    __shared__ int H[PD_IH][PD_TX + 1];
    const int tid = threadIdx.x;
    const int sw = s.w, sh = s.h;
    const bool interior = xa >= 0 && sy0 >= 0 && xa + FS_IW <= sw && sy0 + FS_IH <= sh;
    if (interior) {
        // thread -> (row r0, dword c4), rows r0 + RP p: all loads in flight before the
        // first LDS store
        constexpr int DW = FS_IW / 4, RP = 256 / DW, NP = (FS_IH + RP - 1) / RP;  // 34 dwords per row
        const int r0 = tid / DW, c4 = tid - r0 * DW;
        if (r0 < RP) {
            const uint8_t* src = s.data + (size_t)(sy0 + r0) * s.pitch + xa + 4 * c4;
            uint32_t v[NP];
#pragma unroll
            for (int p = 0; p < NP; p++)
                v[p] = *(const __attribute__((address_space(1))) uint32_t*)(src + (size_t)(min(r0 + p * RP, FS_IH - 1) - r0) *
                                                                                   s.pitch);
            // (rows past the tile load and store its last row again, the same bytes:
            // no branch, so no wait between the loads)
#pragma unroll
            for (int p = 0; p < NP; p++) *reinterpret_cast<uint32_t*>(&T[min(r0 + p * RP, FS_IH - 1)][4 * c4]) = v[p];
        }
    } else {
        // a border tile: a staged row is a whole source row (REFLECT_101 maps rows to
        // rows), so every dword inside the columns [0, sw) is still one load; only
        // the dwords crossing or beyond a side edge take bytes with the column
        // reflection
        constexpr int DW = FS_IW / 4;
        for (int k = tid; k < FS_IH * DW; k += 256) {
            const int r = k / DW, c4 = k - r * DW;
            const uint8_t* row = s.data + (size_t)refl101(sy0 + r, sh) * s.pitch;
            const int xc = xa + 4 * c4;
            uint32_t v;
            if (xc >= 0 && xc + 3 < sw) {
                v = *reinterpret_cast<const uint32_t*>(row + xc);
            } else {
                v = 0;
#pragma unroll
                for (int b = 0; b < 4; b++) v |= (uint32_t)row[refl101(xc + b, sw)] << (8 * b);
            }
            *reinterpret_cast<uint32_t*>(&T[r][4 * c4]) = v;
        }
    }
    __syncthreads();
    // ---- pyrDown rows: T column 2 + j holds level-l column sx0 + j; a task
    // makes 4 outputs (c = 4q .. 4q + 3) from 4 aligned dwords of its row ----
    for (int k = tid; k < PD_IH * (PD_TX / 4); k += 256) {
        const int r = k >> 4, q = k & 15;
        const uint4 v = *reinterpret_cast<const uint4*>(&T[r][8 * q]);
        const unsigned w4[4] = {v.x, v.y, v.z, v.w};
        // byte pairs P(i) = (b_i, b_i+4) as 16-bit lanes: outputs m = 0, 2 and m = 1, 3
        // are one packed lane each (sums <= 16 * 255, no carry between the halves)
        typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
        u16x2 P[7];  // P[i - 2], i = 2 .. 8
#pragma unroll
        for (int i = 2; i <= 8; i++)
            P[i - 2] = __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(w4[(i >> 2) + 1], w4[i >> 2],
                                                                       0x0c000c00u | (i & 3) | ((4u + (i & 3)) << 16)));
        const unsigned e = __builtin_bit_cast(unsigned, (u16x2)(P[0] + P[4] + (P[1] + P[3]) * (unsigned short)4 +
                                                                P[2] * (unsigned short)6));
        const unsigned o = __builtin_bit_cast(unsigned, (u16x2)(P[2] + P[6] + (P[3] + P[5]) * (unsigned short)4 +
                                                                P[4] * (unsigned short)6));
        H[r][4 * q + 0] = (int)(e & 0xFFFFu);
        H[r][4 * q + 1] = (int)(o & 0xFFFFu);
        H[r][4 * q + 2] = (int)(e >> 16);
        H[r][4 * q + 3] = (int)(o >> 16);
    }
    // ---- Scharr of level l pixels (2x0 + i, 2y0 + j), i < 128, j < 32: T[2 + j][4 + i];
    // a task: 4 columns x 4 rows from 3 aligned dwords per staged row, one 16-byte
    // store per row (columns >= sw are never written: the zero border stays) ----
    if constexpr (SCH) {
        uint32_t* __restrict__ out = ders[tile.z].data[level];
        const int op = ders[tile.z].pitch[level];
        const int g = tid & 31, q = tid >> 5;
        const int x = 2 * x0 + 4 * g;
        // staged rows 1 + 4q .. 6 + 4q, T columns 3 + 4g .. 8 + 4g
        s16x2 pr[6][4];
#pragma unroll
        for (int rr = 0; rr < 6; rr++) {
            const uint8_t* trow = &T[1 + 4 * q + rr][0];
            scharr_pairs(*reinterpret_cast<const unsigned*>(trow + 4 * g),
                         *reinterpret_cast<const unsigned*>(trow + 4 * g + 4),
                         *reinterpret_cast<const unsigned*>(trow + 4 * g + 8), pr[rr]);
        }
        if (x < sw) {
#pragma unroll
            for (int jj = 0; jj < 4; jj++) {
                const int y = 2 * y0 + 4 * q + jj;
                if (y >= sh) break;
                unsigned o[4];
                scharr_row(pr[jj], pr[jj + 1], pr[jj + 2], o);
                // global (not flat) stores: no LDS counter traffic behind them
                __attribute__((address_space(1))) uint32_t* dst =
                    (__attribute__((address_space(1))) uint32_t*)(out + (size_t)y * op + x);
                if (x + 3 < sw) {
                    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
                    const u32x4 v = {o[0], o[1], o[2], o[3]};
                    if constexpr (NT)
                        __builtin_nontemporal_store(v, (__attribute__((address_space(1))) u32x4*)dst);
                    else
                        *(__attribute__((address_space(1))) u32x4*)dst = v;
                } else {
#pragma unroll
                    for (int m = 0; m < 4; m++)
                        if (x + m < sw) dst[m] = o[m];
                }
            }
        }
    }
    __syncthreads();
    // level l's border pixels whose sources lie under this tile (after the last
    // barrier: no wait for these stores)
    if (pad_src)
        pad_owned(const_cast<uint8_t*>(s.data), sw, sh, s.pitch, 2 * x0, min(2 * x0 + 2 * PD_TX, sw), 2 * y0,
                  min(2 * y0 + 2 * PD_TY, sh), [&](int x, int y) { return T[y - sy0][x - xa]; },
                  [&](int y) { return (const uint8_t*)&T[y - sy0][2 * x0 - xa]; });
    // ---- pyrDown columns: 4 output rows per thread from 11 sliding H rows ----
    const int c = tid & 63;
    const int x = x0 + c;
    if (x >= d.w) return;
    __attribute__((address_space(1))) uint8_t* dst = (__attribute__((address_space(1))) uint8_t*)d.data;
    const int r0 = (tid >> 6) * (PD_TY / 4);
    int hv[2 * (PD_TY / 4) + 3];
#pragma unroll
    for (int i = 0; i < 2 * (PD_TY / 4) + 3; i++) hv[i] = H[2 * r0 + i][c];
#pragma unroll
    for (int i = 0; i < PD_TY / 4; i++) {
        const int y = y0 + r0 + i;
        if (y < d.h) {
            const int sum = hv[2 * i] + 4 * hv[2 * i + 1] + 6 * hv[2 * i + 2] + 4 * hv[2 * i + 3] + hv[2 * i + 4];
            dst[(size_t)y * d.pitch + x] = (uint8_t)((sum + 128) >> 8);
        }
    }
}

}  // namespace

static hipError_t pyramid_scharr_levels(const PyrDesc* d_descs, const DerivDesc* d_ders, int nseq, int w, int h,
                                        int nlevels, hipStream_t st) {
    int lw = w, lh = h;
    for (int l = 0; l + 1 < nlevels; l++) {
        const int nw = (lw + 1) / 2, nh = (lh + 1) / 2;
        dim3 grid((nw + PD_TX - 1) / PD_TX, (nh + PD_TY - 1) / PD_TY, nseq);
        // non-temporal derivative stores: the chain alone 97.6 -> 89.5 us per 64
        // frames against plain stores, the step unchanged (LK reads them a step later)
        hipLaunchKernelGGL(pyr_scharr_kernel<true>, grid, dim3(256), 0, st, d_descs, d_ders, l, 0);
        lw = nw;
        lh = nh;
    }
    // the coarsest level's derivative (no pyrDown after it), then the borders
    hipError_t e = launch_scharr_level(d_descs, d_ders, nseq, lw, lh, nlevels - 1, st);
    if (e != hipSuccess) return e;
    return launch_pyramid_pad(d_descs, nseq, w, h, nlevels, st);
}

// ---------------------------------------------------------------------------
// Fused chain: levels 2 .. c of a pyramid (c = nlevels - 1) from level 1, the
// Scharr derivatives of levels 1 .. c (SCHARR) and the borders of levels 1 .. c,
// in ONE launch (one block per tile of the coarsest level, per sequence). The
// per-level launches it replaces were latency-bound from level 1 on (level 1->2
// 17 us, 2->3 13, Scharr of 3 5, borders 14 for 64 KITTI frames,
// profiles/r02_pyramid_chain.txt) and each one queued behind whatever ran beside
// it. A block owns the rectangle under its level-c tile at every level (level l:
// the tile scaled by 2^(c-l), clipped to the level) and computes, in LDS, the
// region R_l = owned +- halo_l of every level: halo_c = 1 (the 3x3 Scharr; 0
// without it), halo_l = 2 halo_(l+1) + 2 (the 5-tap pyrDown of R_(l+1)), level 1
// staged from HBM. Entries of R_l outside the level hold the REFLECT_101 pixel
// (the border rule of both pyrDown and Scharr), so every tap is a plain LDS read.
// Each block writes its owned pixels, their derivatives and the border pixels
// whose sources it owns (pad_owned): no two blocks write the same byte, and no
// block reads another's output. Bit-exact integer arithmetic as the per-level
// kernels (same taps, same rounding).
// Compile-time shape of the chain of levels S .. C (level S staged from HBM): the
// level-C tile TW x TH (its level-S footprint is 128 x 32), per level l the
// owned tile OW x OH, the halos (y: hy_C = 1 for the 3x3 Scharr, hy_l = 2 hy_(l+1)
// + 2 for the 5-tap pyrDown; x: the same rounded up to 4 so that every region
// row keeps the owned columns dword-aligned), region RW x RH at pitch PW, LDS
// offsets (all levels stay resident: the store phase reads them all).
template <int C, bool SCHARR, int S>
struct ChainShape {
    static constexpr int TW = 128 >> (C - S), TH = 32 >> (C - S);
    static constexpr int hy(int l) { return l >= C ? (SCHARR ? 1 : 0) : 2 * hy(l + 1) + 2; }
    static constexpr int hx(int l) { return l >= C ? (SCHARR ? 4 : 0) : (2 * hx(l + 1) + 2 + 3) & ~3; }
    static constexpr int OW(int l) { return TW << (C - l); }
    static constexpr int OH(int l) { return TH << (C - l); }
    static constexpr int RW(int l) { return OW(l) + 2 * hx(l); }
    static constexpr int RH(int l) { return OH(l) + 2 * hy(l); }
    static constexpr int PW(int l) { return (RW(l) + 15) & ~15; }
    static constexpr int off(int l) { return l <= S ? 0 : off(l - 1) + PW(l - 1) * RH(l - 1); }
    static constexpr int hrows(int l) { return 2 * RH(l) + 3; }  // rows pass of level l
    static constexpr int hbytes() {
        int b = 0;
        for (int l = S + 1; l <= C; l++) b = b > hrows(l) * RW(l) * 2 ? b : hrows(l) * RW(l) * 2;
        return b;
    }
    static constexpr int off_h() { return (off(C + 1) + 15) & ~15; }
    static constexpr int lds() { return off_h() + hbytes(); }
};

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as_u16x2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ uint32_t as_u32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }
// bytes X (low half) and Y (high half) of the 8 bytes {lo, hi} as a u16 pair
__device__ __forceinline__ u16x2 byte_pair(uint32_t hi, uint32_t lo, int X, int Y) {
    return as_u16x2(__builtin_amdgcn_perm(hi, lo, 0x0C000C00u | ((unsigned)Y << 16) | (unsigned)X));
}

// Level l of the chain's phase 1 (LDS only): level 1 staged from HBM (rows
// reflected by index, columns dword-wise where the dword lies inside the level,
// byte-wise reflected otherwise); level l >= 2 by pyrDown of level l-1's region,
// then its entries outside the level set to the reflected pixel.
template <int C, bool SCHARR, int S, int l>
__device__ __forceinline__ void chain_build(const PyrDesc& P, uint8_t* lds, uint16_t* H) {
    using Sh = ChainShape<C, SCHARR, S>;
    constexpr int RW = Sh::RW(l), RH = Sh::RH(l), PW = Sh::PW(l);
    const int tid = threadIdx.x;
    const ImgLevel& L = P.lv[l];
    const int w = L.w, h = L.h;
    const XcdTile tile = xcd_tile();  // (the chain's tiles in XCD order, as pyr_scharr_kernel's)
    const int gx = tile.x * Sh::OW(l) - Sh::hx(l), gy = tile.y * Sh::OH(l) - Sh::hy(l);
    uint8_t* __restrict__ R = lds + Sh::off(l);
    if constexpr (l == S) {
        constexpr int DW = RW / 4;
        for (int k = tid; k < RH * DW; k += 256) {
            const int r = k / DW, q = k - r * DW;
            const uint8_t* src = L.data + (size_t)refl101(gy + r, h) * L.pitch;
            const int x = gx + 4 * q;
            uint32_t v;
            if (x >= 0 && x + 4 <= w) {
                v = *reinterpret_cast<const uint32_t*>(src + x);
            } else {
                v = 0;
#pragma unroll
                for (int m = 0; m < 4; m++) v |= (uint32_t)src[refl101(x + m, w)] << (8 * m);
            }
            *reinterpret_cast<uint32_t*>(R + r * PW + 4 * q) = v;
        }
        __syncthreads();
    } else {
        constexpr int PWp = Sh::PW(l - 1);
        const uint8_t* __restrict__ pR = lds + Sh::off(l - 1);
        constexpr int NQ = RW / 4, NR = Sh::hrows(l);
        // rows pass: H[r][j] = 1 4 6 4 1 over region row r of level l-1, columns
        // 2j + 2 .. 2j + 6 (where the halos put level-l column j's taps); 4 outputs
        // per task from 16 region bytes, as two packed u16 pairs
        for (int k = tid; k < NR * NQ; k += 256) {
            const int r = k / NQ, q = k - r * NQ;
            const uint4 v = *reinterpret_cast<const uint4*>(pR + r * PWp + 8 * q);
            // outputs 0 / 1 read bytes 2+t / 4+t, outputs 2 / 3 bytes 6+t / 8+t (tap t)
            const u16x2 a0 = byte_pair(v.y, v.x, 2, 4), a1 = byte_pair(v.y, v.x, 3, 5),
                        a2 = byte_pair(v.y, v.x, 4, 6), a3 = byte_pair(v.y, v.x, 5, 7),
                        a4 = byte_pair(v.z, v.y, 2, 4);
            const u16x2 b0 = byte_pair(v.z, v.y, 2, 4), b1 = byte_pair(v.z, v.y, 3, 5),
                        b2 = byte_pair(v.z, v.y, 4, 6), b3 = byte_pair(v.z, v.y, 5, 7),
                        b4 = byte_pair(v.w, v.z, 2, 4);
            const u16x2 ha = (a0 + a4) + (u16x2)4 * (a1 + a3) + (u16x2)6 * a2;
            const u16x2 hb = (b0 + b4) + (u16x2)4 * (b1 + b3) + (u16x2)6 * b2;
            *reinterpret_cast<uint2*>(H + r * RW + 4 * q) = make_uint2(as_u32(ha), as_u32(hb));
        }
        __syncthreads();
        // columns pass: R[i][j] = (1 4 6 4 1 over H rows 2i .. 2i + 4, + 128) >> 8 in
        // packed u16 (sums <= 65280 + 128), 4 columns per task
        for (int k = tid; k < RH * NQ; k += 256) {
            const int i = k / NQ, q = k - i * NQ;
            const uint16_t* t = H + 2 * i * RW + 4 * q;
            const uint2 r0 = *reinterpret_cast<const uint2*>(t), r1 = *reinterpret_cast<const uint2*>(t + RW),
                        r2 = *reinterpret_cast<const uint2*>(t + 2 * RW),
                        r3 = *reinterpret_cast<const uint2*>(t + 3 * RW),
                        r4 = *reinterpret_cast<const uint2*>(t + 4 * RW);
            const u16x2 sa = (as_u16x2(r0.x) + as_u16x2(r4.x)) + (u16x2)4 * (as_u16x2(r1.x) + as_u16x2(r3.x)) +
                             (u16x2)6 * as_u16x2(r2.x) + (u16x2)128;
            const u16x2 sb = (as_u16x2(r0.y) + as_u16x2(r4.y)) + (u16x2)4 * (as_u16x2(r1.y) + as_u16x2(r3.y)) +
                             (u16x2)6 * as_u16x2(r2.y) + (u16x2)128;
            // the high bytes of the four sums are (s + 128) >> 8
            *reinterpret_cast<uint32_t*>(R + i * PW + 4 * q) = __builtin_amdgcn_perm(as_u32(sb), as_u32(sa), 0x07050301u);
        }
        __syncthreads();
        // entries outside the level: the reflected pixel -- columns first, then the
        // rows, which copy whole region rows including their fixed columns
        const int nxl = max(0, min(-gx, RW)), nxr = max(0, min(gx + RW - w, RW - nxl));
        if (nxl + nxr > 0) {  // columns [0, nxl) and [RW - nxr, RW) of the region
            const int nc = nxl + nxr;
            for (int k = tid; k < RH * nc; k += 256) {
                const int r = k / nc, j = k - r * nc;
                const int c = j < nxl ? j : RW - nxr + (j - nxl);
                R[r * PW + c] = R[r * PW + (refl101(gx + c, w) - gx)];
            }
            __syncthreads();
        }
        const int nyt = max(0, min(-gy, RH)), nyb = max(0, min(gy + RH - h, RH - nyt));
        if (nyt + nyb > 0) {  // rows [0, nyt) and [RH - nyb, RH)
            constexpr int DW = PW / 4;
            const int n = (nyt + nyb) * DW;
            for (int k = tid; k < n; k += 256) {
                const int j = k / DW, q = k - j * DW;
                const int r = j < nyt ? j : RH - nyb + (j - nyt);
                *reinterpret_cast<uint32_t*>(R + r * PW + 4 * q) =
                    *reinterpret_cast<const uint32_t*>(R + (refl101(gy + r, h) - gy) * PW + 4 * q);
            }
            __syncthreads();
        }
    }
}

// Level l of the chain's phase 2 (stores only): the owned tile's derivatives
// (pyr_scharr_kernel's arithmetic, a task = 4 columns x 4 rows from 3 aligned
// dwords of each of 6 region rows), its pixels (l >= 2; level 1 is written by the
// level-0 launch) and the border pixels whose sources it owns.
template <int C, bool SCHARR, int S, int l>
__device__ __forceinline__ void chain_store(const PyrDesc& P, const DerivDesc* ders, const uint8_t* lds) {
    using Sh = ChainShape<C, SCHARR, S>;
    constexpr int PW = Sh::PW(l), HX = Sh::hx(l), HY = Sh::hy(l), OWl = Sh::OW(l), OHl = Sh::OH(l);
    const int tid = threadIdx.x;
    const ImgLevel& L = P.lv[l];
    const int w = L.w, h = L.h;
    const XcdTile tile = xcd_tile();
    const int ox0 = tile.x * OWl, oy0 = tile.y * OHl;
    const int ox1 = min(ox0 + OWl, w), oy1 = min(oy0 + OHl, h);
    const uint8_t* __restrict__ R = lds + Sh::off(l);
    if constexpr (SCHARR) {
        uint32_t* __restrict__ out = ders[tile.z].data[l];
        const int op = ders[tile.z].pitch[l];
        constexpr int NG = OWl / 4, NT = NG * (OHl / 4);
        for (int k = tid; k < NT; k += 256) {
            const int qq = k / NG, g = k - qq * NG;
            const int x = ox0 + 4 * g;
            if (x >= w || oy0 + 4 * qq >= h) continue;
            s16x2 pr[6][4];
#pragma unroll
            for (int rr = 0; rr < 6; rr++) {
                const uint8_t* trow = R + (HY + 4 * qq - 1 + rr) * PW + HX + 4 * g - 4;
                scharr_pairs(*reinterpret_cast<const unsigned*>(trow), *reinterpret_cast<const unsigned*>(trow + 4),
                             *reinterpret_cast<const unsigned*>(trow + 8), pr[rr]);
            }
#pragma unroll
            for (int jj = 0; jj < 4; jj++) {
                const int y = oy0 + 4 * qq + jj;
                if (y >= h) break;
                unsigned o[4];
                scharr_row(pr[jj], pr[jj + 1], pr[jj + 2], o);
                __attribute__((address_space(1))) uint32_t* d =
                    (__attribute__((address_space(1))) uint32_t*)(out + (size_t)y * op + x);
                if (x + 3 < w) {
                    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
                    *(__attribute__((address_space(1))) u32x4*)d = u32x4{o[0], o[1], o[2], o[3]};
                } else {
#pragma unroll
                    for (int m = 0; m < 4; m++)
                        if (x + m < w) d[m] = o[m];
                }
            }
        }
    }
    uint8_t* __restrict__ dst = const_cast<uint8_t*>(L.data);
    if constexpr (l > S) {
        constexpr int NQ = OWl / 4;
        for (int k = tid; k < NQ * OHl; k += 256) {
            const int i = k / NQ, q = k - i * NQ;
            const int x = ox0 + 4 * q, y = oy0 + i;
            if (x >= w || y >= h) continue;
            const uint32_t v = *reinterpret_cast<const uint32_t*>(R + (HY + i) * PW + HX + 4 * q);
            uint8_t* d = dst + (size_t)y * L.pitch + x;
            if (x + 3 < w) {
                *reinterpret_cast<uint32_t*>(d) = v;
            } else {
#pragma unroll
                for (int m = 0; m < 4; m++)
                    if (x + m < w) d[m] = (uint8_t)(v >> (8 * m));
            }
        }
    }
    const int gx = ox0 - HX, gy = oy0 - HY;
    pad_owned(dst, w, h, L.pitch, ox0, ox1, oy0, oy1, [&](int x, int y) { return R[(y - gy) * PW + (x - gx)]; },
              [&](int y) { return R + (y - gy) * PW + HX; });
}

template <int C, bool SCHARR, int S, int... I>
__device__ __forceinline__ void chain_all(const PyrDesc& P, const DerivDesc* ders, uint8_t* lds, uint16_t* H,
                                          std::integer_sequence<int, I...>) {
    (chain_build<C, SCHARR, S, I + S>(P, lds, H), ...);
    (chain_store<C, SCHARR, S, I + S>(P, ders, lds), ...);
}

template <int C, bool SCHARR, int S>
__global__ __launch_bounds__(256) void pyr_chain_kernel(const PyrDesc* __restrict__ descs,
                                                        const DerivDesc* __restrict__ ders) {
    using Sh = ChainShape<C, SCHARR, S>;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    chain_all<C, SCHARR, S>(descs[xcd_tile().z], ders, lds, reinterpret_cast<uint16_t*>(lds + Sh::off_h()),
                            std::make_integer_sequence<int, C - S + 1>{});
}

template <int C, bool SCHARR, int S>
static void launch_chain(const PyrDesc* d_descs, const DerivDesc* d_ders, int nseq, int w, int h, hipStream_t st) {
    using Sh = ChainShape<C, SCHARR, S>;
    static_assert(Sh::lds() <= 65536, "chain LDS");
    int wc = w, hc = h;
    for (int l = 0; l < C; l++) {
        wc = (wc + 1) / 2;
        hc = (hc + 1) / 2;
    }
    const dim3 grid((wc + Sh::TW - 1) / Sh::TW, (hc + Sh::TH - 1) / Sh::TH, nseq);
    hipLaunchKernelGGL((pyr_chain_kernel<C, SCHARR, S>), grid, dim3(256), Sh::lds(), st, d_descs, d_ders);
}

// The chain's first level: the last two levels of the pyramid (one level for a
// two-level pyramid). Measured at the KITTI batch (64 frames), the chain of
// levels 1 .. 3 in one launch ran 47 us: its regions' halos (level 1 staged
// 184 x 52 for a 128 x 32 tile) cost more VALU than the launches they save, so
// the larger levels keep the per-level pyr_scharr / pyr_down launches (with their
// sources' borders fused in) and only the small levels are chained.
constexpr int chain_start(int c) { return c > 1 ? c - 1 : 1; }

template <bool SCHARR>
static void launch_chain_c(int c, const PyrDesc* d_descs, const DerivDesc* d_ders, int nseq, int w, int h,
                           hipStream_t st) {
    switch (c) {
        case 1: launch_chain<1, SCHARR, chain_start(1)>(d_descs, d_ders, nseq, w, h, st); break;
        case 2: launch_chain<2, SCHARR, chain_start(2)>(d_descs, d_ders, nseq, w, h, st); break;
        case 3: launch_chain<3, SCHARR, chain_start(3)>(d_descs, d_ders, nseq, w, h, st); break;
        case 4: launch_chain<4, SCHARR, chain_start(4)>(d_descs, d_ders, nseq, w, h, st); break;
        case 5: launch_chain<5, SCHARR, chain_start(5)>(d_descs, d_ders, nseq, w, h, st); break;
        case 6: launch_chain<6, SCHARR, chain_start(6)>(d_descs, d_ders, nseq, w, h, st); break;
        case 7: launch_chain<7, SCHARR, chain_start(7)>(d_descs, d_ders, nseq, w, h, st); break;
    }
}

// SVO_PYR_FUSED=0: the per-level launches (A/B; read at every launch, so a test
// can run both forms in one process)
static bool fused_on() {
    const char* e = std::getenv("SVO_PYR_FUSED");
    return !(e && e[0] == '0');
}

// pyramid (levels 1 ..) + borders of nseq frames: level 0 -> 1 with level 0's
// border, then the fused chain (levels 2 .. and the borders of levels 1 ..)
hipError_t launch_pyramid_batched(const PyrDesc* d_descs, int nseq, int w, int h, int nlevels, hipStream_t st) {
    const int c = nlevels - 1;
    if (!fused_on() || c < 1 || c >= kMaxLevels) return pyramid_levels(d_descs, nseq, w, h, nlevels, st);
    // levels 1 .. chain_start(c) one launch each, every launch also writing its
    // source level's border; then the chain
    int lw = w, lh = h;
    for (int l = 1; l <= chain_start(c); l++) {
        lw = (lw + 1) / 2;
        lh = (lh + 1) / 2;
        const dim3 grid((lw + PD_TX - 1) / PD_TX, (lh + PD_TY - 1) / PD_TY, nseq);
        if (xcd_tiles_on())
            hipLaunchKernelGGL((pyr_scharr_kernel<true, false, true>), grid, dim3(256), 0, st, d_descs,
                               (const DerivDesc*)nullptr, l - 1, 1);
        else
            hipLaunchKernelGGL((pyr_scharr_kernel<true, false>), grid, dim3(256), 0, st, d_descs,
                               (const DerivDesc*)nullptr, l - 1, 1);
    }
    launch_chain_c<false>(c, d_descs, nullptr, nseq, w, h, st);
    return hipGetLastError();
}

// pyramid (levels 1 ..), derivative levels 0 .. and borders of nseq frames: level
// 0 -> 1 with level 0's derivative and border, then the fused chain
hipError_t launch_pyramid_scharr_batched(const PyrDesc* d_descs, const DerivDesc* d_ders, int nseq, int w, int h,
                                         int nlevels, hipStream_t st) {
    const int c = nlevels - 1;
    if (!fused_on() || c < 1 || c >= kMaxLevels)
        return pyramid_scharr_levels(d_descs, d_ders, nseq, w, h, nlevels, st);
    // level l -> l + 1 + level l's derivative and border, l < chain_start(c); then the chain
    int lw = w, lh = h;
    for (int l = 0; l < chain_start(c); l++) {
        lw = (lw + 1) / 2;
        lh = (lh + 1) / 2;
        const dim3 grid((lw + PD_TX - 1) / PD_TX, (lh + PD_TY - 1) / PD_TY, nseq);
        if (xcd_tiles_on())
            hipLaunchKernelGGL((pyr_scharr_kernel<true, true, true>), grid, dim3(256), 0, st, d_descs, d_ders, l, 1);
        else
            hipLaunchKernelGGL(pyr_scharr_kernel<true>, grid, dim3(256), 0, st, d_descs, d_ders, l, 1);
    }
    launch_chain_c<true>(c, d_descs, d_ders, nseq, w, h, st);
    return hipGetLastError();
}

}  // namespace svo
