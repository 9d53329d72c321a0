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
#include <cstdlib>

#include "common.hpp"

namespace svo {

__device__ __forceinline__ int refl101(int p, int len) {
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        p = p < 0 ? -p : 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

constexpr int PD_TX = 64;   // output tile width
constexpr int PD_TY = 16;   // output tile height
constexpr int PD_IW = 2 * PD_TX + 4;  // 132 input columns
constexpr int PD_IH = 2 * PD_TY + 4;  // 36 input rows

__device__ __forceinline__ void pyr_down_tile(const uint8_t* __restrict__ src, int sw, int sh,
                                              int sp, uint8_t* __restrict__ dst, int dw, int dh,
                                              int dp) {
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

// Batched form: blockIdx.z = sequence, level l of descs[z] from level l-1.
__global__ __launch_bounds__(256) void pyr_down_batched_kernel(const PyrDesc* __restrict__ descs,
                                                               int level) {
    const PyrDesc& P = descs[blockIdx.z];
    const ImgLevel& s = P.lv[level - 1];
    const ImgLevel& d = P.lv[level];
    if ((int)blockIdx.x * PD_TX >= d.w || (int)blockIdx.y * PD_TY >= d.h) return;
    // same body as pyr_down_kernel (inlined call keeps one copy of the math)
    pyr_down_tile(s.data, s.w, s.h, s.pitch, const_cast<uint8_t*>(d.data), d.w, d.h, d.pitch);
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

hipError_t launch_pyramid_batched(const PyrDesc* d_descs, int nseq, int w, int h, int nlevels,
                                  hipStream_t st) {
    int lw = w, lh = h;
    for (int l = 1; l < nlevels; l++) {
        lw = (lw + 1) / 2;
        lh = (lh + 1) / 2;
        dim3 grid((lw + PD_TX - 1) / PD_TX, (lh + PD_TY - 1) / PD_TY, nseq);
        hipLaunchKernelGGL(pyr_down_batched_kernel, grid, dim3(256), 0, st, d_descs, l);
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

// NT: the derivative and level stores as non-temporal (streaming) stores
template <bool NT>
__global__ __launch_bounds__(256) void pyr_scharr_kernel(const PyrDesc* __restrict__ descs,
                                                         const DerivDesc* __restrict__ ders, int level) {
    const PyrDesc& P = descs[blockIdx.z];
    const ImgLevel& s = P.lv[level];
    const ImgLevel& d = P.lv[level + 1];
    const int x0 = blockIdx.x * PD_TX, y0 = blockIdx.y * PD_TY;
    const int sx0 = 2 * x0 - 2, sy0 = 2 * y0 - 2;
    const int xa = sx0 - 2;  // multiple of 4 (x0 is a multiple of 64)
    __shared__ __attribute__((aligned(16))) uint8_t T[FS_IH][FS_IW + 8];  // rows 16-byte aligned (b128 reads)
    __shared__ int H[PD_IH][PD_TX + 1];
    const int tid = threadIdx.x;
    const int sw = s.w, sh = s.h;
    const bool interior = xa >= 0 && sy0 >= 0 && xa + FS_IW <= sw && sy0 + FS_IH <= sh;
    if (interior) {
        constexpr int DW = FS_IW / 4;  // 34 dwords per row
        for (int k = tid; k < FS_IH * DW; k += 256) {
            const int r = k / DW, c4 = k - r * DW;
            *reinterpret_cast<uint32_t*>(&T[r][4 * c4]) =
                *reinterpret_cast<const uint32_t*>(s.data + (size_t)(sy0 + r) * s.pitch + xa + 4 * c4);
        }
    } else {
        for (int k = tid; k < FS_IH * FS_IW; k += 256) {
            const int r = k / FS_IW, c = k - r * FS_IW;
            T[r][c] = s.data[(size_t)refl101(sy0 + r, sh) * s.pitch + refl101(xa + c, sw)];
        }
    }
    __syncthreads();
    // ---- pyrDown rows: T column 2 + j holds level-l column sx0 + j; a task
    // makes 4 outputs (c = 4q .. 4q + 3) from 4 aligned dwords of its row ----
    for (int k = tid; k < PD_IH * (PD_TX / 4); k += 256) {
        const int r = k >> 4, q = k & 15;
        const uint4 v = *reinterpret_cast<const uint4*>(&T[r][8 * q]);
        const unsigned w4[4] = {v.x, v.y, v.z, v.w};
        int bt[16];
#pragma unroll
        for (int i = 0; i < 16; i++) bt[i] = (w4[i >> 2] >> (8 * (i & 3))) & 0xFF;
#pragma unroll
        for (int m = 0; m < 4; m++)
            H[r][4 * q + m] = bt[2 * m + 2] + 4 * bt[2 * m + 3] + 6 * bt[2 * m + 4] + 4 * bt[2 * m + 5] + bt[2 * m + 6];
    }
    // ---- Scharr of level l pixels (2x0 + i, 2y0 + j), i < 128, j < 32: T[2 + j][4 + i];
    // a task: 4 columns x 4 rows from 3 aligned dwords per staged row, one 16-byte
    // store per row (columns >= sw are never written: the zero border stays) ----
    {
        uint32_t* __restrict__ out = ders[blockIdx.z].data[level];
        const int op = ders[blockIdx.z].pitch[level];
        const int g = tid & 31, q = tid >> 5;
        const int x = 2 * x0 + 4 * g;
        int rows[6][6];  // staged rows 1 + 4q .. 6 + 4q, T columns 3 + 4g .. 8 + 4g
#pragma unroll
        for (int rr = 0; rr < 6; rr++) {
            const uint8_t* trow = &T[1 + 4 * q + rr][0];
            const unsigned a0 = *reinterpret_cast<const unsigned*>(trow + 4 * g);
            const unsigned a1 = *reinterpret_cast<const unsigned*>(trow + 4 * g + 4);
            const unsigned a2 = *reinterpret_cast<const unsigned*>(trow + 4 * g + 8);
            rows[rr][0] = a0 >> 24;
            rows[rr][1] = a1 & 0xFF;
            rows[rr][2] = (a1 >> 8) & 0xFF;
            rows[rr][3] = (a1 >> 16) & 0xFF;
            rows[rr][4] = a1 >> 24;
            rows[rr][5] = a2 & 0xFF;
        }
        if (x < sw) {
#pragma unroll
            for (int jj = 0; jj < 4; jj++) {
                const int y = 2 * y0 + 4 * q + jj;
                if (y >= sh) break;
                unsigned o[4];
#pragma unroll
                for (int m = 0; m < 4; m++) {
                    const int tl = rows[jj][m], tm = rows[jj][m + 1], tr = rows[jj][m + 2];
                    const int ml = rows[jj + 1][m], mr = rows[jj + 1][m + 2];
                    const int bl = rows[jj + 2][m], bm = rows[jj + 2][m + 1], br = rows[jj + 2][m + 2];
                    const int ix = (3 * (tr + br) + 10 * mr) - (3 * (tl + bl) + 10 * ml);
                    const int iy = 3 * ((br - tr) + (bl - tl)) + 10 * (bm - tm);
                    o[m] = ((unsigned)(iy * (1 << kDerShift)) << 16) | ((unsigned)(ix * (1 << kDerShift)) & 0xFFFFu);
                }
                uint32_t* dst = out + (size_t)y * op + x;
                if (x + 3 < sw) {
                    if constexpr (NT) {
                        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
                        const u32x4 v = {o[0], o[1], o[2], o[3]};
                        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst));
                    } else {
                        *reinterpret_cast<uint4*>(dst) = make_uint4(o[0], o[1], o[2], o[3]);
                    }
                } else {
#pragma unroll
                    for (int m = 0; m < 4; m++)
                        if (x + m < sw) dst[m] = o[m];
                }
            }
        }
    }
    __syncthreads();
    // ---- pyrDown columns: 4 output rows per thread from 11 sliding H rows ----
    const int c = tid & 63;
    const int x = x0 + c;
    if (x >= d.w) return;
    uint8_t* __restrict__ dst = const_cast<uint8_t*>(d.data);
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

hipError_t launch_pyramid_scharr_batched(const PyrDesc* d_descs, const DerivDesc* d_ders, int nseq, int w, int h,
                                         int nlevels, hipStream_t st) {
    int lw = w, lh = h;
    for (int l = 0; l + 1 < nlevels; l++) {
        const int nw = (lw + 1) / 2, nh = (lh + 1) / 2;
        dim3 grid((nw + PD_TX - 1) / PD_TX, (nh + PD_TY - 1) / PD_TY, nseq);
        // non-temporal derivative stores (SVO_PYR_NT=0: plain): the chain alone
        // 97.6 -> 89.5 us per 64 frames, the step unchanged (LK reads them a step later)
        static const bool nt = [] {
            const char* e = std::getenv("SVO_PYR_NT");
            return !(e && e[0] == '0');
        }();
        if (nt)
            hipLaunchKernelGGL(pyr_scharr_kernel<true>, grid, dim3(256), 0, st, d_descs, d_ders, l);
        else
            hipLaunchKernelGGL(pyr_scharr_kernel<false>, grid, dim3(256), 0, st, d_descs, d_ders, l);
        lw = nw;
        lh = nh;
    }
    // the coarsest level's derivative (no pyrDown after it), then the borders
    hipError_t e = launch_scharr_level(d_descs, d_ders, nseq, lw, lh, nlevels - 1, st);
    if (e != hipSuccess) return e;
    return launch_pyramid_pad(d_descs, nseq, w, h, nlevels, st);
}

}  // namespace svo
