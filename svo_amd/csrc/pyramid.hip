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
// rewrite a few interior pixels with their own values). Blocks of one level
// stride over the dwords.
__device__ __forceinline__ void pad_level(const ImgLevel& L, int blk, int nblk) {
    constexpr int SIDE = kPyrPad / 4 + 1;  // dwords per row on each side (right side: alignment)
    const int w = L.w, h = L.h, dw = (w + 2 * kPyrPad + 3) / 4;
    const int n_tb = 2 * kPyrPad * dw, n = n_tb + 2 * SIDE * h;
    uint8_t* __restrict__ d = const_cast<uint8_t*>(L.data);
    for (int k = blk * 256 + (int)threadIdx.x; k < n; k += nblk * 256) {
        int x0, y;
        if (k < n_tb) {
            const int r = k / dw, c = k - r * dw;
            y = r < kPyrPad ? r - kPyrPad : h + (r - kPyrPad);
            x0 = 4 * c - kPyrPad;
        } else {
            const int k2 = k - n_tb, r = k2 / (2 * SIDE), c = k2 - r * (2 * SIDE);
            y = r;
            x0 = c < SIDE ? -kPyrPad + 4 * c : (w & ~3) + 4 * (c - SIDE);
            if (c > 0 && c < SIDE && x0 >= 0) continue;  // left side: SIDE - 1 dwords suffice
        }
        const uint8_t* srow = d + (ptrdiff_t)refl101(y, h) * L.pitch;
        unsigned v = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) v |= (unsigned)srow[refl101(x0 + i, w)] << (8 * i);
        *reinterpret_cast<unsigned*>(d + (ptrdiff_t)y * L.pitch + x0) = v;
    }
}

constexpr int PAD_BLOCKS = 8;  // blocks per (level, sequence)

__global__ __launch_bounds__(256) void pad_batched_kernel(const PyrDesc* __restrict__ descs) {
    pad_level(descs[blockIdx.z].lv[blockIdx.y], blockIdx.x, gridDim.x);
}
__global__ __launch_bounds__(256) void pad_kernel(PyrDesc d) { pad_level(d.lv[blockIdx.y], blockIdx.x, gridDim.x); }

hipError_t launch_pyramid_pad(const PyrDesc* d_descs, int nseq, int w, int h, int nlevels, hipStream_t st) {
    (void)w;
    (void)h;
    hipLaunchKernelGGL(pad_batched_kernel, dim3(PAD_BLOCKS, nlevels, nseq), dim3(256), 0, st, d_descs);
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
    hipLaunchKernelGGL(pad_kernel, dim3(PAD_BLOCKS, img->nlevels), dim3(256), 0, st, img->desc);
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

__global__ __launch_bounds__(256) void pyr_scharr_kernel(const PyrDesc* __restrict__ descs,
                                                         const DerivDesc* __restrict__ ders, int level) {
    const PyrDesc& P = descs[blockIdx.z];
    const ImgLevel& s = P.lv[level];
    const ImgLevel& d = P.lv[level + 1];
    const int x0 = blockIdx.x * PD_TX, y0 = blockIdx.y * PD_TY;
    const int sx0 = 2 * x0 - 2, sy0 = 2 * y0 - 2;
    const int xa = sx0 - 2;  // multiple of 4 (x0 is a multiple of 64)
    __shared__ __attribute__((aligned(16))) uint8_t T[FS_IH][FS_IW];
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
    // ---- pyrDown: T column 2 + j holds level-l column sx0 + j ----
    for (int k = tid; k < PD_IH * PD_TX; k += 256) {
        const int r = k >> 6, c = k & 63;
        const uint8_t* t = &T[r][2 * c + 2];
        H[r][c] = t[0] + 4 * t[1] + 6 * t[2] + 4 * t[3] + t[4];
    }
    // ---- Scharr of level l pixels (2x0 + i, 2y0 + j), i < 128, j < 32: T[2 + j][4 + i] ----
    {
        uint32_t* __restrict__ out = ders[blockIdx.z].data[level];
        const int op = ders[blockIdx.z].pitch[level];
        const int i = tid & 127, j0 = (tid >> 7) * 16;
        const int x = 2 * x0 + i;
        if (x < sw) {
            const int tc = 4 + i;
            int tl = T[1 + j0][tc - 1], tm = T[1 + j0][tc], tr = T[1 + j0][tc + 1];
            int ml = T[2 + j0][tc - 1], mm = T[2 + j0][tc], mr = T[2 + j0][tc + 1];
#pragma unroll 4
            for (int jj = 0; jj < 16; jj++) {
                const int y = 2 * y0 + j0 + jj;
                const int br = T[3 + j0 + jj][tc + 1], bm = T[3 + j0 + jj][tc], bl = T[3 + j0 + jj][tc - 1];
                if (y < sh) {
                    const int ix = (3 * (tr + br) + 10 * mr) - (3 * (tl + bl) + 10 * ml);
                    const int iy = 3 * ((br - tr) + (bl - tl)) + 10 * (bm - tm);
                    out[(size_t)y * op + x] = ((unsigned)(iy * (1 << kDerShift)) << 16) | ((unsigned)(ix * (1 << kDerShift)) & 0xFFFFu);
                }
                tl = ml; tm = mm; tr = mr;
                ml = bl; mm = bm; mr = br;
            }
        }
    }
    __syncthreads();
    const int c = tid & 63;
    const int x = x0 + c;
    if (x >= d.w) return;
    uint8_t* __restrict__ dst = const_cast<uint8_t*>(d.data);
#pragma unroll
    for (int i = 0; i < PD_TY / 4; i++) {
        const int r = (tid >> 6) * (PD_TY / 4) + i;
        const int y = y0 + r;
        if (y < d.h) {
            const int sum = H[2 * r][c] + 4 * H[2 * r + 1][c] + 6 * H[2 * r + 2][c] + 4 * H[2 * r + 3][c] +
                            H[2 * r + 4][c];
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
        hipLaunchKernelGGL(pyr_scharr_kernel, grid, dim3(256), 0, st, d_descs, d_ders, l);
        lw = nw;
        lh = nh;
    }
    // the coarsest level's derivative (no pyrDown after it), then the borders
    hipError_t e = launch_scharr_level(d_descs, d_ders, nseq, lw, lh, nlevels - 1, st);
    if (e != hipSuccess) return e;
    return launch_pyramid_pad(d_descs, nseq, w, h, nlevels, st);
}

}  // namespace svo
