// Scharr derivative pyramid (lkpyramid.cpp calcSharrDeriv) for gfx950.
//
// OpenCV computes the derivative of every prev-pyramid level inside each
// calcOpticalFlowPyrLK call (R:src/tracking.cpp:101, :160). Here it is computed
// once per frame for all levels and all sequences of a batch (one launch per
// level), stored as packed int16 pairs (Ix | Iy << 16) per pixel, and read by
// the LK kernel. Bit-exact integer arithmetic:
//   t0 = 3*(r[y-1] + r[y+1]) + 10*r[y],  t1 = r[y+1] - r[y-1]   (rows REFLECT_101)
//   Ix = t0[x+1] - t0[x-1],  Iy = 3*(t1[x+1] + t1[x-1]) + 10*t1[x] (cols REFLECT_101)
// HBM: reads w*h, writes 4*w*h bytes per level.
#include "common.hpp"

namespace svo {

namespace {

__device__ __forceinline__ int refl101(int p, int len) {
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        p = p < 0 ? -p : 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

constexpr int SC_TX = 64, SC_TY = 16;
constexpr int SC_IW = SC_TX + 2, SC_IH = SC_TY + 2;

__global__ __launch_bounds__(256) void scharr_kernel(const PyrDesc* __restrict__ pyrs,
                                                     const DerivDesc* __restrict__ ders, int level) {
    const ImgLevel& L = pyrs[blockIdx.z].lv[level];
    const int w = L.w, h = L.h;
    const int x0 = blockIdx.x * SC_TX, y0 = blockIdx.y * SC_TY;
    if (x0 >= w || y0 >= h) return;
    uint32_t* __restrict__ out = ders[blockIdx.z].data[level];
    const int op = ders[blockIdx.z].pitch[level];
    __shared__ uint8_t T[SC_IH][SC_IW + 2];
    const int tid = threadIdx.x;
    const bool inside = x0 >= 1 && y0 >= 1 && x0 + SC_IW - 1 <= w && y0 + SC_IH - 1 <= h;
    for (int k = tid; k < SC_IH * SC_IW; k += 256) {
        const int r = k / SC_IW, c = k - r * SC_IW;
        int y = y0 - 1 + r, x = x0 - 1 + c;
        if (!inside) {
            y = refl101(y, h);
            x = refl101(x, w);
        }
        T[r][c] = L.data[(size_t)y * L.pitch + x];
    }
    __syncthreads();
    const int c = tid & 63;
    const int x = x0 + c;
    if (x >= w) return;
    // column reflect of the vertically filtered rows == reflect of the image columns
#pragma unroll
    for (int i = 0; i < SC_TY / 4; i++) {
        const int r = (tid >> 6) * (SC_TY / 4) + i;
        const int y = y0 + r;
        if (y >= h) break;
        const int tl = T[r][c], tm = T[r][c + 1], tr = T[r][c + 2];
        const int ml = T[r + 1][c], mr = T[r + 1][c + 2];
        const int bl = T[r + 2][c], bm = T[r + 2][c + 1], br = T[r + 2][c + 2];
        const int ix = (3 * (tr + br) + 10 * mr) - (3 * (tl + bl) + 10 * ml);
        const int iy = 3 * ((br - tr) + (bl - tl)) + 10 * (bm - tm);
        out[(size_t)y * op + x] = ((unsigned)(iy * (1 << kDerShift)) << 16) | ((unsigned)(ix * (1 << kDerShift)) & 0xFFFFu);
    }
}

}  // namespace

hipError_t launch_scharr(const PyrDesc* d_pyrs, const DerivDesc* d_ders, int nseq, int w, int h, int nlevels,
                         hipStream_t st) {
    int lw = w, lh = h;
    for (int l = 0; l < nlevels; l++) {
        dim3 grid((lw + SC_TX - 1) / SC_TX, (lh + SC_TY - 1) / SC_TY, nseq);
        hipLaunchKernelGGL(scharr_kernel, grid, dim3(256), 0, st, d_pyrs, d_ders, l);
        lw = (lw + 1) / 2;
        lh = (lh + 1) / 2;
    }
    return hipGetLastError();
}

hipError_t launch_scharr_level(const PyrDesc* d_pyrs, const DerivDesc* d_ders, int nseq, int lw, int lh, int level,
                               hipStream_t st) {
    dim3 grid((lw + SC_TX - 1) / SC_TX, (lh + SC_TY - 1) / SC_TY, nseq);
    hipLaunchKernelGGL(scharr_kernel, grid, dim3(256), 0, st, d_pyrs, d_ders, level);
    return hipGetLastError();
}

size_t deriv_layout(int w, int h, int nlevels, size_t* off, int* pitch) {
    size_t total = 0;
    int lw = w, lh = h;
    for (int l = 0; l < nlevels; l++) {
        pitch[l] = (lw + 2 * kDerPad + 15) & ~15;
        off[l] = total + ((size_t)kDerPad * pitch[l] + kDerPad) * 4;
        total += (size_t)pitch[l] * (lh + 2 * kDerPad) * 4;
        total = (total + 255) & ~(size_t)255;
        lw = (lw + 1) / 2;
        lh = (lh + 1) / 2;
    }
    return total;
}

}  // namespace svo
