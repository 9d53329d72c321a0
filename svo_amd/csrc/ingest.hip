// Colour ingest: the reference loader reads KITTI's colour
// images and converts them on the host, R:include/async_image_loader.h:63-69
// (cv::imread -> cv::cvtColor(COLOR_BGR2GRAY)). Here the BGR rows travel over
// PCIe as they are (through a pinned double buffer, capi.cpp) and this kernel
// writes the grey level 0 of the device pyramid directly, so there is no grey
// staging image.
//
// OpenCV's CV_8U RGB2Gray (color_rgb: R2Y 4899, G2Y 9617, B2Y 1868, yuv_shift
// 14, rounding constant 1 << 13 folded into the red table) is exact integer
// arithmetic: gray = (1868 B + 9617 G + 4899 R + 8192) >> 14.
//
// Byte-moving kernel, HBM bound: 3 B in + 1 B out per pixel. One thread makes
// four pixels from three aligned dwords and stores one dword.
#include "common.hpp"

namespace svo {

__device__ __forceinline__ uint32_t gray_of(uint32_t b, uint32_t g, uint32_t r) {
    return (b * 1868u + g * 9617u + r * 4899u + 8192u) >> 14;
}

// bgr: packed rows, `bpitch` bytes apart (multiple of 4); dst: level 0 rows.
__global__ void __launch_bounds__(256) bgr_to_gray_kernel(const uint8_t* __restrict__ bgr, int bpitch,
                                                          uint8_t* __restrict__ dst, int pitch, int w, int h) {
    const int y = blockIdx.y;
    const int q = blockIdx.x * 256 + threadIdx.x;  // quad of pixels
    const int x = q * 4;
    if (x >= w || y >= h) return;
    const uint8_t* s = bgr + (size_t)y * bpitch + (size_t)x * 3;
    uint8_t* d = dst + (size_t)y * pitch + x;
    if (x + 4 <= w) {
        const uint32_t* s4 = reinterpret_cast<const uint32_t*>(s);
        const uint32_t a = s4[0], b = s4[1], c = s4[2];
        // bytes: a = B0 G0 R0 B1, b = G1 R1 B2 G2, c = R2 B3 G3 R3
        const uint32_t g0 = gray_of(a & 255, (a >> 8) & 255, (a >> 16) & 255);
        const uint32_t g1 = gray_of(a >> 24, b & 255, (b >> 8) & 255);
        const uint32_t g2 = gray_of((b >> 16) & 255, b >> 24, c & 255);
        const uint32_t g3 = gray_of((c >> 8) & 255, (c >> 16) & 255, c >> 24);
        *reinterpret_cast<uint32_t*>(d) = g0 | (g1 << 8) | (g2 << 16) | (g3 << 24);
    } else {
        for (int i = 0; x + i < w; i++) d[i] = (uint8_t)gray_of(s[3 * i], s[3 * i + 1], s[3 * i + 2]);
    }
}

hipError_t launch_bgr_to_gray(const uint8_t* bgr, int bpitch, uint8_t* dst, int pitch, int w, int h,
                              hipStream_t st) {
    if (w <= 0 || h <= 0 || (bpitch & 3) || bpitch < 3 * w) return hipErrorInvalidValue;
    const int quads = (w + 3) / 4;
    dim3 grid((quads + 255) / 256, h);
    hipLaunchKernelGGL(bgr_to_gray_kernel, grid, dim3(256), 0, st, bgr, bpitch, dst, pitch, w, h);
    return hipGetLastError();
}


// Streamed frames (svo_frontend_queue_frames): level 0 of every sequence's slot
// from a device staging block that mirrors the host frames byte for byte (rows
// `spitch` bytes apart, sequences `seq_stride` apart: one contiguous H2D copy per
// run of sequences -- a pitched 2D copy moves row by row, ~0.1 GB/s at KITTI's
// 1241-byte rows). BGR: the conversion above; grey: a copy. The rows need not be
// 4-byte aligned (1241, 3723 B): unaligned dword loads (global memory allows
// them). Grid (quads / 256, h, S); each sequence's level 0 from the descriptor
// array (its borders are the pyramid chain's to write).
typedef uint32_t u32a1 __attribute__((aligned(1)));
template <bool BGR>
__global__ void __launch_bounds__(256) ingest_batched_kernel(const uint8_t* __restrict__ stage, size_t seq_stride,
                                                             int spitch, const PyrDesc* __restrict__ descs, int w,
                                                             int h) {
    const int s = blockIdx.z, y = blockIdx.y;
    const int x = (blockIdx.x * 256 + threadIdx.x) * 4;
    if (x >= w) return;
    const ImgLevel L = descs[s].lv[0];
    const uint8_t* src = stage + (size_t)s * seq_stride + (size_t)y * spitch + (size_t)x * (BGR ? 3 : 1);
    uint8_t* d = const_cast<uint8_t*>(L.data) + (size_t)y * L.pitch + x;
    if (x + 4 <= w) {
        uint32_t out;
        const u32a1* s4 = reinterpret_cast<const u32a1*>(src);
        if (BGR) {
            const uint32_t a = s4[0], b = s4[1], c = s4[2];
            out = gray_of(a & 255, (a >> 8) & 255, (a >> 16) & 255) |
                  gray_of(a >> 24, b & 255, (b >> 8) & 255) << 8 |
                  gray_of((b >> 16) & 255, b >> 24, c & 255) << 16 |
                  gray_of((c >> 8) & 255, (c >> 16) & 255, c >> 24) << 24;
        } else {
            out = s4[0];
        }
        *reinterpret_cast<uint32_t*>(d) = out;  // (level 0 rows are 64-byte aligned at x = 0)
    } else {
        for (int i = 0; x + i < w; i++)
            d[i] = BGR ? (uint8_t)gray_of(src[3 * i], src[3 * i + 1], src[3 * i + 2]) : src[i];
    }
}

hipError_t launch_ingest_batched(const uint8_t* stage, size_t seq_stride, int spitch, const PyrDesc* descs, int S,
                                 int w, int h, bool bgr, hipStream_t st) {
    if (w <= 0 || h <= 0 || S <= 0 || spitch < (bgr ? 3 : 1) * w) return hipErrorInvalidValue;
    dim3 grid(((w + 3) / 4 + 255) / 256, h, S);
    if (bgr)
        hipLaunchKernelGGL(ingest_batched_kernel<true>, grid, dim3(256), 0, st, stage, seq_stride, spitch, descs, w, h);
    else
        hipLaunchKernelGGL(ingest_batched_kernel<false>, grid, dim3(256), 0, st, stage, seq_stride, spitch, descs, w,
                           h);
    return hipGetLastError();
}

}  // namespace svo
