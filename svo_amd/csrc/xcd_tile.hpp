// XCD-aware tile order for the image-tile kernels (fast.hip, pyramid.hip).
//
// gfx950 deals a launch's blocks round-robin over its 8 XCDs (linear block ids
// b, b + 8, b + 16, ... run on one XCD, each with its own 4 MiB L2). In plain
// raster order a tile's left, right, upper and lower neighbours all run on other
// XCDs, so every staged halo row / column is fetched again from HBM (or MALL) by
// a second XCD: the FAST and pyrDown tiles read 2-4x their frame's bytes. Here
// the tiles one XCD runs are consecutive in raster order (x fastest, then y, then
// the sequence), and the neighbours' halos come from that XCD's L2.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdlib>

namespace svo {

struct XcdTile {
    int x, y, z;
};

// The tile (x, y, z) of a (gridDim.x, gridDim.y, gridDim.z) launch this block
// computes: a bijection on the grid for any block count.
__device__ __forceinline__ XcdTile xcd_tile() {
    const unsigned gx = gridDim.x, gxy = gridDim.x * gridDim.y;
    const unsigned n = gxy * gridDim.z;
    const unsigned b = blockIdx.x + gx * blockIdx.y + gxy * blockIdx.z;
    // XCD slot k = b % 8 runs blocks k, k + 8, ...: q + 1 of them for k < r, q otherwise
    const unsigned q = n >> 3, r = n & 7, k = b & 7;
    const unsigned t = k * q + min(k, r) + (b >> 3);
    XcdTile o;
    o.z = (int)(t / gxy);
    const unsigned rem = t - (unsigned)o.z * gxy;
    o.y = (int)(rem / gx);
    o.x = (int)(rem - (unsigned)o.y * gx);
    return o;
}

// SVO_XCD_TILES=0: plain raster order for the two tile kernels whose launch takes
// an XT template flag -- fast_detect_q_kernel<.., XT> (fast.hip) and
// pyr_scharr_kernel<.., .., XT> (pyramid.hip). It does NOT switch the other
// users of xcd_tile(), which always run in XCD order: fast_box_filter_kernel and
// fast_emit_kernel (fast.hip), pyr_chain_kernel and its tail (pyramid.hip); LK
// has its own switch (SVO_LK_XCD, lk.hip). The recorded A/B
// (profiles/r04/n_xcd_tiles_ab.txt) therefore measures those two kernels'
// mapping only.
inline bool xcd_tiles_on() {
    static const bool on = [] {
        const char* e = std::getenv("SVO_XCD_TILES");
        return !(e && e[0] == '0');
    }();
    return on;
}

}  // namespace svo
