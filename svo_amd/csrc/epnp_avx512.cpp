// The RANSAC minimal solver in AVX-512 lanes (epnp_lanes.hpp, 8 subsets per
// register); this file alone is built with -mavx512f and called only on CPUs
// that have it (epnp_pixels_batch, pose.cpp).
#include "pose.hpp"

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>

// Every helper this file compiles -- epnp.hpp, linalg.hpp and simd_svd.hpp's
// inline functions and classes included -- is built with this file's
// instruction set. Under their own namespace name (svo_isa_avx512) they get
// symbols of their own: the linker can never fold one of them into the generic
// code's copy of the same helper (which a non-AVX512 CPU executes).
#define svo svo_isa_avx512
#include "epnp_lanes.hpp"
#undef svo

namespace svo {

void epnp_batch_avx512(int count, const float* const* obj, const float* const* img, const int* const* idx,
                     const double K[9], double (*R)[9], double (*t)[3], bool* ok) {
    if (count <= 8)
        svo_isa_avx512::epnp_lanes<8, 1>(count, obj, img, idx, K, R, t, ok);
    else
        svo_isa_avx512::epnp_lanes<8, 2>(count, obj, img, idx, K, R, t, ok);
}

}  // namespace svo
