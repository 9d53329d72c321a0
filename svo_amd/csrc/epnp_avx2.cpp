// The RANSAC minimal solver in AVX2 lanes (epnp_lanes.hpp, 4 subsets per
// register); this file alone is built with -mavx2 and called only on CPUs that
// have it (epnp_pixels_batch, pose.cpp).
#include "pose.hpp"

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>

// Every helper this file compiles -- epnp.hpp, linalg.hpp and simd_svd.hpp's
// inline functions and classes included -- is built with this file's
// instruction set. Under their own namespace name (svo_isa_avx2) they get
// symbols of their own: the linker can never fold one of them into the generic
// code's copy of the same helper (which a non-AVX2 CPU executes).
#define svo svo_isa_avx2
#include "epnp_lanes.hpp"
#undef svo

namespace svo {

void epnp_batch_avx2(int count, const float* const* obj, const float* const* img, const int* const* idx,
                     const double K[9], double (*R)[9], double (*t)[3], bool* ok) {
    if (count <= 4)
        svo_isa_avx2::epnp_lanes<4, 1>(count, obj, img, idx, K, R, t, ok);
    else if (count <= 8)
        svo_isa_avx2::epnp_lanes<4, 2>(count, obj, img, idx, K, R, t, ok);
    else
        svo_isa_avx2::epnp_lanes<4, 4>(count, obj, img, idx, K, R, t, ok);
}

}  // namespace svo
