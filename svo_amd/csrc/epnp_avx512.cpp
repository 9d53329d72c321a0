// The RANSAC minimal solver in AVX-512 lanes (epnp_lanes.hpp, 8 subsets per
// register); this file alone is built with -mavx512f and called only on CPUs
// that have it (epnp_pixels_batch, pose.cpp).
#include "epnp_lanes.hpp"
#include "pose.hpp"

namespace svo {

void epnp_batch_avx512(int count, const float* const* obj, const float* const* img, const int* const* idx,
                       const double K[9], double (*R)[9], double (*t)[3], bool* ok) {
    if (count <= 8)
        epnp_lanes<8, 1>(count, obj, img, idx, K, R, t, ok);
    else
        epnp_lanes<8, 2>(count, obj, img, idx, K, R, t, ok);
}

}  // namespace svo
