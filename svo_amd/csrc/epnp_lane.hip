// RANSAC's EPnP minimal solver on the GPU, one LANE per 5-point subset: each
// lane runs the front end's host solver itself (epnp.hpp: calib3d's epnp.cpp
// with OpenCV's Jacobi SVDs, la::cv), operation for operation in the scalar
// order -- the form epnp_lanes.hpp runs in host SIMD lanes, bit-identical to the
// oracle (tests/test_epnp_cpu.py) -- instead of spreading one subset over a
// wave (epnp_wave.hip, a QL variant). 64 subsets per wave, the subset's data in
// the lane's private memory. svo_epnp_subsets(device = 6).
#include "common.hpp"
#include "epnp.hpp"

namespace svo {

namespace {

__global__ __launch_bounds__(64) void epnp_lane_kernel(const float* __restrict__ subsets, int m,
                                                       const double* __restrict__ Kd, double* __restrict__ Rt,
                                                       int* __restrict__ ok) {
    const int j = blockIdx.x * 64 + threadIdx.x;
    if (j >= m) return;
    double K[9];
#pragma unroll
    for (int i = 0; i < 9; i++) K[i] = Kd[i];
    float sp[25];
#pragma unroll
    for (int i = 0; i < 25; i++) sp[i] = subsets[25 * (size_t)j + i];
    double R[9], t[3];
    const bool v = epnp_pixels(sp, sp + 15, nullptr, 5, K, R, t);
    ok[j] = v ? 1 : 0;
#pragma unroll
    for (int i = 0; i < 9; i++) Rt[12 * (size_t)j + i] = R[i];
#pragma unroll
    for (int i = 0; i < 3; i++) Rt[12 * (size_t)j + 9 + i] = t[i];
}

}  // namespace

hipError_t launch_epnp_lanes(const float* subsets, int m, const double* K, double* Rt, int* ok, hipStream_t st) {
    if (m <= 0) return hipSuccess;
    hipLaunchKernelGGL(epnp_lane_kernel, dim3((m + 63) / 64), dim3(64), 0, st, subsets, m, K, Rt, ok);
    return hipGetLastError();
}

}  // namespace svo
