// RANSAC's EPnP minimal solver on the GPU, one 64-lane wave per 5-point subset
// (epnp_wave.hpp), bit-identical to the host solver the front end uses
// (epnp.hpp). Measured and kept off the front end's path: a single
// hypothesis takes ~150 us of serial double-precision chain against ~7.5 us on
// a host core; it pays only for thousands of hypotheses at once.
#include "common.hpp"
#include "epnp_wave.hpp"

namespace svo {

namespace {

__global__ __launch_bounds__(64) void epnp_wave_kernel(const float* __restrict__ subsets, int m, const double* Kd,
                                                       double* __restrict__ Rt, int* __restrict__ ok) {
    __shared__ wep::Work S;
    const int j = blockIdx.x, lane = threadIdx.x;
    if (j >= m) return;
    double K[9];
#pragma unroll
    for (int i = 0; i < 9; i++) K[i] = Kd[i];
    const float* sp = subsets + 25 * (size_t)j;
    double R[9], t[3];
    const bool v = wep::solve5(S, lane, sp, sp + 15, K, R, t);
    if (lane == 0) {
        ok[j] = v ? 1 : 0;
#pragma unroll
        for (int i = 0; i < 9; i++) Rt[12 * (size_t)j + i] = R[i];
#pragma unroll
        for (int i = 0; i < 3; i++) Rt[12 * (size_t)j + 9 + i] = t[i];
    }
}

}  // namespace

hipError_t launch_epnp_wave(const float* subsets, int m, const double* K, double* Rt, int* ok, hipStream_t st) {
    if (m <= 0) return hipSuccess;
    hipLaunchKernelGGL(epnp_wave_kernel, dim3(m), dim3(64), 0, st, subsets, m, K, Rt, ok);
    return hipGetLastError();
}

}  // namespace svo
