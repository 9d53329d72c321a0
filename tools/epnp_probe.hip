// Probe: latency of the shared EPnP minimal solver (svo_amd/csrc/epnp.hpp) run
// one hypothesis per lane on the GPU, and whether its poses are bit-identical
// to the host's. Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off
//   -I svo_amd/csrc -I include tools/epnp_probe.hip -o tools/epnp_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "epnp.hpp"

using namespace svo;

__global__ void __launch_bounds__(64) epnp_kernel(const float* obj, const float* img, const int* idx, int m,
                                                  const double* K, double* out, int* ok) {
    const int j = blockIdx.x * 64 + threadIdx.x;
    if (j >= m) return;
    double Kl[9];
    for (int i = 0; i < 9; i++) Kl[i] = K[i];
    double R[9], t[3];
    ok[j] = epnp_pixels(obj, img, idx + 5 * j, 5, Kl, R, t) ? 1 : 0;
    for (int i = 0; i < 9; i++) out[12 * j + i] = R[i];
    for (int i = 0; i < 3; i++) out[12 * j + 9 + i] = t[i];
}

int main(int argc, char** argv) {
    const int n = 2000;
    const int m = argc > 1 ? atoi(argv[1]) : 6400;
    const int bs = argc > 2 ? atoi(argv[2]) : 64;
    (void)bs;
    std::mt19937 g(7);
    std::uniform_real_distribution<float> U(-1, 1);
    const double K[9] = {718.856, 0, 607.1928, 0, 718.856, 185.2157, 0, 0, 1};
    std::vector<float> obj(3 * n), img(2 * n);
    for (int i = 0; i < n; i++) {
        float X = 10 * U(g), Y = 3 * U(g), Z = 15 + 10 * U(g);
        obj[3 * i] = X;
        obj[3 * i + 1] = Y;
        obj[3 * i + 2] = Z;
        img[2 * i] = (float)(K[0] * X / Z + K[2] + 0.3 * U(g));
        img[2 * i + 1] = (float)(K[4] * Y / Z + K[5] + 0.3 * U(g));
    }
    std::vector<int> idx(5 * m);
    std::uniform_int_distribution<int> ui(0, n - 1);
    for (int j = 0; j < m; j++)
        for (int k = 0; k < 5; k++) {
            int v;
            bool dup;
            do {
                v = ui(g);
                dup = false;
                for (int q = 0; q < k; q++) dup |= idx[5 * j + q] == v;
            } while (dup);
            idx[5 * j + k] = v;
        }
    float *dobj, *dimg;
    int *didx, *dok;
    double *dK, *dout;
    hipMalloc(&dobj, sizeof(float) * 3 * n);
    hipMalloc(&dimg, sizeof(float) * 2 * n);
    hipMalloc(&didx, sizeof(int) * 5 * m);
    hipMalloc(&dok, sizeof(int) * m);
    hipMalloc(&dK, sizeof(double) * 9);
    hipMalloc(&dout, sizeof(double) * 12 * m);
    hipMemcpy(dobj, obj.data(), sizeof(float) * 3 * n, hipMemcpyHostToDevice);
    hipMemcpy(dimg, img.data(), sizeof(float) * 2 * n, hipMemcpyHostToDevice);
    hipMemcpy(didx, idx.data(), sizeof(int) * 5 * m, hipMemcpyHostToDevice);
    hipMemcpy(dK, K, sizeof(K), hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 3; rep++) {
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(epnp_kernel, dim3((m + 63) / 64), dim3(64), 0, 0, dobj, dimg, didx, m, dK, dout, dok);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("m=%d  gpu epnp: %.3f ms\n", m, ms);
    }
    std::vector<double> gout(12 * m);
    std::vector<int> gok(m);
    hipMemcpy(gout.data(), dout, sizeof(double) * 12 * m, hipMemcpyDeviceToHost);
    hipMemcpy(gok.data(), dok, sizeof(int) * m, hipMemcpyDeviceToHost);
    auto t0 = std::chrono::steady_clock::now();
    int same = 0, okc = 0;
    double maxd = 0;
    for (int j = 0; j < m; j++) {
        double R[9], t[3];
        bool ok = epnp_pixels(obj.data(), img.data(), &idx[5 * j], 5, K, R, t);
        okc += ok;
        bool eq = ok == (bool)gok[j];
        for (int i = 0; i < 9 && ok; i++) {
            eq &= R[i] == gout[12 * j + i];
            maxd = std::fmax(maxd, std::fabs(R[i] - gout[12 * j + i]));
        }
        for (int i = 0; i < 3 && ok; i++) {
            eq &= t[i] == gout[12 * j + 9 + i];
            maxd = std::fmax(maxd, std::fabs(t[i] - gout[12 * j + 9 + i]) / 10);
        }
        same += eq;
    }
    double host_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    printf("host epnp (1 thread): %.3f ms for %d (%.2f us each); ok %d; bit-identical %d / %d; max |d| %.3g\n",
           host_ms, m, 1e3 * host_ms / m, okc, same, m, maxd);
    return 0;
}
