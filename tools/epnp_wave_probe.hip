// Probe: the wave-cooperative EPnP (svo_amd/csrc/epnp_wave.hpp, one 64-lane wave
// per hypothesis) against the host solver (epnp.hpp): bit-identity of R / t and
// latency per launch for a step's worth of hypotheses (128) and for many.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I svo_amd/csrc -I include \
//         tools/epnp_wave_probe.hip -o tools/epnp_wave_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "epnp.hpp"
// phase stamps of hypothesis 0 (s_memtime, lane 0): 1 tred2, 2 back-transform,
// 3 tql2, 4 sort, 5 make_L, 6 betas + Gauss-Newton + R,t (7 end)
__device__ unsigned long long g_stamps[8];
#define WEP_STAMP(k)                                                                 \
    do {                                                                             \
        if (blockIdx.x == 0 && threadIdx.x == 0) g_stamps[k] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#include "epnp_wave.hpp"

using namespace svo;

__global__ void __launch_bounds__(64) epnp_wave_kernel(const float* samp, int m, const double* Kd, double* out, int* ok) {
    __shared__ wep::Work S;
    const int j = blockIdx.x, lane = threadIdx.x;
    if (j >= m) return;
    double K[9];
    for (int i = 0; i < 9; i++) K[i] = Kd[i];
    const float* sp = samp + 25 * (size_t)j;
    double R[9], t[3];
    WEP_STAMP(0);
    const bool v = wep::solve5(S, lane, sp, sp + 15, K, R, t);
    if (lane == 0) {
        ok[j] = v ? 1 : 0;
        for (int i = 0; i < 9; i++) out[12 * j + i] = R[i];
        for (int i = 0; i < 3; i++) out[12 * j + 9 + i] = t[i];
    }
}

int main(int argc, char** argv) {
    const int n = 2000;
    const int mbig = argc > 1 ? atoi(argv[1]) : 8192;
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
    // 5-point subsets as the front end gathers them: obj[5][3] then img[5][2]
    std::vector<float> samp(25 * (size_t)mbig);
    std::uniform_int_distribution<int> ui(0, n - 1);
    for (int j = 0; j < mbig; j++) {
        int idx[5];
        for (int k = 0; k < 5; k++) {
            int v;
            bool dup;
            do {
                v = ui(g);
                dup = false;
                for (int q = 0; q < k; q++) dup |= idx[q] == v;
            } while (dup);
            idx[k] = v;
        }
        float* s = &samp[25 * (size_t)j];
        for (int k = 0; k < 5; k++) {
            for (int c = 0; c < 3; c++) s[3 * k + c] = obj[3 * idx[k] + c];
            for (int c = 0; c < 2; c++) s[15 + 2 * k + c] = img[2 * idx[k] + c];
        }
    }
    float* dsamp;
    double *dK, *dout;
    int* dok;
    (void)hipMalloc(&dsamp, sizeof(float) * samp.size());
    (void)hipMalloc(&dK, sizeof(double) * 9);
    (void)hipMalloc(&dout, sizeof(double) * 12 * mbig);
    (void)hipMalloc(&dok, sizeof(int) * mbig);
    (void)hipMemcpy(dsamp, samp.data(), sizeof(float) * samp.size(), hipMemcpyHostToDevice);
    (void)hipMemcpy(dK, K, sizeof(K), hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int m : {1, 128, 1024, mbig}) {
        float best = 1e30f;
        for (int rep = 0; rep < 5; rep++) {
            (void)hipEventRecord(e0, 0);
            hipLaunchKernelGGL(epnp_wave_kernel, dim3(m), dim3(64), 0, 0, dsamp, m, dK, dout, dok);
            (void)hipEventRecord(e1, 0);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            best = std::fmin(best, ms);
        }
        printf("wave EPnP: %5d hypotheses, %8.1f us per launch (best of 5)\n", m, 1e3 * best);
    }
    {
        unsigned long long st[8];
        (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stamps), sizeof(st));
        const char* nm[7] = {"prelude + M^T M", "tred2", "back-transform", "tql2", "sort", "make_L",
                             "betas + Gauss-Newton + R,t"};
        printf("phases of one hypothesis (s_memtime, shader clock cycles):");
        for (int k = 0; k < 7; k++) printf(" %s %llu;", nm[k], st[k + 1] - st[k]);
        printf("\n");
    }
    std::vector<double> gout(12 * (size_t)mbig);
    std::vector<int> gok(mbig);
    (void)hipMemcpy(gout.data(), dout, sizeof(double) * gout.size(), hipMemcpyDeviceToHost);
    (void)hipMemcpy(gok.data(), dok, sizeof(int) * mbig, hipMemcpyDeviceToHost);
    auto t0 = std::chrono::steady_clock::now();
    int same = 0, okc = 0, okm = 0;
    double maxd = 0;
    for (int j = 0; j < mbig; j++) {
        double R[9], t[3];
        const float* s = &samp[25 * (size_t)j];
        const bool ok = epnp_pixels(s, s + 15, nullptr, 5, K, R, t);
        okc += ok;
        okm += ok == (bool)gok[j];
        bool eq = ok == (bool)gok[j];
        for (int i = 0; i < 9 && ok; i++) {
            eq &= R[i] == gout[12 * j + i];
            maxd = std::fmax(maxd, std::fabs(R[i] - gout[12 * j + i]));
        }
        for (int i = 0; i < 3 && ok; i++) {
            eq &= t[i] == gout[12 * j + 9 + i];
            maxd = std::fmax(maxd, std::fabs(t[i] - gout[12 * j + 9 + i]));
        }
        same += eq;
    }
    const double host_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    printf("host EPnP (1 thread): %.2f us per hypothesis; valid %d, flags equal %d / %d; R,t bit-identical %d / %d; "
           "max |d| %.3g\n",
           1e3 * host_ms / mbig, okc, okm, mbig, same, mbig, maxd);
    return same == mbig ? 0 : 1;
}
