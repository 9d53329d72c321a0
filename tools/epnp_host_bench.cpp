// Host timing of the EPnP minimal solver (svo_amd/csrc/epnp.hpp) as the frontend's
// RANSAC runs it: random 5-point subsets of a synthetic scene, one thread.
// Build: g++/clang++ -O3 -ffp-contract=off -I svo_amd/csrc -I include tools/epnp_host_bench.cpp
#include <chrono>
#include <cstdio>
#include <random>
#include <vector>


#include "epnp.hpp"

using namespace svo;

int main() {
    const int n = 2000, m = 20000;
    std::mt19937 g(7);
    std::uniform_real_distribution<float> U(-1, 1);
    const double K[9] = {718.856, 0, 607.1928, 0, 718.856, 185.2157, 0, 0, 1};
    std::vector<float> obj(3 * n), img(2 * n);
    for (int i = 0; i < n; i++) {
        float X = 10 * U(g), Y = 3 * U(g), Z = 15 + 10 * U(g);
        obj[3 * i] = X, obj[3 * i + 1] = Y, obj[3 * i + 2] = Z;
        img[2 * i] = (float)(K[0] * X / Z + K[2] + 0.3 * U(g));
        img[2 * i + 1] = (float)(K[4] * Y / Z + K[5] + 0.3 * U(g));
    }
    std::vector<int> idx(5 * m);
    for (auto& v : idx) v = (int)(g() % n);
    double acc = 0;
    auto t0 = std::chrono::steady_clock::now();
    for (int j = 0; j < m; j++) {
        double R[9], t[3];
        if (epnp_pixels(obj.data(), img.data(), &idx[5 * j], 5, K, R, t)) acc += R[0] + t[2];
    }
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / m;
    std::printf("epnp %.2f us per hypothesis (checksum %.6f)\n", us, acc);
    return 0;
}
