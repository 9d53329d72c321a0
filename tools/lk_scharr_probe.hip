// On-the-fly Scharr probe: what the derivative
// half of lk_multi_kernel's per-level setup costs when the (Ix | Iy) pairs are
// gathered from the stored derivative pyramid (the product), against computing
// them from the prev image staged in LDS once per feature and level.
//
// Both kernels do exactly the derivative work of the product's setup and nothing
// else: 4 features per wave, 16 lanes per feature, each lane 4 strips of 8 rows
// (7 output rows + the bilinear's next row), 4 levels; per output row the
// bilinear Ix and Iy sums of the four taps with the product's v_dot2 arithmetic,
// accumulated into per-lane checksums that both kernels must reproduce exactly.
//  G ("gather", the product): per strip row one 8-byte (Ix | Iy) pair load from
//    the padded derivative level + 4 v_perm regrouping (Ix(x) | Ix(x+1)) and
//    (Iy(x) | Iy(x+1)) for the v_dot2s.
//  F ("on the fly"): per feature and level the 24 x 24 prev-image region (the
//    22 x 22 derivative footprint + the Scharr halo) staged in LDS by dword loads,
//    Ix and Iy of the 22 x 22 pixels computed by the 16 lanes (3-10-3 stencil, x4
//    as stored) into two int16 planes, then each strip row reads its (x, x+1)
//    pairs from the planes (no perms: the plane layout is the dot2 layout).
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/lk_scharr_probe tools/lk_scharr_probe.hip
//   tools/lk_scharr_probe            (rocprofv3 --pmc SQ_INSTS_VALU ... for the mix)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

constexpr int PAD = 32, LEVELS = 4, FPW = 4, LPF = 16, K = 4, NR = 7;
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x2a4 __attribute__((ext_vector_type(2), aligned(4)));

struct Level {
    const uint8_t* img;   // interior origin, pitch ip
    const uint32_t* der;  // interior origin, pitch dp (elements): (Ix | Iy << 16) x4
    int w, h, ip, dp;
};
struct Pyr {
    Level lv[LEVELS];
};

__device__ __forceinline__ int sdot2(unsigned a, unsigned b, int c) {
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(s16x2, a), __builtin_bit_cast(s16x2, b), c, false);
}

// the lane's strips and the feature's window origin at a level (identical in both kernels)
__device__ __forceinline__ void strip_of(int l, int k, int& sc, int& sr, bool& real) {
    const int s = l + LPF * k;
    real = s < 63;
    const int v = real ? s : 0;
    sc = v % 21;
    sr = (v / 21) * NR;
}

__global__ __launch_bounds__(64, 3) void gather_kernel(const Pyr* __restrict__ pyr, const float2* __restrict__ pts, int n,
                                                       int* __restrict__ out) {
    const int lane = threadIdx.x, g = lane / LPF, l = lane % LPF;
    const int seq = blockIdx.y, pt = blockIdx.x * FPW + g;
    const Pyr& P = pyr[seq];
    const float2 p = pts[(size_t)seq * n + (pt < n ? pt : n - 1)];
    const unsigned W0 = 0x20001000u, W1 = 0x08000800u;  // fixed tap weights (any: both kernels equal)
    int acc = 0;
    for (int level = LEVELS - 1; level >= 0; level--) {
        const Level& L = P.lv[level];
        const float sc = __builtin_amdgcn_ldexpf(1.f, -level);
        const int sx = min(max((int)(p.x * sc) - 10, 0), L.w - 22), sy = min(max((int)(p.y * sc) - 10, 0), L.h - 22);
#pragma unroll
        for (int k = 0; k < K; k++) {
            int scol, srow;
            bool real;
            strip_of(l, k, scol, srow, real);
            const uint32_t* d = L.der + (size_t)(sy + srow) * L.dp + sx + scol;
            u32x2a4 D[NR + 1];
#pragma unroll
            for (int r = 0; r <= NR; r++) D[r] = *reinterpret_cast<const u32x2a4*>(d + (size_t)r * L.dp);
#pragma unroll
            for (int r = 0; r < NR; r++) {
                const unsigned X0 = __builtin_amdgcn_perm(D[r].y, D[r].x, 0x05040100u);
                const unsigned X1 = __builtin_amdgcn_perm(D[r + 1].y, D[r + 1].x, 0x05040100u);
                const unsigned Y0 = __builtin_amdgcn_perm(D[r].y, D[r].x, 0x07060302u);
                const unsigned Y1 = __builtin_amdgcn_perm(D[r + 1].y, D[r + 1].x, 0x07060302u);
                const int gx = sdot2(X0, W0, sdot2(X1, W1, 0)), gy = sdot2(Y0, W0, sdot2(Y1, W1, 0));
                acc += real ? (gx ^ (gy << 1)) : 0;
            }
        }
    }
    if (pt < n) atomicAdd(out + seq, acc);
}

// 24 x 24 staged region per feature (4-byte aligned start column: 28 columns read)
constexpr int SW = 28, SH = 24, DWD = 22;
__global__ __launch_bounds__(64, 3) void fly_kernel(const Pyr* __restrict__ pyr, const float2* __restrict__ pts, int n,
                                                    int* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint8_t S[FPW][SH][SW];
    __shared__ __attribute__((aligned(16))) int16_t GXp[FPW][DWD][DWD + 2], GYp[FPW][DWD][DWD + 2];
    const int lane = threadIdx.x, g = lane / LPF, l = lane % LPF;
    const int seq = blockIdx.y, pt = blockIdx.x * FPW + g;
    const Pyr& P = pyr[seq];
    const float2 p = pts[(size_t)seq * n + (pt < n ? pt : n - 1)];
    const unsigned W0 = 0x20001000u, W1 = 0x08000800u;
    int acc = 0;
    for (int level = LEVELS - 1; level >= 0; level--) {
        const Level& L = P.lv[level];
        const float sc = __builtin_amdgcn_ldexpf(1.f, -level);
        const int sx = min(max((int)(p.x * sc) - 10, 0), L.w - 22), sy = min(max((int)(p.y * sc) - 10, 0), L.h - 22);
        // stage rows sy-1 .. sy+22, columns from (sx-1) & ~3 (7 dwords per row), 16 lanes per feature
        const int xa = (sx - 1) & ~3, off = sx - 1 - xa;
        for (int k = l; k < SH * (SW / 4); k += LPF) {
            const int r = k / (SW / 4), q = k - r * (SW / 4);
            *reinterpret_cast<uint32_t*>(&S[g][r][4 * q]) =
                *reinterpret_cast<const uint32_t*>(L.img + (ptrdiff_t)(sy - 1 + r) * L.ip + xa + 4 * q);
        }
        __syncthreads();
        // Ix, Iy (x 4, as stored) of the 22 x 22 pixels: separable 3-10-3
        for (int k = l; k < DWD * DWD; k += LPF) {
            const int y = k / DWD, x = k - y * DWD;
            const uint8_t* c = &S[g][y + 1][off + x + 1];
            const int tl = c[-SW - 1], tm = c[-SW], tr = c[-SW + 1], ml = c[-1], mr = c[1], bl = c[SW - 1],
                      bm = c[SW], br = c[SW + 1];
            GXp[g][y][x] = (int16_t)(4 * ((3 * (tr + br) + 10 * mr) - (3 * (tl + bl) + 10 * ml)));
            GYp[g][y][x] = (int16_t)(4 * (3 * ((br - tr) + (bl - tl)) + 10 * (bm - tm)));
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < K; k++) {
            int scol, srow;
            bool real;
            strip_of(l, k, scol, srow, real);
            unsigned X[NR + 1], Y[NR + 1];
#pragma unroll
            for (int r = 0; r <= NR; r++) {
                const int rr = min(srow + r, DWD - 1);
                X[r] = (uint16_t)GXp[g][rr][scol] | ((unsigned)(uint16_t)GXp[g][rr][scol + 1] << 16);
                Y[r] = (uint16_t)GYp[g][rr][scol] | ((unsigned)(uint16_t)GYp[g][rr][scol + 1] << 16);
            }
#pragma unroll
            for (int r = 0; r < NR; r++) {
                const int gx = sdot2(X[r], W0, sdot2(X[r + 1], W1, 0)), gy = sdot2(Y[r], W0, sdot2(Y[r + 1], W1, 0));
                acc += real ? (gx ^ (gy << 1)) : 0;
            }
        }
        __syncthreads();
    }
    if (pt < n) atomicAdd(out + seq, acc);
}

int main() {
    const int S = 64, n = 2000, W = 1241, H = 376;
    std::mt19937 rng(7);
    std::vector<Pyr> hp(S);
    std::vector<void*> bufs;
    // random images (smoothed noise) and their exact x4 Scharr planes, levels 0..3, padded
    for (int s = 0; s < S; s++) {
        int w = W, h = H;
        for (int lv = 0; lv < LEVELS; lv++) {
            const int ip = (w + 2 * PAD + 63) & ~63, dp = (w + 2 * PAD + 15) & ~15;
            std::vector<uint8_t> img((size_t)ip * (h + 2 * PAD));
            for (auto& v : img) v = (uint8_t)(rng() & 0xFF);
            std::vector<uint32_t> der((size_t)dp * (h + 2 * PAD), 0);
            auto I = [&](int x, int y) { return (int)img[(size_t)(y + PAD) * ip + x + PAD]; };
            for (int y = -PAD + 1; y < h + PAD - 1; y++)
                for (int x = -PAD + 1; x < w + PAD - 1; x++) {
                    const int ix = (3 * (I(x + 1, y - 1) + I(x + 1, y + 1)) + 10 * I(x + 1, y)) -
                                   (3 * (I(x - 1, y - 1) + I(x - 1, y + 1)) + 10 * I(x - 1, y));
                    const int iy = 3 * ((I(x + 1, y + 1) - I(x + 1, y - 1)) + (I(x - 1, y + 1) - I(x - 1, y - 1))) +
                                   10 * (I(x, y + 1) - I(x, y - 1));
                    der[(size_t)(y + PAD) * dp + x + PAD] =
                        ((uint32_t)(uint16_t)(int16_t)(4 * iy) << 16) | (uint16_t)(int16_t)(4 * ix);
                }
            void *di, *dd;
            CK(hipMalloc(&di, img.size()));
            CK(hipMalloc(&dd, der.size() * 4));
            CK(hipMemcpy(di, img.data(), img.size(), hipMemcpyHostToDevice));
            CK(hipMemcpy(dd, der.data(), der.size() * 4, hipMemcpyHostToDevice));
            bufs.push_back(di);
            bufs.push_back(dd);
            hp[s].lv[lv] = {(const uint8_t*)di + (size_t)PAD * ip + PAD, (const uint32_t*)dd + (size_t)PAD * dp + PAD, w,
                            h, ip, dp};
            w = (w + 1) / 2;
            h = (h + 1) / 2;
        }
        if (s == 7) break;  // 8 distinct pyramids, shared round-robin (host time)
    }
    for (int s = 8; s < S; s++) hp[s] = hp[s % 8];
    std::vector<float2> pts((size_t)S * n);
    for (auto& q : pts) q = make_float2(20.f + (float)(rng() % (W - 40)), 20.f + (float)(rng() % (H - 40)));
    Pyr* dpyr;
    float2* dpts;
    int *og, *of;
    CK(hipMalloc(&dpyr, sizeof(Pyr) * S));
    CK(hipMalloc(&dpts, sizeof(float2) * pts.size()));
    CK(hipMalloc(&og, sizeof(int) * S));
    CK(hipMalloc(&of, sizeof(int) * S));
    CK(hipMemcpy(dpyr, hp.data(), sizeof(Pyr) * S, hipMemcpyHostToDevice));
    CK(hipMemcpy(dpts, pts.data(), sizeof(float2) * pts.size(), hipMemcpyHostToDevice));
    const dim3 grid((n + FPW - 1) / FPW, S);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](bool fly, int* o) {
        float best = 1e9f;
        for (int r = 0; r < 6; r++) {
            CK(hipMemset(o, 0, sizeof(int) * S));
            CK(hipEventRecord(e0, 0));
            if (fly)
                hipLaunchKernelGGL(fly_kernel, grid, dim3(64), 0, 0, dpyr, dpts, n, o);
            else
                hipLaunchKernelGGL(gather_kernel, grid, dim3(64), 0, 0, dpyr, dpts, n, o);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        return best * 1e3f;
    };
    const float tg = timeit(false, og), tf = timeit(true, of);
    std::vector<int> hg(S), hf(S);
    CK(hipMemcpy(hg.data(), og, sizeof(int) * S, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hf.data(), of, sizeof(int) * S, hipMemcpyDeviceToHost));
    int eq = 0;
    for (int s = 0; s < S; s++) eq += hg[s] == hf[s];
    std::printf("derivative part of LK setup, %d x %d features x %d levels (4 per wave):\n", S, n, LEVELS);
    std::printf("  gather (stored (Ix|Iy) pairs + perms): %8.1f us\n", tg);
    std::printf("  on the fly (LDS-staged I, 3-10-3):     %8.1f us\n", tf);
    std::printf("  checksums equal: %d / %d sequences\n", eq, S);
    return eq == S ? 0 : 1;
}
