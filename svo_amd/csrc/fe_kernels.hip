// Batched device-side glue of the tracking loop (R:src/tracking.cpp:240-269):
// post-LK compaction + map-point gather + RANSAC subset draws, outlier
// compaction + keyframe candidates, and the keyframe append (stereo filter,
// DLT triangulation, new map points). One launch covers every sequence of the
// batch (blockIdx = sequence), so a frame step costs the same number of
// launches for 1 or 512 sequences.
#include <algorithm>
#include <cstdlib>

#include "dlt.hpp"
#include "frontend.hpp"
#include "suffstats.hpp"

namespace svo {

namespace {

// Block size of the per-sequence post-LK / tail kernels: 4 waves, so that a block
// finds room on a CU while another slice's LK still occupies the GPU (a
// 1024-thread block waits for a whole CU to drain).
constexpr int kFeBlock = 256;
// The append / keyframe kernels triangulate every candidate with one thread (a
// ~2k-flop double Jacobi SVD, 128 VGPRs). 256 threads per sequence: a block of
// 1024 such threads needs a whole CU's registers and waited for one to drain
// beside FAST's pre-detection (keyframe_fused 91 us in the step); at 256 (one
// wave per SIMD) it starts at once (36 us in the step, 833.6 vs 874 us step
// period in the same trace); the usual ~50-100 candidates still take one pass.
constexpr int kAppendBlock = 256;
// post_lk: its chain of dependent passes (compaction chunks, map-point gathers)
// is latency-bound; 512 threads halve the chunks of a 2000-feature sequence
// against 256 and still fit beside FAST's 256-thread blocks
constexpr int kPostBlock = 512;

// Stable compaction of one sequence by a keep predicate, by a BS-thread block:
// keep(i) for i < n, kept entries load(i, x, y, mid) moved to their rank in
// xy_out / mid_out (in place allowed: every read of a chunk precedes its writes,
// and an entry never moves up). Returns the kept count.
template <int BS, typename Keep, typename Load>
__device__ __forceinline__ int block_compact_fn(int n, Keep keep, Load load, float* xy_out, int* mid_out, int* wsum,
                                                int* base_s) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (tid == 0) *base_s = 0;
    __syncthreads();
    for (int c0 = 0; c0 < n; c0 += BS) {
        const int i = c0 + tid;
        const bool k = i < n && keep(i);
        const unsigned long long bal = __ballot(k);
        if (lane == 0) wsum[wv] = __popcll(bal);
        __syncthreads();
        int off = *base_s;
        for (int q = 0; q < wv; q++) off += wsum[q];
        float x = 0.f, y = 0.f;
        int m = 0;
        if (k) load(i, x, y, m);
        __syncthreads();  // every read of this chunk before any write (in place allowed)
        if (k) {
            const int d = off + __popcll(bal & ((1ull << lane) - 1ull));
            xy_out[2 * d] = x;
            xy_out[2 * d + 1] = y;
            mid_out[d] = m;
        }
        if (tid == 0) {
            int tot = 0;
            for (int q = 0; q < BS / 64; q++) tot += wsum[q];
            *base_s += tot;
        }
        __syncthreads();
    }
    return *base_s;
}

// The same compaction for an out-of-place output with at most kCompactChunks
// chunks of BS: every chunk's keep test is issued up front (one bit per chunk per
// thread), the (chunk, wave) counts go to LDS, ONE wave turns them into exclusive
// offsets, then every kept entry is loaded and written -- two barriers instead of
// three per chunk, and the chunks' global reads in flight together instead of one
// chunk per barrier round (the post-LK / keyframe kernels sit on the step's
// critical path, where each round trip is latency). cnt: >= kCompactChunks * BS / 64
// ints of LDS.
constexpr int kCompactChunks = 32;
struct NoHook {
    __device__ void operator()(int) const {}
    __device__ void operator()(int, int) const {}
};
// after_scan(total): every thread, once the kept count is known (before the
// entries move); emit(d, m): per kept entry, after its move to rank d (mid m)
template <int BS, typename Keep, typename Load, typename AfterScan = NoHook, typename Emit = NoHook>
__device__ __forceinline__ int block_compact_batched(int n, Keep keep, Load load, float* xy_out, int* mid_out,
                                                     int* cnt, int* base_s, AfterScan after_scan = {},
                                                     Emit emit = {}) {
    constexpr int NW = BS / 64;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int nch = (n + BS - 1) / BS;
    unsigned flags = 0;
    for (int c = 0; c < nch; c++) {
        const int i = c * BS + tid;
        const bool k = i < n && keep(i);
        flags |= (unsigned)k << c;
        const unsigned long long bal = __ballot(k);
        if (lane == 0) cnt[c * NW + wv] = __popcll(bal);
    }
    __syncthreads();
    if (wv == 0) {
        // exclusive scan of the nch * NW counts (chunk-major, then wave), E per lane
        constexpr int EMAX = (kCompactChunks * NW + 63) / 64;
        const int ne = nch * NW, E = (ne + 63) / 64;
        int v[EMAX];
        int sum = 0;
#pragma unroll
        for (int e = 0; e < EMAX; e++) {
            const int j = lane * E + e;
            v[e] = e < E && j < ne ? cnt[j] : 0;
            sum += v[e];
        }
        int inc = sum;  // inclusive wave scan of the lane sums
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(inc, o);
            if (lane >= o) inc += t;
        }
        int run = inc - sum;
#pragma unroll
        for (int e = 0; e < EMAX; e++) {
            const int j = lane * E + e;
            if (e < E && j < ne) cnt[j] = run;
            run += v[e];
        }
        if (lane == 63) *base_s = inc;
    }
    __syncthreads();
    after_scan(*base_s);
    for (int c = 0; c < nch; c++) {
        const bool k = (flags >> c) & 1u;
        const unsigned long long bal = __ballot(k);
        if (k) {
            const int i = c * BS + tid;
            const int d = cnt[c * NW + wv] + __popcll(bal & ((1ull << lane) - 1ull));
            float x, y;
            int m;
            load(i, x, y, m);
            xy_out[2 * d] = x;
            xy_out[2 * d + 1] = y;
            mid_out[d] = m;
            emit(d, m);
        }
    }
    const int total = *base_s;
    __syncthreads();  // cnt / base_s reusable
    return total;
}

// in place (xy_in == xy_out) or beyond kCompactChunks chunks: the per-chunk form
template <int BS, typename Keep>
__device__ __forceinline__ int block_compact(int n, Keep keep, const float* xy_in, const int* mid_in, float* xy_out,
                                             int* mid_out, int* wsum, int* base_s, int* cnt = nullptr) {
    auto load = [&](int i, float& x, float& y, int& m) {
        x = xy_in[2 * i];
        y = xy_in[2 * i + 1];
        m = mid_in[i];
    };
    if (cnt && xy_in != xy_out && n <= kCompactChunks * BS)
        return block_compact_batched<BS>(n, keep, load, xy_out, mid_out, cnt, base_s);
    return block_compact_fn<BS>(n, keep, load, xy_out, mid_out, wsum, base_s);
}

// x mod n for 32-bit x, n >= 1, with a precomputed m = floor((2^32 - 1) / n)
__device__ __forceinline__ unsigned fast_mod(unsigned x, unsigned n, unsigned m) {
    const unsigned q = __umulhi(x, m);
    unsigned r = x - q * n;
    while (r >= n) r -= n;
    return r;
}

// Pending keyframe map points of sequence s to the world frame:
// p_w = R p + t, the SE3d action (svo::SE3d::operator*, Sophus' T * p),
// evaluated operation by operation (-ffp-contract=off).
__device__ __forceinline__ void finalize_body(const PendingMap& P, int s) {
    const int n = P.pend_n[s];
    if (n <= 0) return;
    const double* T = P.pose + 12 * (size_t)s;
    double* X = P.map + 3 * ((size_t)s * P.map_cap + P.pend0[s]);
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const double x = X[3 * i], y = X[3 * i + 1], z = X[3 * i + 2];
        X[3 * i] = T[0] * x + T[1] * y + T[2] * z + T[9];
        X[3 * i + 1] = T[3] * x + T[4] * y + T[5] * z + T[10];
        X[3 * i + 2] = T[6] * x + T[7] * y + T[8] * z + T[11];
    }
    __syncthreads();
    if (threadIdx.x == 0) P.pend_n[s] = 0;
}

__global__ __launch_bounds__(kFeBlock) void finalize_map_kernel(PendingMap P) { finalize_body(P, blockIdx.x); }

// RANSAC subset draws of sequence s (OpenCV's MWC RNG; they depend only on n),
// one thread, the subset being drawn in registers (its duplicate tests were a
// chain of dependent LDS reads: ~260 per sequence on the critical path)
__device__ __forceinline__ void ransac_draws(int n, int nh, int* idx) {
    const unsigned m = 0xFFFFFFFFu / (unsigned)n;
    uint64_t sr = ~0ull;
    for (int j = 0; j < nh; j++) {
        int cur[5];
#pragma unroll
        for (int i = 0; i < 5; i++) {
            int v;
            bool dup;
            do {
                sr = (uint64_t)(uint32_t)sr * 4164903690u + (uint32_t)(sr >> 32);
                v = (int)fast_mod((uint32_t)sr, (unsigned)n, m);
                dup = false;
#pragma unroll
                for (int k = 0; k < i; k++) dup |= cur[k] == v;
            } while (dup);
            cur[i] = v;
        }
#pragma unroll
        for (int i = 0; i < 5; i++) idx[5 * j + i] = cur[i];
    }
}

__global__ __launch_bounds__(kPostBlock) void post_lk_kernel(PostLkBatch B) {
    const int s = blockIdx.x;
    const size_t o = (size_t)s * B.cap;
    __shared__ int wsum[kPostBlock / 64];
    __shared__ int base_s;
    __shared__ unsigned long long it_s;
    __shared__ int idx[5 * 64];
    __shared__ int cnt[kCompactChunks * kPostBlock / 64];
    const int tid = threadIdx.x, lane = tid & 63;
    if (tid == 0) it_s = 0;
    finalize_body(B.pm, s);  // (ends with a barrier when it has work; it_s is set before the next one)
    const int n_in = B.n_in[s];
    const uint8_t* __restrict__ st = B.status + o;
    long long it = 0;
    for (int i = tid; i < n_in; i += kPostBlock) it += B.iters[o + i];
    const double* __restrict__ map = B.pm.map + 3 * (size_t)s * B.pm.map_cap;
    const bool nh_ok = B.nh > 0 && B.nh <= 64;
    int n;
    if (n_in <= kCompactChunks * kPostBlock) {
        // the status compaction moves each kept entry and gathers its map point
        // (one dependent round trip less than a separate gather pass); thread 0
        // replays the RANSAC draws while the block moves the entries
        const float* __restrict__ xy_in = B.xy_in + 2 * o;
        const int* __restrict__ mid_in = B.mid_in + o;
        float* __restrict__ obj = B.obj + 3 * o;
        n = block_compact_batched<kPostBlock>(
            n_in, [&](int i) { return st[i] != 0; },
            [&](int i, float& x, float& y, int& m) {
                x = xy_in[2 * i];
                y = xy_in[2 * i + 1];
                m = mid_in[i];
            },
            B.xy_out + 2 * o, B.mid_out + o, cnt, &base_s,
            [&](int total) {
                if (tid == 0 && total > 5 && nh_ok) ransac_draws(total, B.nh, idx);
            },
            [&](int d, int m) {
                const double* X = map + 3 * (size_t)m;
                obj[3 * d] = (float)X[0];
                obj[3 * d + 1] = (float)X[1];
                obj[3 * d + 2] = (float)X[2];
            });
    } else {
        n = block_compact<kPostBlock>(n_in, [&](int i) { return st[i] != 0; }, B.xy_in + 2 * o, B.mid_in + o,
                                      B.xy_out + 2 * o, B.mid_out + o, wsum, &base_s);
        if (tid == 0 && n > 5 && nh_ok) ransac_draws(n, B.nh, idx);
        const int* __restrict__ mid = B.mid_out + o;
        for (int i = tid; i < n; i += kPostBlock) {
            const double* X = map + 3 * (size_t)mid[i];
            B.obj[3 * (o + i)] = (float)X[0];
            B.obj[3 * (o + i) + 1] = (float)X[1];
            B.obj[3 * (o + i) + 2] = (float)X[2];
        }
    }
    for (int off = 32; off > 0; off >>= 1) it += __shfl_xor(it, off);
    if (lane == 0) atomicAdd(&it_s, (unsigned long long)it);
    const bool draws = n > 5 && nh_ok;
    __syncthreads();
    if (tid == 0) {
        B.n_out[s] = n;
        B.h_n[s] = n;
        B.h_iters[s] = (long long)it_s;
    }
    if (draws) {
        // the subsets' points from the compacted arrays just written (obj holds
        // (float) of the map point, as the separate gather did)
        const float* __restrict__ xy = B.xy_out + 2 * o;
        const float* __restrict__ obj = B.obj + 3 * o;
        float* __restrict__ dst = B.h_samp + (size_t)25 * B.nh * s;
        for (int k = tid; k < 5 * B.nh; k += kPostBlock) {
            const int j = k / 5, i = k - 5 * j, p = idx[k];
            float* h = dst + 25 * j;
            h[3 * i] = obj[3 * p];
            h[3 * i + 1] = obj[3 * p + 1];
            h[3 * i + 2] = obj[3 * p + 2];
            h[15 + 2 * i] = xy[2 * p];
            h[15 + 2 * i + 1] = xy[2 * p + 1];
        }
    }
}

// Outlier compaction by the inlier bits + the keyframe's take (tail_kernel's
// body, BS threads); copy_cand: also copy the candidates to st_xy (the stereo
// LK's input; a speculative prep already wrote them otherwise).
template <int BS>
__device__ __forceinline__ void tail_body(const TailBatch& T, int s, bool copy_cand, int* wsum, int* base_s,
                                          int* n_kept, int* take_out, int* cnt, double (*spart)[kSuffStats]) {
    const size_t o = (size_t)s * T.cap;
    const uint32_t* __restrict__ bits = T.bits + (size_t)s * T.words_cap;
    if (T.stats_out) {
        static_assert(BS == kSuffThreads, "the statistics' reduction order is that of 256 threads");
        suffstats_block(T.stats_obj + 3 * o, T.xy_in + 2 * o, T.n_in[s], bits, T.ifx, T.ify, T.cx, T.cy, spart,
                        T.stats_out + kSuffStats * (size_t)s);
    }
    const int n = block_compact<BS>(
        T.n_in[s], [&](int i) { return ((bits[i >> 5] >> (i & 31)) & 1u) != 0; }, T.xy_in + 2 * o, T.mid_in + o,
        T.xy_out + 2 * o, T.mid_out + o, wsum, base_s, cnt);
    // new-feature candidates of the keyframe: the first `take` masked corners
    int take = min(max(T.n_target[s] - n, 0), min(T.cand_n[s], T.cand_cap));
    take = min(take, T.cap - n);
    take = max(min(take, T.map_cap - T.map_n[s]), 0);
    if (copy_cand) {
        const float* c = T.cand + (size_t)T.cand_elem * ((size_t)s * T.cand_cap);
        for (int j = threadIdx.x; j < take; j += BS) {
            T.st_xy[2 * (o + j)] = c[(size_t)T.cand_elem * j];
            T.st_xy[2 * (o + j) + 1] = c[(size_t)T.cand_elem * j + 1];
        }
    }
    if (threadIdx.x == 0) {
        T.n_out[s] = n;
        T.st_n[s] = take;
        if (T.h_over) T.h_over[s] = max(T.cand_n[s] - take, 0);
    }
    *n_kept = n;
    *take_out = take;
}

__global__ __launch_bounds__(kFeBlock) void tail_kernel(TailBatch T) {
    __shared__ int wsum[kFeBlock / 64];
    __shared__ int base_s;
    __shared__ int cnt[kCompactChunks * kFeBlock / 64];
    __shared__ double spart[kSuffThreads / 64][kSuffStats];
    int n, take;
    tail_body<kFeBlock>(T, blockIdx.x, true, wsum, &base_s, &n, &take, cnt, spart);
}

// findLeftFeaturesInRight's filter + triangulateNewMapPoints for one stereo match:
// keep = status && |yR - yL| < y_threshold (float) && p.z > 0 (x3: the point in the
// left camera frame)
__device__ __forceinline__ bool stereo_point(const float (&P)[24], float y_threshold, bool status, float xl, float yl,
                                             float xr, float yr, float (&x3)[3]) {
    bool keep = status && fabsf(yr - yl) < y_threshold;
    if (keep) {
        float h[4];
        dlt_point(P, xl, yl, xr, yr, h);
        dlt_euclidean(h, x3);
        keep = x3[2] > 0.f;  // triangulateNewMapPoints: p_w.z > 0
    }
    return keep;
}

// The append of the stereo matches of st_xy[0, take) of sequence s, n0 features
// already kept: the filter and the points come from stereo_tri_kernel (A.st_X).
template <int BS>
__device__ __forceinline__ void append_body(const AppendBatch& A, int s, int n0, int take, int* wsum, int* base_sp) {
    int& base_s = *base_sp;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const size_t o = (size_t)s * A.cap;
    const int m0 = A.map_n[s];
    __syncthreads();  // base_s / wsum reuse after the caller's own block work
    if (tid == 0) base_s = 0;
    __syncthreads();
    for (int c0 = 0; c0 < take; c0 += BS) {
        const int j = c0 + tid;
        bool keep = false;
        float xl = 0.f, yl = 0.f, x3[3] = {0.f, 0.f, 0.f};
        if (j < take) {
            xl = A.st_xy[2 * (o + j)];
            yl = A.st_xy[2 * (o + j) + 1];
            const float4 v = A.st_X[o + j];
            x3[0] = v.x;
            x3[1] = v.y;
            x3[2] = v.z;
            keep = v.w != 0.f;
        }
        const unsigned long long bal = __ballot(keep);
        if (lane == 0) wsum[wv] = __popcll(bal);
        __syncthreads();
        int off = base_s;
        for (int q = 0; q < wv; q++) off += wsum[q];
        if (keep) {
            const int d = off + __popcll(bal & ((1ull << lane) - 1ull));
            const size_t f = o + n0 + d;
            A.xy[2 * f] = xl;
            A.xy[2 * f + 1] = yl;
            A.mid[f] = m0 + d;
            // left camera frame (double of the float point, as Eigen::Vector3d{p_w.x,
            // p_w.y, p_w.z}); the pose is applied once known (PendingMap)
            double* X = A.map + 3 * ((size_t)s * A.map_cap + m0 + d);
            X[0] = (double)x3[0];
            X[1] = (double)x3[1];
            X[2] = (double)x3[2];
        }
        __syncthreads();
        if (tid == 0) {
            int tot = 0;
            for (int q = 0; q < BS / 64; q++) tot += wsum[q];
            base_s += tot;
        }
        __syncthreads();
    }
    if (tid == 0) {
        const int added = base_s;
        A.n[s] = n0 + added;
        A.map_n[s] = m0 + added;
        A.pend0[s] = m0;
        A.pend_n[s] = added;
        if (A.added) A.added[s] = added;
        if (A.h_n) A.h_n[s] = n0 + added;
        if (A.h_added) A.h_added[s] = added;
    }
}

template <int BS>
__global__ __launch_bounds__(BS) void append_kernel(AppendBatch A) {
    __shared__ int wsum[BS / 64];
    __shared__ int base_s;
    const int s = blockIdx.x;
    append_body<BS>(A, s, A.n[s], A.st_n[s], wsum, &base_s);
}

template <int BS>
__global__ __launch_bounds__(BS) void keyframe_fused_kernel(TailBatch T, AppendBatch A) {
    __shared__ int wsum[BS / 64];
    __shared__ int base_s;
    __shared__ int cnt[kCompactChunks * BS / 64];
    __shared__ double spart[kSuffThreads / 64][kSuffStats];
    const int s = blockIdx.x;
    int n, take;
    tail_body<BS>(T, s, false, wsum, &base_s, &n, &take, cnt, spart);
    append_body<BS>(A, s, n, take, wsum, &base_s);
}

// one 64-lane wave per block: the candidates of a sequence are ~ the margin (tens),
// and a lone wave fits beside LK's three per SIMD where a 256-thread block waits
__global__ __launch_bounds__(64, 6) void stereo_tri_kernel(StereoTriBatch B) {
    const int s = blockIdx.y;
    const int n = B.spec_n[s];
    const size_t o = (size_t)s * B.cap;
    for (int j = blockIdx.x * 64 + threadIdx.x; j < n; j += gridDim.x * 64) {
        const float xl = B.st_xy[2 * (o + j)], yl = B.st_xy[2 * (o + j) + 1];
        float x3[3] = {0.f, 0.f, 0.f};
        // the projection matrices converted per point: hoisted out of the loop, their
        // 24 doubles stayed live through the solve (157 VGPRs)
        float P[24];
#pragma unroll
        for (int k = 0; k < 24; k++) {
            P[k] = B.P[k];
            asm volatile("" : "+s"(P[k]));
        }
        const bool keep = stereo_point(P, B.y_threshold, B.st_status[o + j] != 0, xl, yl, B.st_next[2 * (o + j)],
                                       B.st_next[2 * (o + j) + 1], x3);
        B.st_X[o + j] = make_float4(x3[0], x3[1], x3[2], keep ? 1.f : 0.f);
    }
}

__global__ __launch_bounds__(kFeBlock) void stereo_prep_kernel(StereoPrepBatch B) {
    const int s = blockIdx.x;
    int spec = min(max(B.n_target[s] - B.n_tracked[s] + B.margin, 0), min(B.cand_n[s], B.cand_cap));
    spec = max(min(min(spec, B.cap), B.map_cap - B.map_n[s]), 0);
    const float* c = B.cand + (size_t)B.cand_elem * ((size_t)s * B.cand_cap);
    float* dst = B.st_xy + 2 * (size_t)s * B.cap;
    for (int j = threadIdx.x; j < spec; j += kFeBlock) {
        dst[2 * j] = c[(size_t)B.cand_elem * j];
        dst[2 * j + 1] = c[(size_t)B.cand_elem * j + 1];
    }
    if (threadIdx.x == 0) B.spec_n[s] = spec;
}

}  // namespace

hipError_t launch_post_lk(const PostLkBatch& b, int nseq, hipStream_t st) {
    if (b.nh > 64) return hipErrorInvalidValue;
    hipLaunchKernelGGL(post_lk_kernel, dim3(nseq), dim3(kPostBlock), 0, st, b);
    return hipGetLastError();
}

hipError_t launch_finalize_map(const PendingMap& pm, int nseq, hipStream_t st) {
    hipLaunchKernelGGL(finalize_map_kernel, dim3(nseq), dim3(kFeBlock), 0, st, pm);
    return hipGetLastError();
}

hipError_t launch_tail(const TailBatch& tb, int nseq, hipStream_t st) {
    hipLaunchKernelGGL(tail_kernel, dim3(nseq), dim3(kFeBlock), 0, st, tb);
    return hipGetLastError();
}

hipError_t launch_append(const AppendBatch& b, int nseq, hipStream_t st) {
    hipLaunchKernelGGL(append_kernel<kAppendBlock>, dim3(nseq), dim3(kAppendBlock), 0, st, b);
    return hipGetLastError();
}

hipError_t launch_keyframe_fused(const TailBatch& tb, const AppendBatch& ab, int nseq, hipStream_t st) {
    hipLaunchKernelGGL(keyframe_fused_kernel<kAppendBlock>, dim3(nseq), dim3(kAppendBlock), 0, st, tb, ab);
    return hipGetLastError();
}

hipError_t launch_stereo_tri(const StereoTriBatch& b, int nseq, int max_n, hipStream_t st) {
    const int gx = std::max(1, std::min((max_n + 63) / 64, 256));
    hipLaunchKernelGGL(stereo_tri_kernel, dim3(gx, nseq), dim3(64), 0, st, b);
    return hipGetLastError();
}

hipError_t launch_stereo_prep(const StereoPrepBatch& b, int nseq, hipStream_t st) {
    hipLaunchKernelGGL(stereo_prep_kernel, dim3(nseq), dim3(kFeBlock), 0, st, b);
    return hipGetLastError();
}

}  // namespace svo
