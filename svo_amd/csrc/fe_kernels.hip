// Batched device-side glue of the tracking loop (R:src/tracking.cpp:240-269):
// stable compaction of tracked / inlier features, map-point gather for PnP,
// and keyframe top-up with new map points. One launch covers every sequence of
// the batch (blockIdx = sequence), so a frame step costs the same number of
// launches for 1 or 512 sequences.
#include "frontend.hpp"

namespace svo {

namespace {

// Stable order-preserving compaction of features [0, n_in[s]) of sequence s
// (one 1024-thread block per sequence). keep = status[i] (u8) or bit i of bits.
__global__ __launch_bounds__(1024) void compact_kernel(CompactBatch B) {
    const int s = blockIdx.x;
    const int n = B.n_in[s];
    const size_t o = (size_t)s * B.cap;
    __shared__ int wsum[16];
    __shared__ int base_s;
    __shared__ long long it_s;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (tid == 0) {
        base_s = 0;
        it_s = 0;
    }
    __syncthreads();
    long long it = 0;
    for (int c0 = 0; c0 < n; c0 += 1024) {
        const int i = c0 + tid;
        bool keep = false;
        if (i < n) {
            keep = B.status ? B.status[o + i] != 0 : ((B.bits[(size_t)s * B.words_cap + (i >> 5)] >> (i & 31)) & 1u);
            if (B.iters) it += B.iters[o + i];
        }
        const unsigned long long bal = __ballot(keep);
        if (lane == 0) wsum[wv] = __popcll(bal);
        __syncthreads();
        int off = base_s;
        for (int k = 0; k < wv; k++) off += wsum[k];
        if (keep) {
            const int d = off + __popcll(bal & ((1ull << lane) - 1ull));
            B.xy_out[2 * (o + d)] = B.xy_in[2 * (o + i)];
            B.xy_out[2 * (o + d) + 1] = B.xy_in[2 * (o + i) + 1];
            B.mid_out[o + d] = B.mid_in[o + i];
        }
        __syncthreads();
        if (tid == 0) {
            int tot = 0;
            for (int k = 0; k < 16; k++) tot += wsum[k];
            base_s += tot;
        }
        __syncthreads();
    }
    if (B.iters) {
        for (int off = 32; off > 0; off >>= 1) it += __shfl_xor(it, off);
        if (lane == 0) atomicAdd((unsigned long long*)&it_s, (unsigned long long)it);
    }
    __syncthreads();
    if (tid == 0) {
        B.n_out[s] = base_s;
        if (B.iters_sum) B.iters_sum[s] = it_s;
    }
}

// obj[s][i] = (float) map[s][mid[s][i]]  (solvePnPRansac converts Point3d to CV_32F)
__global__ __launch_bounds__(256) void gather_kernel(const int* __restrict__ n, const int* __restrict__ mid,
                                                     const double* __restrict__ map, int cap, int map_cap,
                                                     float* __restrict__ obj) {
    const int s = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n[s]) return;
    const size_t o = (size_t)s * cap + i;
    const double* X = map + 3 * ((size_t)s * map_cap + mid[o]);
    obj[3 * o] = (float)X[0];
    obj[3 * o + 1] = (float)X[1];
    obj[3 * o + 2] = (float)X[2];
}

// Keyframe top-up: append the first (n_target - n) candidates (bucketed FAST
// output, raster/bucket order) as new features with new map points. The map
// point stands in for triangulateNewMapPoints (R:src/tracking.cpp:120-152):
// the synthetic scene gives the depth of every pixel ray (scene.py).
__global__ __launch_bounds__(256) void append_kernel(AppendBatch B) {
    const int s = blockIdx.x;
    __shared__ int take_s, n0_s, m0_s;
    if (threadIdx.x == 0) {
        const int n0 = B.n[s];
        const int cand = min(B.cand_n[s], B.cand_cap);
        int take = min(max(B.n_target - n0, 0), cand);
        take = min(take, B.cap - n0);
        take = min(take, B.map_cap - B.map_n[s]);
        take = max(take, 0);
        take_s = take;
        n0_s = n0;
        m0_s = B.map_n[s];
    }
    __syncthreads();
    const int take = take_s, n0 = n0_s, m0 = m0_s;
    const double* R = B.rot + 9 * (size_t)s;  // world -> camera of this frame
    const double fx = B.K[0], fy = B.K[4], cx = B.K[2], cy = B.K[5];
    const double seed = (double)B.depth_seed[s];
    for (int j = threadIdx.x; j < take; j += 256) {
        const float* c = B.cand + (size_t)B.cand_elem * ((size_t)s * B.cand_cap + j);
        const float x = c[0], y = c[1];
        const size_t o = (size_t)s * B.cap + n0 + j;
        B.xy[2 * o] = x;
        B.xy[2 * o + 1] = y;
        B.mid[o] = m0 + j;
        const double rx = (x - cx) / fx, ry = (y - cy) / fy;
        const double wx = R[0] * rx + R[3] * ry + R[6];
        const double wy = R[1] * rx + R[4] * ry + R[7];
        const double wz = R[2] * rx + R[5] * ry + R[8];
        const double cu = fx * wx / wz + cx, cv = fy * wy / wz + cy;
        const double rho = 12.0 + 5.0 * sin(cu / 97.0 + seed) + 4.0 * cos(cv / 61.0 - 0.5 * seed);
        double* X = B.map + 3 * ((size_t)s * B.map_cap + m0 + j);
        X[0] = wx / wz * rho;
        X[1] = wy / wz * rho;
        X[2] = rho;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        B.n[s] = n0 + take;
        B.map_n[s] = m0 + take;
        if (B.added) B.added[s] = take;
    }
}

// RANSAC subset prefetch: the draws of RANSACPointSetRegistrator::getSubset
// (cv::RNG(-1) MWC, uniform(0, n) = next() % n, redraw duplicates) depend only
// on n, so the device replays them for the first `nh` hypotheses of every
// sequence and gathers the drawn points: per hypothesis obj[5][3] then
// img[5][2] floats. One block per sequence: lane 0 draws, the block gathers.
__global__ __launch_bounds__(256) void ransac_sample_kernel(const int* __restrict__ counts, const float* __restrict__ obj,
                                                            const float* __restrict__ img, int cap, int nh,
                                                            float* __restrict__ samp) {
    __shared__ int idx[5 * 64];
    const int s = blockIdx.x;
    const int n = counts[s];
    if (n <= 5 || nh > 64) return;  // n <= 5: solved directly from all points, on the host
    if (threadIdx.x == 0) {
        uint64_t st = ~0ull;
        for (int j = 0; j < nh; j++)
            for (int i = 0; i < 5; i++) {
                int v;
                bool dup;
                do {
                    st = (uint64_t)(uint32_t)st * 4164903690u + (uint32_t)(st >> 32);
                    v = (int)((uint32_t)st % (unsigned)n);
                    dup = false;
                    for (int k = 0; k < i; k++) dup |= idx[5 * j + k] == v;
                } while (dup);
                idx[5 * j + i] = v;
            }
    }
    __syncthreads();
    const float* o = obj + (size_t)3 * cap * s;
    const float* im = img + (size_t)2 * cap * s;
    float* dst = samp + (size_t)25 * nh * s;
    for (int k = threadIdx.x; k < 5 * nh; k += blockDim.x) {
        const int j = k / 5, i = k - 5 * j, p = idx[k];
        float* h = dst + 25 * j;
        h[3 * i] = o[3 * p];
        h[3 * i + 1] = o[3 * p + 1];
        h[3 * i + 2] = o[3 * p + 2];
        h[15 + 2 * i] = im[2 * p];
        h[15 + 2 * i + 1] = im[2 * p + 1];
    }
}

// Block size of the per-sequence post-LK / tail kernels: 4 waves, so that a block
// finds room on a CU while another slice's LK still occupies the GPU (a
// 1024-thread block waits for a whole CU to drain).
constexpr int kFeBlock = 256;

// Stable compaction of one sequence by a keep predicate, by a kFeBlock-thread
// block: keep(i) for i < n, kept entries of xy / mid moved to their rank.
template <bool SC1 = false, typename Keep>
__device__ __forceinline__ int block_compact(int n, Keep keep, const float* __restrict__ xy_in,
                                             const int* __restrict__ mid_in, float* __restrict__ xy_out,
                                             int* __restrict__ mid_out, int* wsum, int* base_s) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (tid == 0) *base_s = 0;
    __syncthreads();
    for (int c0 = 0; c0 < n; c0 += kFeBlock) {
        const int i = c0 + tid;
        const bool k = i < n && keep(i);
        const unsigned long long bal = __ballot(k);
        if (lane == 0) wsum[wv] = __popcll(bal);
        __syncthreads();
        int off = *base_s;
        for (int q = 0; q < wv; q++) off += wsum[q];
        float x = 0.f, y = 0.f;
        int m = 0;
        if (k) {
            if (SC1) {  // xy_in = streamed LK records {x, tag}, {y, tag} (sc1 loads)
                const unsigned long long* r = reinterpret_cast<const unsigned long long*>(xy_in + 4 * i);
                x = __uint_as_float((unsigned)__hip_atomic_load(r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                y = __uint_as_float((unsigned)__hip_atomic_load(r + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            } else {
                x = xy_in[2 * i];
                y = xy_in[2 * i + 1];
            }
            m = mid_in[i];
        }
        __syncthreads();  // every read of this chunk before any write (in place allowed)
        if (k) {
            const int d = off + __popcll(bal & ((1ull << lane) - 1ull));
            xy_out[2 * d] = x;
            xy_out[2 * d + 1] = y;
            mid_out[d] = m;
        }
        if (tid == 0) {
            int tot = 0;
            for (int q = 0; q < kFeBlock / 64; q++) tot += wsum[q];
            *base_s += tot;
        }
        __syncthreads();
    }
    return *base_s;
}

// x mod n for 32-bit x, n >= 1, with a precomputed m = floor((2^32 - 1) / n)
__device__ __forceinline__ unsigned fast_mod(unsigned x, unsigned n, unsigned m) {
    const unsigned q = __umulhi(x, m);
    unsigned r = x - q * n;
    while (r >= n) r -= n;
    return r;
}

__global__ __launch_bounds__(kFeBlock) void post_lk_kernel(PostLkBatch B) {
    const int s = blockIdx.x;
    const size_t o = (size_t)s * B.cap;
    __shared__ int wsum[kFeBlock / 64];
    __shared__ int base_s;
    __shared__ unsigned long long it_s;
    __shared__ int idx[5 * 64];
    const int tid = threadIdx.x, lane = tid & 63;
    if (tid == 0) it_s = 0;
    const int n_in = B.n_in[s];
    const uint8_t* __restrict__ st = B.status + o;
    long long it = 0;
    int n;
    if (B.rec) {
        // streamed: wait for this sequence's LK records (bounded: a lost producer
        // ends the wait after ~1 s and raises h_fail instead of hanging the GPU)
        const unsigned* __restrict__ rc = B.rec + 4 * o;
        const unsigned stamp = (unsigned)B.lk_stamp;
        auto ld8 = [&](int i, int h) {
            return __hip_atomic_load(reinterpret_cast<const unsigned long long*>(rc + 4 * i + 2 * h), __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
        };
        auto tagged = [&](int i) {
            return (unsigned)(ld8(i, 0) >> 56) == stamp && (unsigned)(ld8(i, 1) >> 32) == stamp;
        };
        if (tid < 64) {
            int spins = 0;
            bool fail = false;
            // cheap probe first: the last feature (its block is dispatched last)
            while (n_in > 0 && !fail && (unsigned)(ld8(n_in - 1, 1) >> 32) != stamp) {
                __builtin_amdgcn_s_sleep(32);
                fail = ++spins > (1 << 20);
            }
            for (;;) {
                bool ok = true;
                for (int i = tid; i < n_in; i += 64) ok &= tagged(i);
                if (__all(ok) || fail) break;
                __builtin_amdgcn_s_sleep(4);
                fail = ++spins > (1 << 20);
            }
            if (fail && tid == 0) {
                __hip_atomic_store(B.h_fail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                it_s = ~0ull;  // tells the block to stop (it_s is re-zeroed below otherwise unused so far)
            }
        }
        __syncthreads();
        if (it_s == ~0ull) return;  // LK never ran beside us (kernels serialised): the host re-runs us after LK
        for (int i = tid; i < n_in; i += kFeBlock) it += (long long)((unsigned)(ld8(i, 0) >> 32) & ((1u << 23) - 1u));
        n = block_compact<true>(
            n_in, [&](int i) { return ((ld8(i, 0) >> 55) & 1ull) != 0; }, reinterpret_cast<const float*>(rc),
            B.mid_in + o, B.xy_out + 2 * o, B.mid_out + o, wsum, &base_s);
    } else {
        for (int i = tid; i < n_in; i += kFeBlock) it += B.iters[o + i];
        n = block_compact(n_in, [&](int i) { return st[i] != 0; }, B.xy_in + 2 * o, B.mid_in + o, B.xy_out + 2 * o,
                          B.mid_out + o, wsum, &base_s);
    }
    for (int off = 32; off > 0; off >>= 1) it += __shfl_xor(it, off);
    if (lane == 0) atomicAdd(&it_s, (unsigned long long)it);
    // wave 0 lane 0 replays the RANSAC draws (they depend only on n) while the
    // block gathers the map points
    const bool draws = n > 5 && B.nh > 0 && B.nh <= 64;
    if (tid == 0 && draws) {
        const unsigned m = 0xFFFFFFFFu / (unsigned)n;
        uint64_t sr = ~0ull;
        for (int j = 0; j < B.nh; j++)
            for (int i = 0; i < 5; i++) {
                int v;
                bool dup;
                do {
                    sr = (uint64_t)(uint32_t)sr * 4164903690u + (uint32_t)(sr >> 32);
                    v = (int)fast_mod((uint32_t)sr, (unsigned)n, m);
                    dup = false;
                    for (int k = 0; k < i; k++) dup |= idx[5 * j + k] == v;
                } while (dup);
                idx[5 * j + i] = v;
            }
    }
    const int* __restrict__ mid = B.mid_out + o;
    const double* __restrict__ map = B.map + 3 * (size_t)s * B.map_cap;
    for (int i = tid; i < n; i += kFeBlock) {
        const double* X = map + 3 * (size_t)mid[i];
        B.obj[3 * (o + i)] = (float)X[0];
        B.obj[3 * (o + i) + 1] = (float)X[1];
        B.obj[3 * (o + i) + 2] = (float)X[2];
    }
    __syncthreads();
    if (tid == 0) {
        B.n_out[s] = n;
        B.h_n[s] = n;
        B.h_iters[s] = (long long)it_s;
    }
    if (draws) {
        const float* __restrict__ xy = B.xy_out + 2 * o;
        float* __restrict__ dst = B.h_samp + (size_t)25 * B.nh * s;
        for (int k = tid; k < 5 * B.nh; k += kFeBlock) {
            const int j = k / 5, i = k - 5 * j, p = idx[k];
            const double* X = map + 3 * (size_t)mid[p];
            float* h = dst + 25 * j;
            h[3 * i] = (float)X[0];
            h[3 * i + 1] = (float)X[1];
            h[3 * i + 2] = (float)X[2];
            h[15 + 2 * i] = xy[2 * p];
            h[15 + 2 * i + 1] = xy[2 * p + 1];
        }
    }
    if (B.h_ready) {
        // publish to the host: every wave's stores drained, then one system release
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(B.h_ready + s, B.stamp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// keyframe top-up of one sequence by its block (append_kernel's body)
__device__ __forceinline__ void append_body(const AppendBatch& B, int s) {
    __shared__ int take_s, n0_s, m0_s;
    if (threadIdx.x == 0) {
        const int n0 = B.n[s];
        const int cand = min(B.cand_n[s], B.cand_cap);
        int take = min(max(B.n_target - n0, 0), cand);
        take = min(take, B.cap - n0);
        take = min(take, B.map_cap - B.map_n[s]);
        take = max(take, 0);
        take_s = take;
        n0_s = n0;
        m0_s = B.map_n[s];
    }
    __syncthreads();
    const int take = take_s, n0 = n0_s, m0 = m0_s;
    const double* R = B.rot + 9 * (size_t)s;  // world -> camera of this frame
    const double fx = B.K[0], fy = B.K[4], cx = B.K[2], cy = B.K[5];
    const double seed = (double)B.depth_seed[s];
    for (int j = threadIdx.x; j < take; j += blockDim.x) {
        const float* c = B.cand + (size_t)B.cand_elem * ((size_t)s * B.cand_cap + j);
        const float x = c[0], y = c[1];
        const size_t o = (size_t)s * B.cap + n0 + j;
        B.xy[2 * o] = x;
        B.xy[2 * o + 1] = y;
        B.mid[o] = m0 + j;
        const double rx = (x - cx) / fx, ry = (y - cy) / fy;
        const double wx = R[0] * rx + R[3] * ry + R[6];
        const double wy = R[1] * rx + R[4] * ry + R[7];
        const double wz = R[2] * rx + R[5] * ry + R[8];
        const double cu = fx * wx / wz + cx, cv = fy * wy / wz + cy;
        const double rho = 12.0 + 5.0 * sin(cu / 97.0 + seed) + 4.0 * cos(cv / 61.0 - 0.5 * seed);
        double* X = B.map + 3 * ((size_t)s * B.map_cap + m0 + j);
        X[0] = wx / wz * rho;
        X[1] = wy / wz * rho;
        X[2] = rho;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        B.n[s] = n0 + take;
        B.map_n[s] = m0 + take;
        if (B.added) B.added[s] = take;
    }
}

__global__ __launch_bounds__(kFeBlock) void tail_kernel(TailBatch T, AppendBatch A) {
    const int s = blockIdx.x;
    __shared__ int wsum[kFeBlock / 64];
    __shared__ int base_s;
    const size_t o = (size_t)s * A.cap;
    const uint32_t* __restrict__ bits = T.bits + (size_t)s * T.words_cap;
    const int n = block_compact(T.n_in[s], [&](int i) { return ((bits[i >> 5] >> (i & 31)) & 1u) != 0; },
                                T.xy_in + 2 * o, T.mid_in + o, A.xy + 2 * o, A.mid + o, wsum, &base_s);
    if (threadIdx.x == 0) A.n[s] = n;
    __syncthreads();
    append_body(A, s);
    if (threadIdx.x == 0) {
        if (T.h_n) T.h_n[s] = A.n[s];
        if (T.h_added && A.added) T.h_added[s] = A.added[s];
    }
}

}  // namespace

hipError_t launch_post_lk(const PostLkBatch& b, int nseq, hipStream_t st) {
    hipLaunchKernelGGL(post_lk_kernel, dim3(nseq), dim3(kFeBlock), 0, st, b);
    return hipGetLastError();
}

hipError_t launch_tail(const TailBatch& tb, const AppendBatch& ab, int nseq, hipStream_t st) {
    hipLaunchKernelGGL(tail_kernel, dim3(nseq), dim3(kFeBlock), 0, st, tb, ab);
    return hipGetLastError();
}

hipError_t launch_ransac_samples(const int* counts, const float* obj, const float* img, int cap, int nh, int nseq,
                                 float* samp, hipStream_t st) {
    if (nh <= 0 || nh > 64) return hipErrorInvalidValue;
    hipLaunchKernelGGL(ransac_sample_kernel, dim3(nseq), dim3(256), 0, st, counts, obj, img, cap, nh, samp);
    return hipGetLastError();
}

hipError_t launch_compact(const CompactBatch& b, int nseq, hipStream_t st) {
    hipLaunchKernelGGL(compact_kernel, dim3(nseq), dim3(1024), 0, st, b);
    return hipGetLastError();
}

hipError_t launch_gather(const int* n, const int* mid, const double* map, int cap, int map_cap, float* obj,
                         int nseq, int max_n, hipStream_t st) {
    if (max_n <= 0) return hipSuccess;
    hipLaunchKernelGGL(gather_kernel, dim3((max_n + 255) / 256, nseq), dim3(256), 0, st, n, mid, map, cap,
                       map_cap, obj);
    return hipGetLastError();
}

hipError_t launch_append(const AppendBatch& b, int nseq, hipStream_t st) {
    hipLaunchKernelGGL(append_kernel, dim3(nseq), dim3(256), 0, st, b);
    return hipGetLastError();
}

}  // namespace svo
