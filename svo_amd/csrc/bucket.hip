// Bucketed feature selection (spatial cap per B x B cell) for gfx950.
//
// Replaces FeatureSet::bucketingFeatures (R:src/bucket.cpp:24-68) with its exact
// output, quirks included:
//   * (nh+1)(nw+1) buckets indexed with stride nw (bucket.cpp:50-53, :62): the
//     readout walks r in [0,nh], c in [0,nw] with idx = r*nw + c, so the bucket
//     of cell (r, nw) == (r+1, 0) is emitted twice;
//   * a full bucket's incoming point always replaces slot 0 (bucket.cpp:86-98:
//     the age loop compares the incoming age, never ages[i]);
//   * per bucket: [p_last if m > k else p_1, p_2 .. p_min(m,k)] in input order.
// Per bucket the output is fixed by four numbers: the count m, the first k point
// indices in input order and the last one -- slot 0 holds the last point when
// m > k, else the first; slots 1 .. k-1 the 2nd .. k-th. One 256-thread
// workgroup per sequence finds them without ranking every point:
//   (A) every point's bucket (kept in scratch), count and last index by LDS
//       atomics (add / max), and the largest count;
//   (B) pass j = 1 .. min(k, largest count): the j-th index of every bucket is the
//       smallest index above the (j-1)-th -- an LDS atomicMin over the points;
//   (C) exclusive scan of min(m, k) in readout order (stride-nw quirk above);
//   (D) scatter.
// Every thread works in every phase (the previous form ranked the points on one
// wave, peel by peel, against counters in global memory). Four waves per block,
// not sixteen: the kernel runs on the FAST stream beside LK, which holds three
// waves on every SIMD, and a 1024-thread workgroup (all sixteen waves resident on
// one CU) could only start where LK had drained -- measured 1.2 ms per launch,
// i.e. the whole LK, with either form. The tables live in LDS when they fit
// (KITTI / 50 px: 200 buckets, 5.6 KB), else in the sequence's global scratch.
#include "common.hpp"

#include <climits>

namespace svo {

namespace {

__device__ __forceinline__ int bucket_of(float x, float y, int B, int nw) {
    int hi = (int)(y / (float)B);
    int wi = (int)(x / (float)B);
    return hi * nw + wi;
}

constexpr int kBucketThreads = 256;

template <bool IN_LDS>
__global__ __launch_bounds__(kBucketThreads) void bucket_kernel(BucketBatch Bt, int B, int nh, int nw, int k) {
    extern __shared__ int lds_tab[];
    const int seq = blockIdx.x;
    const int n = Bt.in_counts ? min(Bt.in_counts[seq], Bt.in_cap) : Bt.n;
    const int E = Bt.in_elem;
    const float* __restrict__ xy = Bt.xy + (size_t)seq * Bt.in_cap * E;
    const int* __restrict__ ages = Bt.ages ? Bt.ages + (size_t)seq * Bt.in_cap : nullptr;
    float* __restrict__ xy_out = Bt.xy_out + 2 * (size_t)seq * Bt.out_cap;
    int* __restrict__ ages_out = Bt.ages_out ? Bt.ages_out + (size_t)seq * Bt.out_cap : nullptr;
    const int cap = Bt.out_cap;
    int* __restrict__ scr = Bt.scr + (size_t)seq * Bt.scr_stride;
    const int nb = (nh + 1) * (nw + 1);
    const int npos = nb;  // readout positions: (nh + 1) x (nw + 1)
    int* bidx = scr;      // n: each point's bucket (-1: outside, dropped)
    // tables: cnt[nb] | last[nb] | first[k][nb] | off[npos + 1]
    int* tab = IN_LDS ? lds_tab : scr + n;
    int* cnt = tab;
    int* last = cnt + nb;
    int* first = last + nb;  // [k][nb]
    int* off = first + (size_t)k * nb;
    __shared__ int maxcnt, carry;
    __shared__ int part[kBucketThreads / 64];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    for (int i = tid; i < nb; i += kBucketThreads) {
        cnt[i] = 0;
        last[i] = -1;
    }
    for (size_t i = tid; i < (size_t)k * nb; i += kBucketThreads) first[i] = INT_MAX;
    if (tid == 0) {
        maxcnt = 0;
        carry = 0;
    }
    __syncthreads();
    // (A) buckets, counts, last indices
    int mymax = 0;
    for (int i = tid; i < n; i += kBucketThreads) {
        int b = bucket_of(xy[E * i], xy[E * i + 1], B, nw);
        if (b < 0 || b >= nb) b = -1;  // out of range: undefined in the reference, dropped
        bidx[i] = b;
        if (b >= 0) {
            mymax = max(mymax, atomicAdd(&cnt[b], 1) + 1);
            atomicMax(&last[b], i);
        }
    }
    if (mymax) atomicMax(&maxcnt, mymax);
    __syncthreads();
    // (B) the first min(k, m) indices per bucket, one rank per pass
    const int passes = min(k, maxcnt);
    for (int j = 0; j < passes; j++) {
        const int* prev = j ? first + (size_t)(j - 1) * nb : nullptr;
        int* cur = first + (size_t)j * nb;
        for (int i = tid; i < n; i += kBucketThreads) {
            const int b = bidx[i];
            if (b >= 0 && cnt[b] > j && (!prev || i > prev[b])) atomicMin(&cur[b], i);
        }
        __syncthreads();
    }
    // (C) exclusive scan of min(m, k) over readout positions q = r (nw + 1) + c
    // (bucket r nw + c), a block's worth of positions per round: wave prefix sums by shuffles,
    // then the waves' totals
    for (int q0 = 0; q0 < npos; q0 += kBucketThreads) {
        const int q = q0 + tid;
        int v = 0;
        if (q < npos) {
            const int r = q / (nw + 1), c = q - r * (nw + 1);
            v = min(cnt[r * nw + c], k);
        }
        int incl = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(incl, o);
            if (lane >= o) incl += t;
        }
        if (lane == 63) part[wid] = incl;
        __syncthreads();
        int before = carry;
        for (int w = 0; w < wid; w++) before += part[w];
        if (q < npos) off[q] = before + incl - v;
        __syncthreads();
        if (tid == kBucketThreads - 1) carry = before + incl;
        __syncthreads();
    }
    if (tid == 0) *(Bt.n_out + seq) = carry;
    // (D) scatter: bucket b's slots in slot order
    for (int q = tid; q < npos; q += kBucketThreads) {
        const int r = q / (nw + 1), c = q - r * (nw + 1);
        const int b = r * nw + c;
        const int m = cnt[b];
        const int mk = min(m, k);
        for (int s = 0; s < mk; s++) {
            const int o = off[q] + s;
            if (o >= cap) break;
            const int i = s == 0 && m > k ? last[b] : first[(size_t)s * nb + b];
            xy_out[2 * o] = xy[E * i];
            xy_out[2 * o + 1] = xy[E * i + 1];
            if (ages_out) ages_out[o] = ages ? ages[i] : 0;
        }
    }
}

constexpr size_t kBucketLdsMax = 96 * 1024;

}  // namespace

size_t bucket_scratch_ints(int img_w, int img_h, int bucket, int per_bucket, int n) {
    const size_t nb = (size_t)(img_h / bucket + 1) * (img_w / bucket + 1);
    return (size_t)n + (size_t)(per_bucket + 2) * nb + nb + 1;  // bucket ids + tables (when not in LDS)
}

hipError_t launch_bucket(const BucketBatch& b, int nseq, int img_w, int img_h, int bucket, int per_bucket,
                         hipStream_t st) {
    const int nh = img_h / bucket, nw = img_w / bucket;
    const size_t nb = (size_t)(nh + 1) * (nw + 1);
    const size_t tab_bytes = sizeof(int) * ((size_t)(per_bucket + 2) * nb + nb + 1);
    if (tab_bytes <= kBucketLdsMax)
        hipLaunchKernelGGL(bucket_kernel<true>, dim3(nseq), dim3(kBucketThreads), tab_bytes, st, b, bucket, nh, nw,
                           per_bucket);
    else
        hipLaunchKernelGGL(bucket_kernel<false>, dim3(nseq), dim3(kBucketThreads), 0, st, b, bucket, nh, nw,
                           per_bucket);
    return hipGetLastError();
}

}  // namespace svo
