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
// One workgroup: (A) stable per-bucket ranks by a wave walking the points in
// input order with ballot/match peeling, (B) slot assignment, (C) exclusive scan
// of per-position sizes in readout order, (D) scatter. Bucket counts live in a
// context scratch buffer (zeroed here).
#include "common.hpp"

namespace svo {

namespace {

__device__ __forceinline__ int bucket_of(float x, float y, int B, int nw) {
    int hi = (int)(y / (float)B);
    int wi = (int)(x / (float)B);
    return hi * nw + wi;
}

__global__ __launch_bounds__(1024) void bucket_kernel(BucketBatch Bt, int B, int nh, int nw, int k) {
    const int seq = blockIdx.x;
    const int n = Bt.in_counts ? min(Bt.in_counts[seq], Bt.in_cap) : Bt.n;
    const int E = Bt.in_elem;
    const float* __restrict__ xy = Bt.xy + (size_t)seq * Bt.in_cap * E;
    const int* __restrict__ ages = Bt.ages ? Bt.ages + (size_t)seq * Bt.in_cap : nullptr;
    float* __restrict__ xy_out = Bt.xy_out + 2 * (size_t)seq * Bt.out_cap;
    int* __restrict__ ages_out = Bt.ages_out ? Bt.ages_out + (size_t)seq * Bt.out_cap : nullptr;
    const int cap = Bt.out_cap;
    int* __restrict__ n_out = Bt.n_out + seq;
    int* __restrict__ scr = Bt.scr + (size_t)seq * Bt.scr_stride;
    const int nb = (nh + 1) * (nw + 1);
    const int npos = (nh + 1) * (nw + 1);
    int* cnt = scr;             // nb
    int* slot = cnt + nb;       // nb * k point indices
    int* rank = slot + (size_t)nb * k;  // n
    int* off = rank + n;        // npos + 1
    const int tid = threadIdx.x;
    for (int i = tid; i < nb; i += 1024) cnt[i] = 0;
    __syncthreads();
    // (A) stable ranks: wave 0 walks the points in order, 64 at a time
    if (tid < 64) {
        const int lane = tid;
        for (int c0 = 0; c0 < n; c0 += 64) {
            const int i = c0 + lane;
            int b = -1;
            if (i < n) {
                b = bucket_of(xy[E * i], xy[E * i + 1], B, nw);
                if (b < 0 || b >= nb) b = -2;  // out of range: undefined in the reference, dropped
            }
            unsigned long long active = __ballot(b >= 0);
            int myrank = -1;
            while (active) {
                const int leader = __ffsll((long long)active) - 1;
                const int lb = __shfl(b, leader);
                const unsigned long long same = __ballot(b == lb);
                const int before = cnt[lb];
                if (b == lb) myrank = before + __popcll(same & ((1ull << lane) - 1ull));
                if (lane == leader) cnt[lb] = before + __popcll(same);
                active &= ~same;
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            }
            if (i < n) rank[i] = b >= 0 ? myrank : -1;
        }
    }
    __syncthreads();
    // (B) slots: ranks < k keep their slot, except rank 0 when m > k; the last
    // point of an overfull bucket owns slot 0
    for (int i = tid; i < n; i += 1024) {
        const int r = rank[i];
        if (r < 0) continue;
        const int b = bucket_of(xy[E * i], xy[E * i + 1], B, nw);
        const int m = cnt[b];
        if (r < k && !(r == 0 && m > k)) slot[(size_t)b * k + r] = i;
        if (m > k && r == m - 1) slot[(size_t)b * k] = i;
    }
    // (C) exclusive scan over readout positions q = r*(nw+1)+c -> idx = r*nw+c
    __shared__ int part[1024];
    __shared__ int carry;
    if (tid == 0) carry = 0;
    __syncthreads();
    for (int q0 = 0; q0 < npos; q0 += 1024) {
        const int q = q0 + tid;
        int v = 0;
        if (q < npos) {
            const int r = q / (nw + 1), c = q - r * (nw + 1);
            v = min(cnt[r * nw + c], k);
        }
        part[tid] = v;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {
            int t = tid >= o ? part[tid - o] : 0;
            __syncthreads();
            part[tid] += t;
            __syncthreads();
        }
        if (q < npos) off[q] = carry + part[tid] - v;
        __syncthreads();
        if (tid == 0) carry += part[1023];
        __syncthreads();
    }
    if (tid == 0) {
        off[npos] = carry;
        *n_out = carry;
    }
    __syncthreads();
    // (D) scatter
    for (int q = tid; q < npos; q += 1024) {
        const int r = q / (nw + 1), c = q - r * (nw + 1);
        const int b = r * nw + c;
        const int m = min(cnt[b], k);
        for (int s = 0; s < m; s++) {
            const int o = off[q] + s;
            if (o >= cap) break;
            const int i = slot[(size_t)b * k + s];
            xy_out[2 * o] = xy[E * i];
            xy_out[2 * o + 1] = xy[E * i + 1];
            if (ages_out) ages_out[o] = ages ? ages[i] : 0;
        }
    }
}

}  // namespace

size_t bucket_scratch_ints(int img_w, int img_h, int bucket, int per_bucket, int n) {
    const size_t nb = (size_t)(img_h / bucket + 1) * (img_w / bucket + 1);
    return nb + nb * per_bucket + (size_t)n + nb + 1;
}

hipError_t launch_bucket(const BucketBatch& b, int nseq, int img_w, int img_h, int bucket, int per_bucket,
                         hipStream_t st) {
    const int nh = img_h / bucket, nw = img_w / bucket;
    hipLaunchKernelGGL(bucket_kernel, dim3(nseq), dim3(1024), 0, st, b, bucket, nh, nw, per_bucket);
    return hipGetLastError();
}

}  // namespace svo
