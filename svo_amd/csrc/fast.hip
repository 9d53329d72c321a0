// FAST-9/16 corner detection + score + non-max suppression + mask + stable
// raster-order compaction for gfx950.
//
// Replaces mDetector->detect(leftImg, keypoints, mask) at R:src/tracking.cpp:82
// (cv::FastFeatureDetector::create(threshold, nonmaxSuppression) at :54-57) and
// the mask rectangles drawn at :76-79. Semantics follow OpenCV 4.x
// features2d/src/fast.cpp FAST_t<16> / fast_score.cpp cornerScore<16> /
// keypoint.cpp runByPixelsMask:
//   * detection area rows/cols 3 .. dim-4; darker: x < v - t, brighter: x > v + t;
//     corner = a circular run of >= 9 (the 25-entry walk of FAST_t is exactly a
//     circular run test on the 16-bit ring mask);
//   * score = cornerScore<16> (max threshold keeping the corner);
//   * NMS: strict '>' against all 8 neighbours, non-corners score 0;
//   * keypoints in raster order (y, then x) -- OpenCV's emission order;
//   * the mask drops keypoints AFTER NMS (masked corners still suppress).
//
// Kernels: (1) tile score kernel -> u16 map {corner bit 8 | score}; (2) per-row
// keep count; (3) per-row stable write at the row's exclusive offset.
#include "common.hpp"
#include "xcd_tile.hpp"

#include <cstdlib>

namespace svo {

namespace {

constexpr int FT_TX = 64, FT_TY = 16;           // output tile
constexpr int FT_IW = FT_TX + 6, FT_IH = FT_TY + 6;

// ring offsets (dx, dy) of makeOffsets(patternSize = 16)
__constant__ int8_t c_ring[16][2] = {{0, 3},  {1, 3},  {2, 2},   {3, 1},   {3, 0},  {3, -1},
                                     {2, -2}, {1, -3}, {0, -3},  {-1, -3}, {-2, -2}, {-3, -1},
                                     {-3, 0}, {-3, 1}, {-2, 2},  {-1, 3}};

__device__ __forceinline__ bool run9(unsigned m16) {
    unsigned m = m16 | (m16 << 16);   // circular
    unsigned r = m & (m >> 1);        // 2 consecutive
    r &= r >> 2;                      // 4
    r &= r >> 4;                      // 8
    r &= m >> 8;                      // 9
    return (r & 0xFFFFu) != 0;
}

// cornerScore<16> (fast_score.cpp) of the pixel with value v and ring values.
__device__ __forceinline__ int corner_score16(int v, const int* ring, int threshold) {
    int d[25];
#pragma unroll
    for (int k = 0; k < 25; k++) d[k] = v - ring[k & 15];
    int a0 = threshold;
#pragma unroll
    for (int k = 0; k < 16; k += 2) {
        int a = min(d[k + 1], d[k + 2]);
        a = min(a, d[k + 3]);
        a = min(a, d[k + 4]);
        a = min(a, d[k + 5]);
        a = min(a, d[k + 6]);
        a = min(a, d[k + 7]);
        a = min(a, d[k + 8]);
        a0 = max(a0, min(a, d[k]));
        a0 = max(a0, min(a, d[k + 9]));
    }
    int b0 = -a0;
#pragma unroll
    for (int k = 0; k < 16; k += 2) {
        int b = max(d[k + 1], d[k + 2]);
        b = max(b, d[k + 3]);
        b = max(b, d[k + 4]);
        b = max(b, d[k + 5]);
        b = max(b, d[k + 6]);
        b = max(b, d[k + 7]);
        b = max(b, d[k + 8]);
        b0 = min(b0, max(b, d[k]));
        b0 = min(b0, max(b, d[k + 9]));
    }
    return (-b0 - 1) & 0xFF;  // (uchar) cast in FAST_t
}

__global__ __launch_bounds__(256) void fast_score_kernel(FastBatch B, int threshold,
                                                         int want_score) {
    const ImgLevel L = B.descs[blockIdx.z].lv[0];
    const uint8_t* __restrict__ img = L.data;
    const int w = L.w, h = L.h, pitch = L.pitch;
    uint16_t* __restrict__ cs = B.cs + (size_t)blockIdx.z * B.npx;
    __shared__ uint8_t T[FT_IH][FT_IW + 2];
    const int x0 = blockIdx.x * FT_TX, y0 = blockIdx.y * FT_TY;
    const int tid = threadIdx.x;
    for (int k = tid; k < FT_IH * FT_IW; k += 256) {
        int r = k / FT_IW, c = k - r * FT_IW;
        int y = y0 - 3 + r, x = x0 - 3 + c;
        T[r][c] = ((unsigned)y < (unsigned)h && (unsigned)x < (unsigned)w) ? img[(size_t)y * pitch + x] : 0;
    }
    __syncthreads();
    const int c = tid & 63;
    const int x = x0 + c;
    if (x >= w) return;
    for (int i = 0; i < FT_TY / 4; i++) {
        const int r = (tid >> 6) * (FT_TY / 4) + i;
        const int y = y0 + r;
        if (y >= h) break;
        uint16_t out = 0;
        if (x >= 3 && x < w - 3 && y >= 3 && y < h - 3) {
            const int v = T[r + 3][c + 3];
            int ring[16];
            unsigned bright = 0, dark = 0;
#pragma unroll
            for (int k = 0; k < 16; k++) {
                ring[k] = T[r + 3 + c_ring[k][1]][c + 3 + c_ring[k][0]];
                bright |= (unsigned)(ring[k] > v + threshold) << k;
                dark |= (unsigned)(ring[k] < v - threshold) << k;
            }
            if (run9(bright) || run9(dark)) {
                const int score = want_score ? corner_score16(v, ring, threshold) : 0;
                out = (uint16_t)(0x100 | score);
            }
        }
        cs[(size_t)y * w + x] = out;
    }
}

__device__ __forceinline__ bool fast_keep(const uint16_t* __restrict__ cs, int w, int x, int y,
                                          int nonmax, const uint8_t* __restrict__ mask) {
    const uint16_t* p = cs + (size_t)y * w + x;
    unsigned v = p[0];
    if (!(v & 0x100)) return false;
    if (nonmax) {
        int s = v & 0xFF;
        // neighbours exist: corners lie in 3..dim-4
        if (!(s > (p[-1] & 0xFF) && s > (p[1] & 0xFF) && s > (p[-w - 1] & 0xFF) &&
              s > (p[-w] & 0xFF) && s > (p[-w + 1] & 0xFF) && s > (p[w - 1] & 0xFF) &&
              s > (p[w] & 0xFF) && s > (p[w + 1] & 0xFF)))
            return false;
    }
    if (mask && mask[(size_t)y * w + x] == 0) return false;
    return true;
}

__global__ __launch_bounds__(256) void fast_count_kernel(FastBatch B, int w, int h, int nonmax) {
    const int y = blockIdx.x;
    const uint16_t* __restrict__ cs = B.cs + (size_t)blockIdx.y * B.npx;
    const uint8_t* __restrict__ mask = B.mask ? B.mask + (size_t)blockIdx.y * B.npx : nullptr;
    int* __restrict__ rowcnt = B.rowcnt + (size_t)blockIdx.y * h;
    __shared__ int wsum[4];
    int cnt = 0;
    if (y >= 3 && y < h - 3)
        for (int x = 3 + threadIdx.x; x < w - 3; x += 256) cnt += fast_keep(cs, w, x, y, nonmax, mask);
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) rowcnt[y] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

__global__ __launch_bounds__(256) void fast_write_kernel(FastBatch B, int w, int h, int nonmax) {
    const int y = blockIdx.x;
    const uint16_t* __restrict__ cs = B.cs + (size_t)blockIdx.y * B.npx;
    const uint8_t* __restrict__ mask = B.mask ? B.mask + (size_t)blockIdx.y * B.npx : nullptr;
    const int* __restrict__ rowcnt = B.rowcnt + (size_t)blockIdx.y * h;
    svo_keypoint* __restrict__ out = B.out + (size_t)blockIdx.y * B.cap;
    const int cap = B.cap;
    int* __restrict__ n_out = B.n_out + blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    __shared__ int wsum[4];
    __shared__ int base_s;
    // exclusive offset of this row: sum of the counts of rows above
    int s = 0;
    for (int r = tid; r < y; r += 256) s += rowcnt[r];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) wsum[wv] = s;
    __syncthreads();
    if (tid == 0) {
        base_s = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        if (y == h - 1) *n_out = base_s + rowcnt[y];
    }
    __syncthreads();
    if (y < 3 || y >= h - 3 || rowcnt[y] == 0) return;
    int base = base_s;
    for (int x0 = 0; x0 < w; x0 += 256) {
        const int x = x0 + tid;
        const bool keep = x >= 3 && x < w - 3 && fast_keep(cs, w, x, y, nonmax, mask);
        const unsigned long long bal = __ballot(keep);
        const int rank = __popcll(bal & ((1ull << lane) - 1ull));
        __syncthreads();
        if (lane == 0) wsum[wv] = __popcll(bal);
        __syncthreads();
        int off = base;
        for (int k = 0; k < wv; k++) off += wsum[k];
        if (keep) {
            const int idx = off + rank;
            if (idx < cap) {
                svo_keypoint kp;
                kp.x = (float)x;
                kp.y = (float)y;
                kp.response = (float)(cs[(size_t)y * w + x] & 0xFF);
                out[idx] = kp;
            }
        }
        base += wsum[0] + wsum[1] + wsum[2] + wsum[3];
    }
}

// ---- fused detection (fast_detect_q_kernel): FAST-9 + score + NMS + box mask for
// a 64 x TY tile of a frame, one 64-bit keep word per (row, 64-px segment) and
// per-row counts. Each wave owns every 4th row of the tile's score region (the
// tile and a 1-pixel halo, whose scores NMS needs) and runs, with no block
// barrier, (A0) the compass pre-test of its rows -> a wave-private queue (ballot
// ranks, no atomics), (A1) the full segment test of the queue, compacted in
// place to the corners, (B) their cornerScore with packed 16-bit min/max (the
// a-chain in the low halves, the negated b-chain in the high ones). One barrier,
// then NMS over the wave's corners only, the box mask ANDed into the finished
// row words. ----
constexpr int FD_TX = 64, FD_TY = 32;
constexpr int FD_SW = FD_TX + 2;  // score region columns (halo 1)
constexpr int FD_IW = FD_TX + 8;  // staged image columns (halo 4)
typedef short fs16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ fs16x2 as_s2(unsigned v) { return __builtin_bit_cast(fs16x2, v); }
__device__ __forceinline__ unsigned as_u(fs16x2 v) { return __builtin_bit_cast(unsigned, v); }

// lanes below this one with their bit set in the wave mask m (v_mbcnt pair)
__device__ __forceinline__ int rank_below(unsigned long long m) {
    return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

// cornerScore<16> (fast_score.cpp) with both chains in one packed pass: low half
// a0 = max_k max(min(a_k, d[k]), min(a_k, d[k+9])) from threshold, high half the
// same on e = -d from -inf (= -B of the b-chain); b0 = min(-a0, B), score = -b0 - 1
__device__ __forceinline__ int corner_score16_pk(int v, const int* ring, int threshold) {
    fs16x2 D[25];
    const fs16x2 sgn = {(short)-1, (short)1};
    const fs16x2 base = {(short)v, (short)-v};
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const fs16x2 r2 = {(short)ring[k], (short)ring[k]};
        D[k] = r2 * sgn + base;  // (v - r, r - v)
    }
#pragma unroll
    for (int k = 16; k < 25; k++) D[k] = D[k - 16];
    fs16x2 acc = {(short)threshold, (short)-32768};
#pragma unroll
    for (int k = 0; k < 16; k += 2) {
        fs16x2 a = __builtin_elementwise_min(D[k + 1], D[k + 2]);
#pragma unroll
        for (int j = 3; j <= 8; j++) a = __builtin_elementwise_min(a, D[k + j]);
        acc = __builtin_elementwise_max(acc, __builtin_elementwise_min(a, D[k]));
        acc = __builtin_elementwise_max(acc, __builtin_elementwise_min(a, D[k + 9]));
    }
    const int a0 = acc.x, nb = acc.y;  // nb = -B
    return (max(a0, nb) - 1) & 0xFF;   // -min(-a0, B) - 1, (uchar) as FAST_t
}

// XT: tiles in XCD order (xcd_tile.hpp)
template <int TY, bool XT = false>
__global__ __launch_bounds__(256) void fast_detect_q_kernel(FastDetBatch B, int threshold, int nonmax) {
    constexpr int QSH = TY + 2, QIH = TY + 8;           // score rows (halo 1), staged rows (halo 4)
    constexpr int QQ = ((QSH + 3) / 4) * FD_SW + 8;      // queue entries per wave
    static_assert(2 * ((QSH + 3) / 4) <= 64, "halo pre-test: one lane per (row, side)");
    static_assert(QSH < 512, "queue entries pack (row << 7 | column) into 16 bits");
    const XcdTile tile = XT ? xcd_tile() : XcdTile{(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z};
    const ImgLevel L = B.descs[tile.z].lv[0];
    const int w = L.w, h = L.h;
    const int x0 = tile.x * FD_TX, y0 = tile.y * TY;
    const size_t seq = tile.z;
    __shared__ __attribute__((aligned(16))) uint8_t T[QIH][FD_IW];
    __shared__ __attribute__((aligned(16))) uint16_t SC[QSH][FD_SW + 2];  // bit 8: corner, low byte: score
    __shared__ uint16_t CQ[4][QQ];
    __shared__ unsigned long long TM[TY];
    __shared__ unsigned long long RB[TY];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const bool inside = B.padded ? x0 - 4 + FD_IW <= L.pitch - kPyrPad && y0 - 4 + QIH <= h + kPyrPad
                                 : x0 >= 4 && y0 >= 4 && x0 - 4 + FD_IW <= w && y0 - 4 + QIH <= h;
    if (inside) {
        // thread -> (row r0, dword c4), rows r0 + RP p: all loads in flight before the
        // first LDS store
        constexpr int DW = FD_IW / 4, RP = 256 / DW, NP = (QIH + RP - 1) / RP;
        const int r0 = tid / DW, c4 = tid - r0 * DW;
        if (r0 < RP) {
            const uint8_t* src = L.data + (size_t)(y0 - 4 + r0) * L.pitch + (x0 - 4 + 4 * c4);
            uint32_t v[NP];
#pragma unroll
            for (int p = 0; p < NP; p++)
                v[p] = *reinterpret_cast<const uint32_t*>(src + (size_t)(min(r0 + p * RP, QIH - 1) - r0) * L.pitch);
            // (rows past the tile load and store its last row again, the same bytes:
            // no branch, so no wait between the loads)
#pragma unroll
            for (int p = 0; p < NP; p++) *reinterpret_cast<uint32_t*>(&T[min(r0 + p * RP, QIH - 1)][4 * c4]) = v[p];
        }
    } else {
        for (int k = tid; k < QIH * FD_IW; k += 256) {
            const int r = k / FD_IW, c = k - r * FD_IW;
            const int y = y0 - 4 + r, x = x0 - 4 + c;
            T[r][c] = ((unsigned)y < (unsigned)h && (unsigned)x < (unsigned)w) ? L.data[(size_t)y * L.pitch + x] : 0;
        }
    }
    const bool boxes = B.box_pts != nullptr;
    if (boxes && tid < TY) TM[tid] = ~0ull;
    if (tid < TY) RB[tid] = 0ull;
    // the wave's score region rows cleared (one dword per lane and row; before the
    // barrier, away from the tests)
    if (lane < (FD_SW + 2) / 2) {
        uint32_t* sc0 = reinterpret_cast<uint32_t*>(&SC[wv][0]) + lane;
#pragma unroll
        for (int i = 0; i < (QSH + 3) / 4; i++)
            if (4 * i + 3 < QSH || wv + 4 * i < QSH) sc0[i * 2 * (FD_SW + 2)] = 0u;
    }
    __syncthreads();
    const int hi_t = threshold, lo_t = -threshold;
    // ---- A0: compass pre-test of this wave's rows sr = wv, wv + 4, ... (lane -> column
    // sc = lane + 1), then the two halo columns of those rows; queue (sr << 7 | sc) ----
    uint16_t* q = CQ[wv];
    int nq = 0;
    auto pretest = [&](int sr, int sc, bool ok) {
        const int y = y0 - 1 + sr, x = x0 - 1 + sc;
        bool cand = false;
        if (ok && x >= 3 && x < w - 3 && y >= 3 && y < h - 3) {
            const int ty = sr + 3, tx = sc + 3;
            const int v = T[ty][tx], hi = v + hi_t, lo = v + lo_t;
            const int p0 = T[ty + 3][tx], p8 = T[ty - 3][tx], p4 = T[ty][tx + 3], p12 = T[ty][tx - 3];
            const bool bright = (p0 > hi || p8 > hi) && (p4 > hi || p12 > hi);
            const bool dark = (p0 < lo || p8 < lo) && (p4 < lo || p12 < lo);
            cand = bright || dark;
        }
        const unsigned long long bal = __builtin_amdgcn_ballot_w64(cand);
        if (cand) q[nq + rank_below(bal)] = (uint16_t)((sr << 7) | sc);
        nq += __popcll(bal);
    };
    {
        // columns 1 .. 64 (lane -> sc = lane + 1), unrolled over the rows: one LDS base
        // per lane (staged row sr, column sc), the five taps at immediate offsets,
        // branch-free (every tap lies inside the staged tile). All rows' tests first
        // (straight-line: the next rows' taps load while a row computes), then the
        // queue writes.
        constexpr int NRW = (QSH + 3) / 4;
        const int wvu = __builtin_amdgcn_readfirstlane(wv);
        const bool colok = x0 + lane >= 3 && x0 + lane < w - 3;
        const uint8_t* tb = &T[wvu][lane + 1];
        unsigned long long bal[NRW];
        unsigned cm = 0;
#pragma unroll
        for (int i = 0; i < NRW; i++) {
            const int sr = wvu + 4 * i;
            bal[i] = 0;
            if (4 * i + 3 < QSH || sr < QSH) {  // (only the last row is not every wave's)
                const uint8_t* t = tb + i * 4 * FD_IW;
                const int v = t[3 * FD_IW + 3], hi = v + hi_t, lo = v + lo_t;
                const int p8 = t[3], p0 = t[6 * FD_IW + 3], p12 = t[3 * FD_IW], p4 = t[3 * FD_IW + 6];
                const int y = y0 - 1 + sr;
                const bool rowok = y >= 3 && y < h - 3;
                const bool bright = min(max(p0, p8), max(p4, p12)) > hi;
                const bool dark = max(min(p0, p8), min(p4, p12)) < lo;
                const bool cand = colok & rowok & (bright | dark);
                bal[i] = __builtin_amdgcn_ballot_w64(cand);
                cm |= (unsigned)cand << i;
            }
        }
#pragma unroll
        for (int i = 0; i < NRW; i++) {
            if ((cm >> i) & 1u) q[nq + rank_below(bal[i])] = (uint16_t)(((wvu + 4 * i) << 7) | (lane + 1));
            nq += __popcll(bal[i]);
        }
    }
    {
        // halo columns 0 and 65 of the wave's rows (<= 9 rows -> 18 positions)
        const int nr = (QSH - wv + 3) / 4;
        const int sr = wv + 4 * (lane >> 1), sc = (lane & 1) * 65;
        pretest(sr, sc, lane < 2 * nr);
    }
    // ---- A1: full segment test of the queue, compacted in place to the corners ----
    int nc = 0;
    for (int base = 0; base < nq; base += 64) {
        const int i = base + lane;
        bool corner = false;
        int k = 0;
        if (i < nq) {
            k = q[i];
            const int sr = k >> 7, sc = k & 127;
            const int ty = sr + 3, tx = sc + 3;
            const int v = T[ty][tx];
            // packed compare: low half r - (v + t + 1) (sign: not brighter), high half
            // r - (v - t) (sign: darker); sign bits gathered to bit q and 16 + q
            const fs16x2 th = {(short)(v + threshold + 1), (short)(v - threshold)};
            unsigned acc = 0;
#pragma unroll
            for (int qq = 0; qq < 16; qq++) {
                const int rv = T[ty + c_ring[qq][1]][tx + c_ring[qq][0]];
                const fs16x2 r2 = {(short)rv, (short)rv};
                const unsigned sg = as_u(r2 - th);
                acc |= (sg >> (15 - qq)) & (0x00010001u << qq);
            }
            corner = run9(~acc & 0xFFFFu) || run9(acc >> 16);
        }
        const unsigned long long bal = __builtin_amdgcn_ballot_w64(corner);
        if (corner) {
            const int sr = k >> 7, sc = k & 127;
            SC[sr][sc] = 0x100;
            q[nc + rank_below(bal)] = (uint16_t)k;  // index <= i: already read
        }
        nc += __popcll(bal);
    }
    // ---- B: cornerScore of the corners (NMS only; a separate pass: a wave's queue
    // may take two A1 passes, its corners rarely more than one) ----
    if (nonmax) {
        for (int i = lane; i < nc; i += 64) {
            const int k = q[i];
            const int sr = k >> 7, sc = k & 127;
            const int ty = sr + 3, tx = sc + 3;
            const int v = T[ty][tx];
            int ring[16];
#pragma unroll
            for (int qq = 0; qq < 16; qq++) ring[qq] = T[ty + c_ring[qq][1]][tx + c_ring[qq][0]];
            SC[sr][sc] = (uint16_t)(0x100 | corner_score16_pk(v, ring, threshold));
        }
    }
    // tile mask from the previous frame's feature boxes
    if (boxes) {
        const int nb = (h + 15) / 16, ncl = (w + 63) / 64;
        const int* __restrict__ cells = B.box_band + seq * (size_t)(nb * ncl + 1);
        const int b0 = max(0, (int)floorf((y0 - B.box_half - 1.f) / 16.f));
        const int b1 = min(nb - 1, (int)floorf((y0 + TY + B.box_half + 1.f) / 16.f));
        const int cb0 = max(0, (int)floorf((x0 - B.box_half - 1.f) / 64.f));
        const int cb1 = min(ncl - 1, (int)floorf((x0 + FD_TX + B.box_half + 1.f) / 64.f));
        const float* __restrict__ pts = B.box_binned + 2 * seq * (size_t)B.box_stride;
        for (int bq = b0; bq <= b1; bq++)
            for (int i = cells[bq * ncl + cb0] + tid, i1 = cells[bq * ncl + cb1 + 1]; i < i1; i += 256) {
                const float px = pts[2 * i], py = pts[2 * i + 1];
                const int xa = (int)__builtin_rintf(px - B.box_half), ya = (int)__builtin_rintf(py - B.box_half);
                const int xb = (int)__builtin_rintf(px + B.box_half), yb = (int)__builtin_rintf(py + B.box_half);
                int xl = min(xa, xb), xr = max(xa, xb), yt = min(ya, yb), yd = max(ya, yb);
                xl = max(xl, max(0, x0));
                xr = min(xr, min(w - 1, x0 + FD_TX - 1));
                yt = max(yt, max(0, y0));
                yd = min(yd, min(h - 1, y0 + TY - 1));
                if (xl > xr || yt > yd) continue;
                const int c0 = xl - x0, c1 = xr - x0;  // 0..63
                const unsigned long long span =
                    (c1 - c0 == 63) ? ~0ull : (((1ull << (c1 - c0 + 1)) - 1ull) << c0);
                for (int y = yt; y <= yd; y++) atomicAnd(&TM[y - y0], ~span);
            }
    }
    __syncthreads();
    // NMS over this wave's corners only (a few % of the pixels): strict maximum over
    // the 8 neighbours' score bytes (non-corners score 0), the host mask per corner,
    // keep bits OR-ed into the row words
    const uint8_t* __restrict__ mask = B.mask ? B.mask + seq * B.npx : nullptr;
    for (int i = lane; i < nc; i += 64) {
        const int k = q[i];
        const int sr = k >> 7, sc = k & 127;
        if (sr < 1 || sr > TY || sc < 1 || sc > FD_TX) continue;  // halo: scores only
        const int x = x0 + sc - 1, y = y0 + sr - 1;
        bool keep = x < w && y < h;
        if (nonmax) {
            auto sb = [&](int y2, int x2) { return (int)reinterpret_cast<const uint8_t*>(&SC[y2][x2])[0]; };
            int m = max(max(sb(sr, sc - 1), sb(sr, sc + 1)), sb(sr - 1, sc - 1));
            m = max(max(m, sb(sr - 1, sc)), sb(sr - 1, sc + 1));
            m = max(max(m, sb(sr + 1, sc - 1)), sb(sr + 1, sc));
            m = max(m, sb(sr + 1, sc + 1));
            keep = keep && sb(sr, sc) > m;
        }
        if (mask && keep) keep = mask[(size_t)y * w + x] != 0;
        if (keep) {
            atomicOr(&RB[sr - 1], 1ull << (sc - 1));
            // (a box may still drop it: then the byte is never read)
            if (B.score_map) B.score_map[seq * B.npx + (size_t)y * w + x] = (uint8_t)(SC[sr][sc] & 0xFF);
        }
    }
    __syncthreads();
    if (tid < TY && y0 + tid < h) {
        const unsigned long long bal = RB[tid] & (boxes ? TM[tid] : ~0ull);
        B.bits[(seq * B.nseg + tile.x) * (size_t)h + y0 + tid] = bal;
    }
}

// ---- box filter of an unmasked detection (kFastBoxes): the previous frame's
// feature boxes rasterised per 64x32 tile exactly as fast_detect_q_kernel<32> does
// (cv::rectangle semantics from the band-binned centres), ANDed into the row words
// the detection wrote (fast_scan_kernel counts them). The boxes are applied after NMS in
// every form, so detecting first and masking later gives the same keypoints. ----
__global__ __launch_bounds__(64) void fast_box_filter_kernel(FastDetBatch B, int w, int h) {
    // one wave per 64 x 32 tile: the lanes first read the box ranges of the tile's
    // bands (one cell range per band), then take the boxes of all bands together
    constexpr int TY = 32;
    const XcdTile tile = xcd_tile();  // (neighbouring tiles' band ranges and words on one L2)
    const int x0 = tile.x * FD_TX, y0 = tile.y * TY;
    const size_t seq = tile.z;
    __shared__ unsigned long long TM[TY];
    __shared__ int band_lo[64], band_end[64];  // box ranges of the tile's bands, concatenated
    const int lane = threadIdx.x;
    if (lane < TY) TM[lane] = ~0ull;
    __syncthreads();
    const int nb = (h + 15) / 16, ncl = (w + 63) / 64;
    const int* __restrict__ cells = B.box_band + seq * (size_t)(nb * ncl + 1);
    const int b0 = max(0, (int)floorf((y0 - B.box_half - 1.f) / 16.f));
    const int b1 = min(nb - 1, (int)floorf((y0 + TY + B.box_half + 1.f) / 16.f));
    const int cb0 = max(0, (int)floorf((x0 - B.box_half - 1.f) / 64.f));
    const int cb1 = min(ncl - 1, (int)floorf((x0 + FD_TX + B.box_half + 1.f) / 64.f));
    const float2* __restrict__ pts = reinterpret_cast<const float2*>(B.box_binned + 2 * seq * (size_t)B.box_stride);
    for (int bb = b0; bb <= b1; bb += 64) {
        const int nband = min(64, b1 - bb + 1);
        int lo = 0, cnt = 0;
        if (lane < nband) {
            lo = cells[(bb + lane) * ncl + cb0];
            cnt = cells[(bb + lane) * ncl + cb1 + 1] - lo;
        }
        // inclusive prefix of the band counts (every lane converged here), to LDS:
        // the box loop below is divergent, where a lane must not read another
        // lane's registers (an inactive source lane reads as 0)
        int incl = cnt;
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(incl, o);
            if (lane >= o) incl += v;
        }
        const int total = __shfl(incl, nband - 1);
        band_lo[lane] = lo;
        band_end[lane] = incl;
        __syncthreads();
        for (int j = lane; j < total; j += 64) {
            // the band holding box j of the concatenated ranges
            int q = 0;
            while (j >= band_end[q]) q++;
            const int i = band_lo[q] + (j - (q > 0 ? band_end[q - 1] : 0));
            const float2 pt = pts[i];
            const int xa = (int)__builtin_rintf(pt.x - B.box_half), ya = (int)__builtin_rintf(pt.y - B.box_half);
            const int xb = (int)__builtin_rintf(pt.x + B.box_half), yb = (int)__builtin_rintf(pt.y + B.box_half);
            int xl = min(xa, xb), xr = max(xa, xb), yt = min(ya, yb), yd = max(ya, yb);
            xl = max(xl, max(0, x0));
            xr = min(xr, min(w - 1, x0 + FD_TX - 1));
            yt = max(yt, max(0, y0));
            yd = min(yd, min(h - 1, y0 + TY - 1));
            if (xl > xr || yt > yd) continue;
            const int c0 = xl - x0, c1 = xr - x0;  // 0..63
            const unsigned long long span = (c1 - c0 == 63) ? ~0ull : (((1ull << (c1 - c0 + 1)) - 1ull) << c0);
            for (int y = yt; y <= yd; y++) atomicAnd(&TM[y - y0], ~span);
        }
        __syncthreads();  // (band_lo / band_end are rewritten by a next round of bands)
    }
    __syncthreads();
    if (lane < TY && y0 + lane < h) {
        unsigned long long* word = B.bits + (seq * B.nseg + tile.x) * (size_t)h + y0 + lane;
        *word &= TM[lane];
    }
}

// Box centres of one sequence binned by cell (16-row band x 64-column tile):
// counting sort, one block per sequence; order within a cell is irrelevant
// (the mask is an AND of boxes).
constexpr int kMaxBoxCells = 12288;
__global__ __launch_bounds__(256) void box_bin_kernel(FastDetBatch B, int w, int h) {
    const size_t seq = blockIdx.x;
    const int nb = (h + 15) / 16, nc = (w + 63) / 64, ncell = nb * nc;
    extern __shared__ int box_lds[];  // [256] chunk totals + [ncell] counts (sized at launch)
    int* part = box_lds;
    int* cnt = box_lds + 256;
    const int n = B.box_counts[seq];
    const float* __restrict__ pts = B.box_pts + 2 * seq * (size_t)B.box_stride;
    float* __restrict__ outp = B.box_binned + 2 * seq * (size_t)B.box_stride;
    int* __restrict__ cells = B.box_band + seq * (size_t)(ncell + 1);
    for (int c = threadIdx.x; c < ncell; c += 256) cnt[c] = 0;
    __syncthreads();
    auto cell_of = [&](float x, float y) {
        int b = (int)floorf(y / 16.f), t = (int)floorf(x / 64.f);
        b = b < 0 ? 0 : b >= nb ? nb - 1 : b;
        t = t < 0 ? 0 : t >= nc ? nc - 1 : t;
        return b * nc + t;
    };
    for (int i = threadIdx.x; i < n; i += 256) atomicAdd(&cnt[cell_of(pts[2 * i], pts[2 * i + 1])], 1);
    __syncthreads();
    // exclusive scan: each thread a contiguous chunk, then the chunk totals
    const int chunk = (ncell + 255) / 256, c0 = threadIdx.x * chunk, c1 = min(ncell, c0 + chunk);
    int acc = 0;
    for (int c = c0; c < c1; c++) acc += cnt[c];
    part[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        int run = 0;
        for (int k = 0; k < 256; k++) {
            const int v = part[k];
            part[k] = run;
            run += v;
        }
        cells[ncell] = run;
    }
    __syncthreads();
    int run = part[threadIdx.x];
    for (int c = c0; c < c1; c++) {
        const int v = cnt[c];
        cells[c] = run;
        cnt[c] = run;  // becomes the running cursor
        run += v;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += 256) {
        const float x = pts[2 * i], y = pts[2 * i + 1];
        const int pos = atomicAdd(&cnt[cell_of(x, y)], 1);
        outp[2 * pos] = x;
        outp[2 * pos + 1] = y;
    }
}

// per-row corner counts (popcounts of the row words the detection / box filter
// wrote: no atomics in those kernels) and their exclusive scan, one sequence per
// 256-thread block (it finds room beside LK, a 1024-thread block waits for a whole
// CU): each thread counts a run of consecutive rows, one block scan of the run sums
constexpr int kScanBlock = 256;
__global__ __launch_bounds__(kScanBlock) void fast_scan_kernel(FastDetBatch B, int h) {
    const size_t seq = blockIdx.x;
    int* __restrict__ cnt = B.rowcnt + seq * h;
    int* __restrict__ off = B.rowoff + seq * h;
    const unsigned long long* __restrict__ words = B.bits + seq * (size_t)h * B.nseg;  // [segment][row]
    __shared__ int part[kScanBlock];
    const int tid = threadIdx.x;
    const int run = (h + kScanBlock - 1) / kScanBlock, y0 = tid * run, y1 = min(h, y0 + run);
    int sum = 0;
    for (int y = y0; y < y1; y++) {  // the row's corners: the popcount of its words
        int c = 0;
        for (int sgi = 0; sgi < B.nseg; sgi++) c += __popcll(words[(size_t)sgi * h + y]);
        cnt[y] = c;
        sum += c;
    }
    part[tid] = sum;
    __syncthreads();
    for (int o = 1; o < kScanBlock; o <<= 1) {
        const int t = tid >= o ? part[tid - o] : 0;
        __syncthreads();
        part[tid] += t;
        __syncthreads();
    }
    int acc = part[tid] - sum;
    for (int y = y0; y < y1; y++) {
        off[y] = acc;
        acc += cnt[y];
    }
    if (tid == kScanBlock - 1) {
        const int total = part[kScanBlock - 1];
        B.n_out[seq] = total;
    }
}

// raster-order write of one row's keypoints (one wave per row); the FAST
// score of a kept corner is recomputed from the image (few pixels)
constexpr int kEmitRows = 8;  // rows per wave: the segment-major words of 8 rows share a line
__global__ __launch_bounds__(64) void fast_emit_kernel(FastDetBatch B, int threshold, int nonmax) {
    const XcdTile tile = xcd_tile();  // (neighbouring row groups' words on one L2)
    const size_t seq = tile.y;
    const ImgLevel L = B.descs[seq].lv[0];
    const int h = L.h;
    for (int y = tile.x * kEmitRows; y < min(h, (tile.x + 1) * kEmitRows); y++) {
        if (B.rowcnt[seq * h + y] == 0) continue;
        const int lane = threadIdx.x;
        int off = B.rowoff[seq * h + y];
        const unsigned long long* bits = B.bits + seq * (size_t)h * B.nseg + y;  // word sgi at bits[sgi * h]
        svo_keypoint* __restrict__ out = B.out + seq * B.cap;
        for (int sgi = 0; sgi < B.nseg; sgi++) {
            const unsigned long long m = bits[(size_t)sgi * h];
            if (!m) continue;
            if ((m >> lane) & 1ull) {
                const int idx = off + __popcll(m & ((1ull << lane) - 1ull));
                if (idx < B.cap) {
                    const int x = sgi * 64 + lane;
                    float resp = 0.f;
                    if (nonmax && B.score_map) {
                        resp = (float)B.score_map[seq * B.npx + (size_t)y * L.w + x];
                    } else if (nonmax) {
                        const uint8_t* p = L.data + (size_t)y * L.pitch + x;
                        int ring[16];
    #pragma unroll
                        for (int q = 0; q < 16; q++) ring[q] = p[c_ring[q][1] * L.pitch + c_ring[q][0]];
                        resp = (float)corner_score16(p[0], ring, threshold);
                    }
                    svo_keypoint kp;
                    kp.x = (float)x;
                    kp.y = (float)y;
                    kp.response = resp;
                    out[idx] = kp;
                }
            }
            off += __popcll(m);
        }
    }
}

__global__ __launch_bounds__(64) void mask_boxes_kernel(int w, int h, const float* __restrict__ pts_all,
                                                        const int* __restrict__ counts, int n0,
                                                        int pts_stride, float half,
                                                        uint8_t* __restrict__ mask_all) {
    const int i = blockIdx.x;
    const int n = counts ? counts[blockIdx.y] : n0;
    if (i >= n) return;
    const float* __restrict__ pts = pts_all + 2 * (size_t)blockIdx.y * pts_stride;
    uint8_t* __restrict__ mask = mask_all + (size_t)blockIdx.y * w * h;
    const float px = pts[2 * i], py = pts[2 * i + 1];
    // cv::rectangle(Point2f -> Point via cvRound, FILLED, inclusive, clipped)
    int xa = (int)__builtin_rintf(px - half), ya = (int)__builtin_rintf(py - half);
    int xb = (int)__builtin_rintf(px + half), yb = (int)__builtin_rintf(py + half);
    int xl = min(xa, xb), xr = max(xa, xb), yt = min(ya, yb), yd = max(ya, yb);
    xl = max(xl, 0);
    yt = max(yt, 0);
    xr = min(xr, w - 1);
    yd = min(yd, h - 1);
    const int bw = xr - xl + 1, bh = yd - yt + 1;
    if (bw <= 0 || bh <= 0) return;
    for (int k = threadIdx.x; k < bw * bh; k += 64) {
        int r = k / bw, c = k - r * bw;
        mask[(size_t)(yt + r) * w + (xl + c)] = 0;
    }
}

}  // namespace

hipError_t launch_fast_score(const FastBatch& b, int nseq, int w, int h, int threshold, int nonmax,
                             hipStream_t st) {
    dim3 grid((w + FT_TX - 1) / FT_TX, (h + FT_TY - 1) / FT_TY, nseq);
    hipLaunchKernelGGL(fast_score_kernel, grid, dim3(256), 0, st, b, threshold, nonmax);
    return hipGetLastError();
}

hipError_t launch_fast_collect(const FastBatch& b, int nseq, int w, int h, int nonmax, hipStream_t st) {
    hipLaunchKernelGGL(fast_count_kernel, dim3(h, nseq), dim3(256), 0, st, b, w, h, nonmax);
    hipLaunchKernelGGL(fast_write_kernel, dim3(h, nseq), dim3(256), 0, st, b, w, h, nonmax);
    return hipGetLastError();
}

hipError_t launch_fast_detect(const FastDetBatch& b0, int nseq, int w, int h, int threshold, int nonmax,
                              hipStream_t st, int stage) {
    FastDetBatch b = b0;
    if (stage == kFastBoxes) {
        if (b.mask) return hipErrorInvalidValue;  // a host mask goes with the detection
        if (b.box_pts) {
            hipError_t e = hipSuccess;
            if (!b.box_prebinned) {
                e = launch_box_bin(b, nseq, w, h, st);
                if (e != hipSuccess) return e;
            }
            hipLaunchKernelGGL(fast_box_filter_kernel, dim3((w + FD_TX - 1) / FD_TX, (h + 31) / 32, nseq), dim3(64),
                               0, st, b, w, h);
        }
        hipLaunchKernelGGL(fast_scan_kernel, dim3(nseq), dim3(kScanBlock), 0, st, b, h);
        hipLaunchKernelGGL(fast_emit_kernel, dim3((h + kEmitRows - 1) / kEmitRows, nseq), dim3(64), 0, st, b, threshold, nonmax);
        return hipGetLastError();
    }
    hipError_t e = hipSuccess;
    if (b.box_pts && !b.box_prebinned) {
        e = launch_box_bin(b, nseq, w, h, st);
        if (e != hipSuccess) return e;
    }
    dim3 grid((w + FD_TX - 1) / FD_TX, (h + FD_TY - 1) / FD_TY, nseq);
    if (xcd_tiles_on())
        hipLaunchKernelGGL((fast_detect_q_kernel<FD_TY, true>), grid, dim3(256), 0, st, b, threshold, nonmax);
    else
        hipLaunchKernelGGL(fast_detect_q_kernel<FD_TY>, grid, dim3(256), 0, st, b, threshold, nonmax);
    if (stage == kFastDetect) return hipGetLastError();
    hipLaunchKernelGGL(fast_scan_kernel, dim3(nseq), dim3(kScanBlock), 0, st, b, h);
    hipLaunchKernelGGL(fast_emit_kernel, dim3((h + kEmitRows - 1) / kEmitRows, nseq), dim3(64), 0, st, b, threshold, nonmax);
    return hipGetLastError();
}

hipError_t launch_box_bin(const FastDetBatch& b, int nseq, int w, int h, hipStream_t st) {
    if (!b.box_pts) return hipSuccess;
    if (fast_box_cells(w, h) - 1 > kMaxBoxCells) return hipErrorInvalidValue;
    // LDS sized to the cell grid (2 KB at KITTI size): the kernel runs beside LK
    // and must fit next to its blocks
    const size_t lds = sizeof(int) * (256 + (size_t)fast_box_cells(w, h));
    hipLaunchKernelGGL(box_bin_kernel, dim3(nseq), dim3(256), lds, st, b, w, h);
    return hipGetLastError();
}

hipError_t launch_mask_boxes(int w, int h, const float* pts, const int* counts, int n, int pts_stride,
                             int nseq, float half, uint8_t* mask, hipStream_t st) {
    hipError_t e = hipMemsetAsync(mask, 255, (size_t)w * h * nseq, st);
    if (e != hipSuccess) return e;
    if (n > 0) hipLaunchKernelGGL(mask_boxes_kernel, dim3(n, nseq), dim3(64), 0, st, w, h, pts, counts, n,
                                  pts_stride, half, mask);
    return hipGetLastError();
}

}  // namespace svo
