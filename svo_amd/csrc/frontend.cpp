// Batched, device-resident tracking front end: the per-frame loop of
// Tracking::startStereo (R:src/tracking.cpp:232-276) for n_seq independent
// stereo sequences advanced in lockstep.
//
//   step(t), for every sequence s at once:
//     pyramid + Scharr of left frame t+1, pyramid of right t   [pyramid.hip]   (beside LK)
//     temporal LK  frame t-1 -> t (21x21, L3, 50 it)     [lk.hip]        trackFrames :154-179
//     mask of boxes around frame t-1's features + FAST   [fast.hip]      extractFeatures :74-92
//     (host) final SQPnP fits of step t-1 -> poses       [pose.cpp]      calculatePose :191-214
//     keyframe points of t-1 to the world frame, keep status == 1,
//       gather map points, first RANSAC subsets          [fe_kernels]    :169-175, :182-187, :141
//     RANSAC: host EPnP chunks <-> GPU scoring launches  [pose.cpp, pnp.hip] calculatePose :191-196
//     drop outliers + the keyframe's first corners       [fe_kernels]    :218-229
//     stereo LK of those corners into right frame t      [lk.hip]        findLeftFeaturesInRight :94-118
//     |yR - yL| < 40, DLT triangulation, z > 0, append   [fe_kernels]    triangulateNewMapPoints :120-152
//
// Which frames are keyframes: every frame, topping the set up to n_features
// (SVO_KF_EVERY, the benchmark), or Tracking::nextFrame's rule (SVO_KF_REFERENCE,
// :68-69) -- a per-sequence target (n_features or 0) the keyframe kernels read.
//
// FAST runs on the GPU beside LK; the host builds RANSAC hypotheses while the GPU
// scores; the final pose fits run on the host while the GPU tracks the next frame,
// so a keyframe's new map points stay in its camera frame until the next step
// moves them to the world frame with that pose (PendingMap, frontend.hpp).
//
// Streams (the box gives a process 4 hardware queues, GPU_MAX_HW_QUEUES): the
// LK stream (LK, post-LK, scoring, keyframe; highest priority), the FAST stream
// (box binning, FAST, speculative stereo LK; lowest), the context stream
// (pyramids, FAST pre-detection) and the copy stream (host copies, SQPnP
// statistics).
#include <pthread.h>
#include <sched.h>

#include <cctype>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "frontend.hpp"
#include "orb.hpp"
#include "linalg.hpp"
#include "pose.hpp"

namespace svo {

namespace {

// Persistent pool for the per-sequence host work (RANSAC hypotheses, pose fits).
// It runs a couple of times per step, microseconds apart: workers busy-poll a
// generation counter for a while after each job (spin_us, SVO_POOL_SPIN_US)
// before sleeping on a condition variable, so a dispatch normally costs no
// futex wake-up. The caller works too and spins on a counter of finished TASKS
// (a worker that wakes late with nothing left to take is not waited for).
// Tasks are claimed by CAS on one word holding (generation, task count, next
// index): a worker still holding a word of an older job -- generation AND count
// -- can never take (or skip) a task of a newer one, whatever the sizes of the
// two jobs (the count is not read from a second variable that a newer job may
// already have rewritten).
// Workers are pinned to `cpus` (the rank's share of the node, svo_host_cpu_plan)
// when it is non-empty. The spin is bounded below one step (SVO_POOL_SPIN_US,
// default 400 us): between the step's two pool jobs the workers stay hot, across
// an idle caller they sleep, so a rank does not burn its cores between steps.
class Pool {
   public:
    explicit Pool(int n, const std::vector<int>& cpus = {}) {
        const char* e = std::getenv("SVO_POOL_SPIN_US");
        spin_us_ = e ? std::atof(e) : 400.0;
        for (int i = 0; i < n; i++) {
            th_.emplace_back([this] { loop(); });
            if (!cpus.empty()) {
                cpu_set_t set;
                CPU_ZERO(&set);
                for (int c : cpus)
                    if (c >= 0 && c < CPU_SETSIZE) CPU_SET(c, &set);
                (void)pthread_setaffinity_np(th_.back().native_handle(), sizeof(set), &set);
            }
        }
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_.store(true);
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    int size() const { return (int)th_.size(); }
    // a job without tasks: sleeping workers wake and every worker starts a new
    // spin window, so a job expected shortly finds them hot (no futex wake-up)
    void prime() {
        if (th_.empty()) return;
        publish(0);
    }
    void run(int n, const std::function<void(int)>& fn) {
        if (th_.empty() || n <= 1 || n > (int)kFieldMask) {
            for (int i = 0; i < n; i++) fn(i);
            return;
        }
        fn_ = &fn;
        done_.store(0, std::memory_order_relaxed);
        const uint64_t g = publish(n);  // the release store of the job word publishes fn_ / done_
        work(g);
        while (done_.load(std::memory_order_acquire) < n) pause();
    }

   private:
    // job word: generation (24 bits) | task count (20) | next index (20)
    static constexpr int kFieldBits = 20;
    static constexpr uint64_t kFieldMask = (1ull << kFieldBits) - 1;
    static constexpr uint64_t kGenMask = (1ull << (64 - 2 * kFieldBits)) - 1;
    static uint64_t gen_of(uint64_t v) { return v >> (2 * kFieldBits); }
    static uint64_t cnt_of(uint64_t v) { return (v >> kFieldBits) & kFieldMask; }
    static uint64_t idx_of(uint64_t v) { return v & kFieldMask; }
    // a new job of n tasks: its word replaces the old one in a single store, so a
    // stale CAS (old generation and count) fails from here on
    uint64_t publish(int n) {
        const uint64_t g = (gen_.load(std::memory_order_relaxed) + 1) & kGenMask;
        next_.store((g << (2 * kFieldBits)) | ((uint64_t)n << kFieldBits), std::memory_order_release);
        {
            std::lock_guard<std::mutex> lk(mu_);
            gen_.store(g, std::memory_order_release);
        }
        if (sleeping_.load(std::memory_order_acquire) > 0) cv_.notify_all();
        return g;
    }
    static void pause() {
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
    }
    void work(uint64_t g) {
        for (;;) {
            uint64_t v = next_.load(std::memory_order_acquire);
            if (gen_of(v) != g || idx_of(v) >= cnt_of(v)) return;
            if (!next_.compare_exchange_weak(v, v + 1, std::memory_order_acq_rel)) continue;
            (*fn_)((int)idx_of(v));
            done_.fetch_add(1, std::memory_order_acq_rel);
        }
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            const auto t0 = std::chrono::steady_clock::now();
            int k = 0;
            while (gen_.load(std::memory_order_acquire) == seen && !stop_.load(std::memory_order_relaxed)) {
                pause();
                if (++k == 256) {
                    k = 0;
                    if (std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() >
                        spin_us_)
                        break;
                }
            }
            if (gen_.load(std::memory_order_acquire) == seen && !stop_.load()) {
                std::unique_lock<std::mutex> lk(mu_);
                sleeping_.fetch_add(1);
                cv_.wait(lk, [&] { return stop_.load() || gen_.load() != seen; });
                sleeping_.fetch_sub(1);
            }
            if (stop_.load()) return;
            seen = gen_.load(std::memory_order_acquire);
            work(seen);
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_;
    const std::function<void(int)>* fn_ = nullptr;
    std::atomic<uint64_t> next_{0}, gen_{0};
    std::atomic<int> done_{0}, sleeping_{0};
    std::atomic<bool> stop_{false};
    double spin_us_ = 400.0;
};

// ---- host core plan (svo_host_cpu_plan) ----
std::vector<int> parse_cpulist(const std::string& txt) {  // "0-3,8,10-11"
    std::vector<int> out;
    std::stringstream ss(txt);
    std::string tok;
    while (std::getline(ss, tok, ',')) {
        if (tok.empty() || tok[0] == '\n') continue;
        const size_t dash = tok.find('-');
        const int a = std::atoi(tok.c_str());
        const int b = dash == std::string::npos ? a : std::atoi(tok.c_str() + dash + 1);
        for (int c = a; c <= b; c++) out.push_back(c);
    }
    return out;
}

// NUMA node of every CPU id (-1: unknown), from /sys/devices/system/node
std::vector<int> cpu_nodes(int max_cpu) {
    std::vector<int> node((size_t)max_cpu + 1, -1);
    for (int m = 0; m < 64; m++) {
        std::ifstream f("/sys/devices/system/node/node" + std::to_string(m) + "/cpulist");
        if (!f) continue;
        std::string txt;
        std::getline(f, txt);
        for (int c : parse_cpulist(txt))
            if (c >= 0 && c <= max_cpu) node[c] = m;
    }
    return node;
}

std::vector<int> host_cpu_plan(int rank, int world, const int* gpu_node) {
    cpu_set_t set;
    CPU_ZERO(&set);
    std::vector<int> allowed;
    if (sched_getaffinity(0, sizeof(set), &set) == 0)
        for (int c = 0; c < CPU_SETSIZE; c++)
            if (CPU_ISSET(c, &set)) allowed.push_back(c);
    if (allowed.empty() || world <= 0 || rank < 0 || rank >= world) return {};
    const std::vector<int> node = cpu_nodes(allowed.back());
    std::stable_sort(allowed.begin(), allowed.end(), [&](int a, int b) { return node[a] < node[b]; });
    auto split = [](const std::vector<int>& cpus, int idx, int k) {
        std::vector<int> out;
        const int m = (int)cpus.size();
        if (m == 0 || k <= 0) return out;
        if (m < k) {  // fewer CPUs than ranks: shared, one each
            out.push_back(cpus[idx % m]);
            return out;
        }
        const int lo = (int)((int64_t)m * idx / k), hi = (int)((int64_t)m * (idx + 1) / k);
        out.assign(cpus.begin() + lo, cpus.begin() + hi);
        return out;
    };
    if (gpu_node && gpu_node[rank] >= 0) {
        // the ranks whose GPUs sit on this rank's node share that node's CPUs
        const int my = gpu_node[rank];
        int idx = 0, k = 0;
        for (int r = 0; r < world; r++)
            if (gpu_node[r] == my) {
                if (r < rank) idx++;
                k++;
            }
        std::vector<int> local;
        for (int c : allowed)
            if (node[c] == my) local.push_back(c);
        if ((int)local.size() >= k) return split(local, idx, k);
    }
    return split(allowed, rank, world);
}

// LOCAL_RANK / LOCAL_WORLD_SIZE as torch.distributed.run sets them (one process per GPU)
int local_rank_env() {
    const char* e = std::getenv("LOCAL_RANK");
    return e ? std::max(0, std::atoi(e)) : 0;
}
int local_world_env() {
    const char* e = std::getenv("LOCAL_WORLD_SIZE");
    return e ? std::max(1, std::atoi(e)) : 1;
}

// host-side step trace (SVO_FE_TRACE=1, read when a front end is created): label
// + microseconds since step start
bool trace_env() {
    const char* e = std::getenv("SVO_FE_TRACE");
    return e && e[0] == '1';
}

// final SQPnP fits on the device (SVO_FE_DEVICE_FITS=1, read at create) instead of
// the host pool (launch_sqpnp_fit: the eigen-decomposition, the SQP runs over
// waves, the search). The host's fits take ~0.17 ms per step and hide behind the
// wait for the post-LK results, while the device's run beside LK and take its
// CUs (DESIGN.md §6 has the measurements), so the host is the default
bool device_fits_env() {
    const char* e = std::getenv("SVO_FE_DEVICE_FITS");
    return e && e[0] == '1';
}

// NUMA node of HIP device d (-1: unknown), from its PCI address in sysfs
int device_numa_node(int d) {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), d) != hipSuccess) return -1;
    std::string id(bus);
    for (auto& ch : id) ch = (char)std::tolower((unsigned char)ch);
    std::ifstream f("/sys/bus/pci/devices/" + id + "/numa_node");
    int v = -1;
    if (f) f >> v;
    return v;
}

constexpr int kPhases = 10;
enum Phase { PH_PYR, PH_LK, PH_POST, PH_STEREO, PH_PNP, PH_TAIL, PH_FAST, PH_BUCKET, PH_APPEND, PH_PYR_R };

// floor of the first RANSAC hypothesis chunk: a floor of 1 saves an EPnP per
// sequence when one hypothesis is predicted, but the misses' extra scoring
// rounds measured 2-6 % slower on the KITTI bench
constexpr int kChunk0 = 2;

}  // namespace

}  // namespace svo

using namespace svo;

struct svo_frontend {
    svo_ctx* ctx = nullptr;
    svo_frontend_config cfg{};
    int S = 0, T = 0, CAP = 0, MAPCAP = 0, WORDS = 0, KCAP = 0, BCAP = 0;
    int W = 0, H = 0, nlev = 0, ml = 0, ml_st = 0;
    size_t npx = 0, bscr = 0;
    std::vector<svo_image*> frames;    // left  [s*T + t]
    std::vector<svo_image*> frames_r;  // right [s*T + t]
    std::vector<PyrDesc> desc_host;    // [t*S + s]
    std::vector<PyrDesc> desc_r_host;  // [t*S + s]
    PyrDesc* d_desc = nullptr;         // [t][s]
    PyrDesc* d_desc_r = nullptr;       // [t][s]
    void* dermem = nullptr;          // Scharr pyramids of frames t-1, t, t+1: [3][s], frame f in f % 3
    DerivDesc* d_der = nullptr;      // [3][s]
    // device state (one allocation)
    void* dmem = nullptr;
    float *xyA, *next_xy, *xyB, *obj, *kps, *cand, *box_binned;
    float *st_xy, *st_next;  // keyframe candidates (left) and their stereo LK matches (right)
    uint8_t* st_status;
    float4* st_X;  // stereo_tri_kernel's points of the speculative candidates
    int* box_band;
    int *midA, *midB, *nA, *nB, *iters, *kn, *bn, *map_n, *rowcnt, *rowoff, *scr, *added, *st_n;
    int *pend0, *pend_n;  // PendingMap ranges
    int* spec_n;          // speculative stereo candidates per sequence (StereoPrepBatch)
    int spec_margin = 32;  // RANSAC drops covered by the speculative stereo LK (SVO_FE_SPEC_MARGIN, < 0: off)
    int min_tracked = 0;   // min over sequences of the last step's tracked count (stereo LK grid hint)
    // early speculation (SVO_FE_SPEC_EARLY=1, the default; SVO_KF_EVERY only): the
    // speculative stereo LK of step t goes out in its first half, behind FAST(t),
    // sized from the features before LK (nA) with margin spec_margin + lk_loss
    int spec_early = 1;
    bool trace = false;  // SVO_FE_TRACE=1 at create
    bool device_fits = false;  // SVO_FE_DEVICE_FITS=1 at create (device_fits_env)
    void* fit_work = nullptr;  // device_fits: sqpnp_fit_work_bytes(S)
    OrbBatch* orb = nullptr;   // cfg.use_orb: the keyframe detector (orb_batch_detect)
    std::vector<ImgLevel> orb_lv0;
    std::vector<int> orb_over;
    int spec_t = -1;       // step whose speculation went out early
    int spec_m = 0;        // its margin (features lost to LK + RANSAC it covers)
    bool spec_was_early = false;
    int lk_loss = 0;       // max over sequences of the last step's LK losses
    int ransac_drop = 0;   // max over sequences of the last step's RANSAC drops
    double post_wait_ms = 0;  // running estimate of the host's wait for the post-LK results
    unsigned long long* fbits;
    uint8_t* status;
    double* map;
    // the tracked-point arrays of a step (xyB, obj, nB) and its inlier bits are
    // double-buffered by step parity: the side work of step t (SQPnP statistics,
    // full copy to the host) reads them while step t+1 already runs
    float *xyB_b[2], *obj_b[2];
    int* nB_b[2];
    int front_t = -1;  // step whose first half (LK .. FAST) is already enqueued
    // host mirrors (pinned): the full point copies for the fits and long RANSAC runs
    void* hmem = nullptr;
    float *h_xyB, *h_obj;  // this step's parity half of h_*_b
    float *h_xyB_b[2], *h_obj_b[2];
    // host-coherent memory the kernels write / read directly (no D2H copies on
    // the critical path): post-LK counts / iteration sums / RANSAC subsets, the
    // keyframe's counts, the inlier bits, statistics, poses, keyframe targets
    void* zout = nullptr;
    int *h_nB, *h_nA, *h_added, *h_target, *h_over;
    long long* h_itsum;
    float* h_samp;
    double *h_stats, *h_pose;   // h_pose: [s][12] camera -> world of the last fitted frame
    double* h_pose6;            // [s][6] rvec, tvec of the last fitted frame (launch_sqpnp_fit)
    SqpnpFitIn* h_fitin;        // [s] the host RANSAC's outcome the device fit starts from
    uint32_t* h_best;           // this step's parity of h_best_b
    uint32_t* h_best_b[2];
    // host-coherent buffers the scoring kernel reads / writes directly (zero-copy:
    // no H2D of the hypotheses, no D2H of bits / counts, no count memset)
    void* zmem = nullptr;
    double* z_hyps = nullptr;     // [s][kRansacChunk][12]
    uint32_t* z_bits = nullptr;   // [s][kRansacChunk][WORDS]
    int* z_cnt = nullptr;         // [s][kRansacChunk] inliers per hypothesis
    std::vector<RansacSeq> rs;
    std::vector<int> pred_iters;  // [s] RANSAC hypotheses the last frame's outlier ratio implies
    std::vector<uint8_t> kf_prev; // [s] the last frame was a keyframe (SVO_KF_REFERENCE)
    // FAST pre-detection (SVO_FE_FAST_PRE=1, the default): frame t+1's detection +
    // NMS without the box mask queued in step t on the context stream (0: FAST
    // detection behind LK(t) on the FAST stream)
    int fast_pre = 1;
    // SVO_FE_PRE_AFTER_POST (default 1): the pre-detection of frame t+1 and its right
    // pyramid are queued behind step t's post-LK (fe_post) instead of behind frame
    // t+1's left pyramid, so that they cannot take the CUs ahead of the critical
    // post-LK when LK runs long (the forward scene: +3 %; the headline: neutral)
    int pre_after_post = 1;
    int pre_pending = -1;          // frame whose pre-detection waits for fe_post
    bool stats_in_tail = false;    // the next fe_keyframe computes the pending SQPnP statistics
    int pre_t = -1;                // frame whose unmasked detection sits in fbits / rowcnt / score_map
    hipEvent_t ev_pre = nullptr;   // that detection done (context stream)
    hipEvent_t ev_fdone = nullptr; // this step's FAST chain done (FAST stream)
    std::vector<double> pose;  // [s][6]
    bool fits_pending = false;
    bool stats_pending = false;
    int stats_parity = 0;  // step parity whose inliers the pending statistics cover
    bool boxes_binned = false;  // box_bin already queued for the next step's FAST
    int pyr_ready = -1;  // frame index whose pyramid + Scharr were built ahead
    hipEvent_t ev_stats = nullptr;  // SQPnP statistics + final fits of the last step done (copy stream)
    // full copies of the tracked points / map points (h_xyB, h_obj): needed only by
    // the final fits, RANSAC past the prefetched subsets and the n <= 5 solve, so
    // they travel on their own stream once requested
    hipStream_t st_copy = nullptr;
    hipEvent_t ev_full = nullptr;  // this step's parity of ev_full_b
    hipEvent_t ev_full_b[2] = {nullptr, nullptr};
    hipEvent_t ev_pyr_r_b[2] = {nullptr, nullptr};  // right pyramid of frame f built: [f & 1]
    int pyr_r_ready = -1;  // frame whose right pyramid was built ahead (in the previous step)
    bool full_queued = false;
    int fit_parity = 0;  // step parity whose RANSAC results the pending fits refine
    uint8_t* score_map = nullptr;  // [s][npx] FAST scores of the kept corners
    Pool* pool = nullptr;
    std::vector<int> host_cpus;  // the pool's pinned CPU set (svo_host_cpu_plan)
    hipStream_t st_lk = nullptr;    // LK, post-LK, scoring, keyframe (highest priority)
    hipStream_t st_fast = nullptr;  // box binning + FAST + bucket + speculative stereo LK (lowest)
    hipEvent_t ev_pyr = nullptr;    // left pyramid of the step's frame built
    hipEvent_t ev_fast = nullptr;   // FAST (and the speculative stereo LK behind it) done
    hipEvent_t ev_lk = nullptr, ev_post = nullptr, ev_tail = nullptr;
    // timing
    hipEvent_t ev[256];
    double phase_ms[kPhases] = {0};
    int64_t phase_n[kPhases] = {0};
    std::vector<std::pair<int, int>> pending;  // (phase, event pair index)
    int ev_used = 0;
    // streamed frames (svo_frontend_queue_frames): pinned H2D of a step's stereo
    // pairs on their own stream into a device staging block (double-buffered by
    // frame parity), the conversion kernel into level 0 of the frame's ring slot;
    // the pyramid builds of that frame wait for ev_up[slot]
    hipStream_t st_up = nullptr;
    uint8_t* up_stage = nullptr;       // [2 side][S x up_cap]: the host frames' bytes (copy and conversion
                                       // run in order on st_up, so one block serves every frame)
    size_t up_cap = 0;                 // staging bytes per sequence (the widest h * stride seen)
    size_t up_seq = 0;                 // h * stride of the last queued frame (sequence stride in staging)
    std::vector<hipEvent_t> ev_up;     // [T] conversion of the slot's frame done
    std::vector<int> up_t;             // [T] frame last streamed into the slot (-1: none)
    std::vector<hipEvent_t> ev_free;   // [T] the slot's frame f read for the last time (after LK(f + 1))
    std::vector<char> free_rec;        // [T] ev_free recorded since the slot was last queued
    int stepped = -1;                  // last completed step (init: t0); -1 before init
};

namespace {

// Phase timing: event pairs from a ring; a pair is folded into the totals once
// its end event has completed (work that runs into the next step is collected
// then), so timing never adds a synchronisation.
constexpr int kEvRing = (int)(sizeof(((svo_frontend*)nullptr)->ev) / sizeof(hipEvent_t));

void ph_fold(svo_frontend* fe, bool wait) {
    std::vector<std::pair<int, int>> keep;
    for (auto& p : fe->pending) {
        if (wait) (void)hipEventSynchronize(fe->ev[p.second + 1]);
        float ms = 0.f;
        const hipError_t e = hipEventElapsedTime(&ms, fe->ev[p.second], fe->ev[p.second + 1]);
        if (e == hipSuccess) {
            fe->phase_ms[p.first] += ms;
            fe->phase_n[p.first] += 1;
        } else if (e == hipErrorNotReady) {
            keep.push_back(p);
        }
    }
    fe->pending.swap(keep);
}

void ph_begin(svo_frontend* fe, int ph, hipStream_t st, int* slot) {
    *slot = -1;
    if (!fe->cfg.timing) return;
    // timing 2: only the big phases (each event pair costs a few us of host time)
    if (fe->cfg.timing == 2 && ph != PH_LK && ph != PH_PYR && ph != PH_FAST && ph != PH_STEREO && ph != PH_PYR_R)
        return;
    if (fe->cfg.timing == 3 && ph != PH_LK) return;  // timing 3: the LK launches only (the roofline's)
    const int sl = fe->ev_used;
    bool wrapped = false;  // ring wrapped onto a pair still in flight
    for (const auto& p : fe->pending) wrapped |= p.second == sl;
    if (wrapped) ph_fold(fe, true);
    fe->ev_used = (fe->ev_used + 2) % kEvRing;
    *slot = sl;
    (void)hipEventRecord(fe->ev[sl], st);
    fe->pending.push_back({ph, sl});
}
void ph_end(svo_frontend* fe, hipStream_t st, int slot) {
    if (slot >= 0) (void)hipEventRecord(fe->ev[slot + 1], st);
}
void ph_collect(svo_frontend* fe) { ph_fold(fe, false); }

template <class T>
T* carve(char*& p, size_t count) {
    p = (char*)(((uintptr_t)p + 255) & ~(uintptr_t)255);
    T* r = (T*)p;
    p += sizeof(T) * count;
    return r;
}

FastDetBatch fe_fast_batch(svo_frontend* fe, const PyrDesc* descs_cur, bool use_mask) {
    FastDetBatch fb{descs_cur, nullptr, fe->fbits, fe->rowcnt, fe->rowoff,
                    (svo_keypoint*)fe->kps, fe->kn, fe->npx, (fe->W + 63) / 64, fe->KCAP};
    fb.score_map = fe->score_map;
    fb.padded = true;  // the frames are svo_image levels
    if (use_mask) {  // boxes around the previous frame's features, rasterised per FAST tile
        fb.box_pts = fe->xyA;
        fb.box_counts = fe->nA;
        fb.box_stride = fe->CAP;
        fb.box_half = fe->cfg.mask_half;
        fb.box_binned = fe->box_binned;
        fb.box_band = fe->box_band;
    }
    return fb;
}

int fe_fast_and_bucket(svo_frontend* fe, const PyrDesc* descs_cur, bool use_mask, hipStream_t st,
                       bool prebinned = false, int stage = kFastAll) {
    svo_ctx* ctx = fe->ctx;
    int slot;
    FastDetBatch fb = fe_fast_batch(fe, descs_cur, use_mask);
    fb.box_prebinned = prebinned;
    ph_begin(fe, PH_FAST, st, &slot);
    SVO_HIP(ctx, launch_fast_detect(fb, fe->S, fe->W, fe->H, fe->cfg.fast_threshold, fe->cfg.fast_nonmax, st, stage));
    ph_end(fe, st, slot);
    if (stage == kFastDetect) return SVO_OK;
    if (fe->cfg.bucket_size > 0) {
        ph_begin(fe, PH_BUCKET, st, &slot);
        BucketBatch bb{fe->kps, 3, fe->KCAP, fe->kn, 0, nullptr, fe->cand, nullptr, fe->BCAP, fe->bn, fe->scr,
                       fe->bscr};
        SVO_HIP(ctx, launch_bucket(bb, fe->S, fe->W, fe->H, fe->cfg.bucket_size, fe->cfg.per_bucket, st));
        ph_end(fe, st, slot);
    }
    return SVO_OK;
}

// ORB keyframe detection of frame t of every sequence (cfg.use_orb): its keypoints
// into kps / kn where FAST's would go, with the box mask around xyA / nA (the
// previous frame's features, R:src/tracking.cpp:76-79) unless use_mask is false.
// Synchronous (orb_batch_detect: device stages, then the host's retainBest).
int fe_orb_detect(svo_frontend* fe, int t, bool use_mask, hipStream_t st) {
    svo_ctx* ctx = fe->ctx;
    const int S = fe->S;
    for (int s = 0; s < S; s++) fe->orb_lv0[s] = fe->desc_host[(size_t)(t % fe->T) * S + s].lv[0];
    auto par = [fe](int n, const std::function<void(int)>& fn) { fe->pool->run(n, fn); };
    SVO_HIP(ctx, orb_batch_detect(fe->orb, fe->orb_lv0.data(), use_mask ? fe->xyA : nullptr, fe->nA, fe->CAP, fe->CAP,
                                  fe->cfg.mask_half, (svo_keypoint*)fe->kps, fe->kn, fe->KCAP, st, par,
                                  fe->orb_over.data()));
    return SVO_OK;
}

// FAST pre-detection: frame tn's FAST detection + NMS without the box mask (the
// mask drops corners after NMS, so it can wait for frame tn-1's features) queued
// on the context stream once the current step's FAST chain has consumed the row
// words (ev_fdone); step tn keeps only the box filter, the recount, scan and emit
// behind its LK (kFastBoxes). NB: from here on the context stream -- the next
// right pyramid and the pyramid after next, both queued behind this detection --
// is serialised behind FAST(tn-1)'s chain on the low-priority FAST stream.
int fe_queue_pre(svo_frontend* fe, int tn) {
    svo_ctx* ctx = fe->ctx;
    hipStream_t st = ctx->stream;
    const PyrDesc* dnext = fe->d_desc + (size_t)(tn % fe->T) * fe->S;
    SVO_HIP(ctx, hipStreamWaitEvent(st, fe->ev_fdone, 0));
    FastDetBatch fb = fe_fast_batch(fe, dnext, false);
    SVO_HIP(ctx, launch_fast_detect(fb, fe->S, fe->W, fe->H, fe->cfg.fast_threshold, fe->cfg.fast_nonmax, st,
                                    kFastDetect));
    SVO_HIP(ctx, hipEventRecord(fe->ev_pre, st));
    fe->pre_t = tn;
    return SVO_OK;
}

// findLeftFeaturesInRight: calcOpticalFlowPyrLK(left, right, pts, 11x11, 3,
// {COUNT+EPS, 30, 0.001}), flags 0 (R:src/tracking.cpp:97-105) of st_xy[0,
// counts[s]) of every sequence of frame t; max_n bounds every count (the grid).
int fe_stereo_lk(svo_frontend* fe, int t, const int* counts, int max_n, hipStream_t st, int grid_hint = 0) {
    svo_ctx* ctx = fe->ctx;
    const svo_frontend_config& c = fe->cfg;
    int slot;
    SVO_HIP(ctx, hipStreamWaitEvent(st, fe->ev_pyr_r_b[t & 1], 0));
    const PyrDesc* dl = fe->d_desc + (size_t)(t % fe->T) * fe->S;
    const PyrDesc* dr = fe->d_desc_r + (size_t)(t % fe->T) * fe->S;
    LKBatch lb{dl, dr, fe->d_der + (size_t)(t % 3) * fe->S, fe->st_xy, fe->st_next, fe->st_status, nullptr, nullptr,
               counts, 0, fe->CAP};
    lb.grid_hint = grid_hint;
    LKParams lp;
    lp.win_w = lp.win_h = c.stereo_win;
    lp.max_level = fe->ml_st;
    lp.max_count = std::min(std::max(c.stereo_max_count, 0), 100);
    const double eps = std::min(std::max(c.stereo_epsilon, 0.0), 10.0);
    lp.eps2 = eps * eps;
    lp.flags = 0;
    lp.cv_order = (c.lk_flags & SVO_LK_OPENCV_ORDER) ? 1 : 0;  // the config's order for both LK calls
    lp.min_eig = (float)c.min_eig;
    lp.want_err = 0;
    lk_apply_env(lp);
    ph_begin(fe, PH_STEREO, st, &slot);
    SVO_HIP(ctx, launch_lk(lb, fe->S, std::min(std::max(max_n, 0), fe->CAP), lp, st));
    ph_end(fe, st, slot);
    return SVO_OK;
}

// stereo_tri_kernel's inputs for the candidates st_xy[0, counts[s]) (the
// speculative ones: spec_n; the serial keyframe's take: st_n)
StereoTriBatch fe_tri_batch(svo_frontend* fe, const int* counts) {
    const svo_frontend_config& c = fe->cfg;
    StereoTriBatch tb;
    tb.st_xy = fe->st_xy;
    tb.st_next = fe->st_next;
    tb.st_status = fe->st_status;
    tb.spec_n = counts;
    tb.cap = fe->CAP;
    tb.y_threshold = c.y_threshold;
    std::memcpy(tb.P, c.P_left, sizeof(float) * 12);
    std::memcpy(tb.P + 12, c.P_right, sizeof(float) * 12);
    tb.st_X = fe->st_X;
    return tb;
}

// The keyframe of every sequence on stream st (R:src/tracking.cpp:247-255):
// outlier compaction (inlier bits `bits`, or every point when n_in is all zero)
// + the first candidates up to the sequence's target (h_target: n_features on a
// keyframe, 0 otherwise) (tail_kernel), their stereo LK into the right frame t
// (findLeftFeaturesInRight), then filter + triangulation + append
// (append_kernel). xy_in / mid_in / n_in: the step's tracked points (compacted
// into xyA / midA / nA). max_take: a host bound on every sequence's candidate
// count (the stereo LK grid). spec: the speculative stereo LK (fe_queue_spec)
// already matched every sequence's take candidates: compaction, filter,
// triangulation and append run as one kernel.
int fe_keyframe(svo_frontend* fe, int t, const int* n_in, const uint32_t* bits, const float* xy_in, const int* mid_in,
                int max_take, hipStream_t st, bool spec = false) {
    svo_ctx* ctx = fe->ctx;
    const svo_frontend_config& c = fe->cfg;
    int slot;
    const bool bucketed = c.bucket_size > 0;
    TailBatch tb;
    tb.n_in = n_in;
    tb.bits = bits;
    tb.words_cap = fe->WORDS;
    tb.xy_in = xy_in;
    tb.mid_in = mid_in;
    tb.xy_out = fe->xyA;
    tb.mid_out = fe->midA;
    tb.n_out = fe->nA;
    tb.cap = fe->CAP;
    tb.n_target = fe->h_target;
    tb.cand = bucketed ? fe->cand : fe->kps;
    tb.cand_elem = bucketed ? 2 : 3;
    tb.cand_cap = bucketed ? fe->BCAP : fe->KCAP;
    tb.cand_n = bucketed ? fe->bn : fe->kn;
    tb.map_n = fe->map_n;
    tb.map_cap = fe->MAPCAP;
    tb.st_xy = fe->st_xy;
    tb.st_n = fe->st_n;
    tb.h_over = fe->h_over;
    if (fe->stats_in_tail) {
        // the pending SQPnP statistics of these inliers (the step's bits and points)
        tb.stats_obj = fe->obj_b[fe->stats_parity];
        tb.stats_out = fe->h_stats;
        tb.ifx = 1. / c.K[0];
        tb.ify = 1. / c.K[4];
        tb.cx = c.K[2];
        tb.cy = c.K[5];
        fe->stats_in_tail = false;
    }
    AppendBatch ab;
    ab.n = fe->nA;
    ab.xy = fe->xyA;
    ab.mid = fe->midA;
    ab.cap = fe->CAP;
    ab.st_xy = fe->st_xy;
    ab.st_n = fe->st_n;
    ab.map = fe->map;
    ab.map_n = fe->map_n;
    ab.map_cap = fe->MAPCAP;
    ab.pend0 = fe->pend0;
    ab.pend_n = fe->pend_n;
    ab.added = fe->added;
    ab.h_n = fe->h_nA;
    ab.h_added = fe->h_added;
    ab.st_X = fe->st_X;
    if (spec) {
        ph_begin(fe, PH_TAIL, st, &slot);
        SVO_HIP(ctx, launch_keyframe_fused(tb, ab, fe->S, st));
        ph_end(fe, st, slot);
        return SVO_OK;
    }
    ph_begin(fe, PH_TAIL, st, &slot);
    SVO_HIP(ctx, launch_tail(tb, fe->S, st));
    ph_end(fe, st, slot);
    int rc = fe_stereo_lk(fe, t, fe->st_n, max_take, st);
    if (rc) return rc;
    // the take's filter + DLT (the same kernel as behind the speculative stereo
    // LK), then the append compacts
    SVO_HIP(ctx, launch_stereo_tri(fe_tri_batch(fe, fe->st_n), fe->S, max_take, st));
    ph_begin(fe, PH_APPEND, st, &slot);
    SVO_HIP(ctx, launch_append(ab, fe->S, st));
    ph_end(fe, st, slot);
    return SVO_OK;
}

// The speculative stereo LK of step t (StereoPrepBatch) on the FAST stream,
// behind FAST (the candidates). The keyframe takes the first target - kept
// candidates, kept <= n_ref, so the first target - n_ref + margin cover the take
// whenever n_ref - kept <= margin. Two forms:
//  - early (fe_front, behind FAST(t)): n_ref = the features before LK (nA, final
//    once the FAST stream has waited for the last keyframe), margin = spec_margin
//    + the last step's largest LK loss; it runs beside LK(t), so the keyframe
//    never waits for it (SVO_KF_EVERY only: the targets of a later step are not
//    known while its first half is queued);
//  - late (fe_post, behind the post-LK): n_ref = the tracked counts (nB), margin
//    = spec_margin; it runs beside the host's RANSAC.
// ev_fast is re-recorded behind it, so the keyframe's wait for FAST covers it too.
int fe_queue_spec(svo_frontend* fe, int t, bool early) {
    svo_ctx* ctx = fe->ctx;
    const svo_frontend_config& c = fe->cfg;
    hipStream_t sf = fe->st_fast;
    const bool bucketed = c.bucket_size > 0;
    // spec_margin is the slack over the last step's losses: an outlier-heavy
    // sequence (the forward / occluder scene drops ~100 of 2000 points a frame)
    // would otherwise miss the speculation every step and run the serial keyframe
    // (capped: a sequence whose RANSAC failed dropped everything)
    const int margin = fe->spec_margin + std::min(fe->ransac_drop, c.n_features / 4) + (early ? fe->lk_loss : 0);
    StereoPrepBatch pb;
    pb.n_tracked = early ? fe->nA : fe->nB;
    pb.cand = bucketed ? fe->cand : fe->kps;
    pb.cand_elem = bucketed ? 2 : 3;
    pb.cand_cap = bucketed ? fe->BCAP : fe->KCAP;
    pb.cand_n = bucketed ? fe->bn : fe->kn;
    pb.map_n = fe->map_n;
    pb.map_cap = fe->MAPCAP;
    pb.cap = fe->CAP;
    pb.n_target = fe->h_target;
    pb.margin = margin;
    pb.st_xy = fe->st_xy;
    pb.spec_n = fe->spec_n;
    if (!early) SVO_HIP(ctx, hipStreamWaitEvent(sf, fe->ev_post, 0));
    SVO_HIP(ctx, launch_stereo_prep(pb, fe->S, sf));
    // grid for the speculation the last step's smallest tracked count implies
    // (+ slack); the kernel's waves loop over any candidates beyond it
    const int max_spec = std::min(c.n_features + margin, fe->CAP);
    const int hint = std::min(fe->CAP, c.n_features - fe->min_tracked + margin + 32);
    int rc = fe_stereo_lk(fe, t, fe->spec_n, max_spec, sf, hint);
    if (rc) return rc;
    SVO_HIP(ctx, launch_stereo_tri(fe_tri_batch(fe, fe->spec_n), fe->S, hint, sf));
    SVO_HIP(ctx, hipEventRecord(fe->ev_fast, sf));
    fe->spec_t = t;
    fe->spec_m = margin;
    fe->spec_was_early = early;
    return SVO_OK;
}

PendingMap fe_pending(svo_frontend* fe) {
    return PendingMap{fe->map, fe->MAPCAP, fe->pend0, fe->pend_n, fe->h_pose};
}

// Frame::pose() of a fitted frame (R:src/tracking.cpp:198-214): the inverse of
// the solvePnPRansac model [R(rvec) | tvec] (svo::SE3d::inverse), identity
// when RANSAC found no model (rvec = tvec = 0, as the host mirror)
void fe_set_pose(svo_frontend* fe, int s, bool ok, const double rvec[3], const double tvec[3]) {
    double* T = fe->h_pose + 12 * (size_t)s;
    double R[9];
    const double zero[3] = {0, 0, 0};
    if (!ok) {
        rvec = zero;
        tvec = zero;
    }
    la::rodrigues(rvec, R);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) T[3 * i + j] = R[3 * j + i];
    for (int i = 0; i < 3; i++) T[9 + i] = -(T[3 * i] * tvec[0] + T[3 * i + 1] * tvec[1] + T[3 * i + 2] * tvec[2]);
}

// Full D2H of the step's tracked points and map points (after the post-LK), on
// the copy stream; queued once per step, when first needed or at the step's end.
int fe_queue_full(svo_frontend* fe) {
    if (fe->full_queued) return SVO_OK;
    svo_ctx* ctx = fe->ctx;
    const size_t S = fe->S, CAP = fe->CAP;
    SVO_HIP(ctx, hipStreamWaitEvent(fe->st_copy, fe->ev_post, 0));
    SVO_HIP(ctx, hipMemcpyAsync(fe->h_xyB, fe->xyB, sizeof(float) * 2 * S * CAP, hipMemcpyDeviceToHost, fe->st_copy));
    SVO_HIP(ctx, hipMemcpyAsync(fe->h_obj, fe->obj, sizeof(float) * 3 * S * CAP, hipMemcpyDeviceToHost, fe->st_copy));
    SVO_HIP(ctx, hipEventRecord(fe->ev_full, fe->st_copy));
    fe->full_queued = true;
    return SVO_OK;
}

// Queue the SQPnP sufficient statistics of the last step's RANSAC inliers on the
// copy stream, written straight to host-coherent memory. The inputs -- inlier
// bits on the host, points from the post-LK kernel the host already waited for
// -- need no device-side wait, so they are queued right behind the keyframe and
// run beside it, ahead of the next LK (a kernel queued beside a running LK waits
// for it: LK leaves no registers free).
int fe_queue_stats(svo_frontend* fe) {
    if (!fe->stats_pending) return SVO_OK;
    svo_ctx* ctx = fe->ctx;
    const int p = fe->stats_parity;
    SVO_HIP(ctx, launch_suffstats(fe->obj_b[p], fe->xyB_b[p], fe->nB_b[p], fe->CAP, fe->h_best_b[p], fe->WORDS, fe->S,
                                  fe->cfg.K, fe->h_stats, fe->st_copy));
    // and, with device_fits, the final SQPnP fits from them on the device: the next
    // post-LK (which moves the keyframe's new map points with these poses) then
    // waits for ev_stats
    if (fe->device_fits)
        SVO_HIP(ctx, launch_sqpnp_fit(fe->h_stats, fe->h_fitin, fe->obj_b[p], fe->nB_b[p], fe->CAP, fe->h_best_b[p],
                                      fe->WORDS, fe->S, fe->h_pose6, fe->h_pose, fe->fit_work, fe->st_copy));
    SVO_HIP(ctx, hipEventRecord(fe->ev_stats, fe->st_copy));
    fe->stats_pending = false;
    return SVO_OK;
}

// Final SQPnP-objective fits of the last step (from the GPU sufficient
// statistics in h_stats): they refine the reported poses, so they run lazily --
// at the next step while the GPU tracks, or when a pose is read. With
// device_fits they ran on the device behind the statistics (fe_queue_stats) and
// the host only reads their poses.
double fe_finish_fits(svo_frontend* fe) {
    if (!fe->fits_pending) return 0.0;
    auto t0 = std::chrono::steady_clock::now();
    (void)hipEventSynchronize(fe->ev_stats);
    if (fe->device_fits) {
        std::memcpy(fe->pose.data(), fe->h_pose6, sizeof(double) * 6 * (size_t)fe->S);
    } else {
        (void)hipEventSynchronize(fe->ev_full_b[fe->fit_parity]);  // cheirality test reads h_obj
        fe->pool->run(fe->S, [&](int s) {
            RansacSeq& r = fe->rs[s];
            r.fit(fe->cfg.K, fe->h_stats + kSqpnpStats * (size_t)s);
            double* P = &fe->pose[6 * (size_t)s];
            if (r.ok) {
                std::memcpy(P, r.rvec, sizeof(r.rvec));
                std::memcpy(P + 3, r.tvec, sizeof(r.tvec));
            } else {
                std::fill(P, P + 6, 0.0);
            }
            fe_set_pose(fe, s, r.ok, P, P + 3);
        });
    }
    fe->fits_pending = false;
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

hipError_t fe_make_stream(hipStream_t* st, int priority) {
    return hipStreamCreateWithPriority(st, hipStreamNonBlocking, priority);
}

}  // namespace

extern "C" {

int svo_frontend_create(svo_ctx* ctx, const svo_frontend_config* cfg, svo_frontend** out) {
    if (!ctx || !cfg || !out) return SVO_ERR_ARG;
    const svo_frontend_config& c = *cfg;
    if (c.width <= 0 || c.height <= 0 || c.n_seq <= 0 || c.n_frames < 2 || c.n_features <= 0 || c.max_level < 0 ||
        !lk_supported(c.win, c.win) || c.stereo_win <= 2 || c.stereo_max_level < 0 ||
        !lk_supported(c.stereo_win, c.stereo_win) || c.pnp_iterations <= 0 ||
        !(c.pnp_confidence > 0 && c.pnp_confidence < 1) ||
        (c.keyframe_rule != SVO_KF_EVERY && c.keyframe_rule != SVO_KF_REFERENCE) ||
        (c.bucket_size > 0 && (c.per_bucket <= 0 || c.width / c.bucket_size <= 0)) ||
        (c.use_orb != 0 && c.use_orb != 1) || (c.use_orb && c.bucket_size > 0))
        return set_error(ctx, SVO_ERR_ARG, "svo_frontend_create: bad config");
    svo_frontend* fe = new svo_frontend();
    fe->ctx = ctx;
    fe->cfg = c;
    fe->S = c.n_seq;
    fe->T = c.n_frames;
    fe->W = c.width;
    fe->H = c.height;
    fe->CAP = (c.n_features + 63) & ~63;
    fe->WORDS = (fe->CAP + 31) / 32;
    fe->KCAP = std::max(4 * fe->CAP, 8192);
    fe->BCAP = ((c.bucket_size > 0) ? (c.height / c.bucket_size + 1) * (c.width / c.bucket_size + 1) * c.per_bucket
                                    : 1) + 64;
    fe->MAPCAP = fe->CAP * (c.n_frames + 2);
    fe->npx = (size_t)c.width * c.height;
    fe->ml = lk_levels_for_window(c.width, c.height, c.win, c.win, c.max_level);
    fe->ml_st = lk_levels_for_window(c.width, c.height, c.stereo_win, c.stereo_win, c.stereo_max_level);
    fe->nlev = std::max(fe->ml, fe->ml_st) + 1;
    fe->bscr = c.bucket_size > 0 ? bucket_scratch_ints(c.width, c.height, c.bucket_size, c.per_bucket, fe->KCAP) : 1;
    const int S = fe->S, CAP = fe->CAP;
    // frames: left and right pyramids of every resident stereo pair
    fe->frames.assign((size_t)S * fe->T, nullptr);
    fe->frames_r.assign((size_t)S * fe->T, nullptr);
    for (auto* v : {&fe->frames, &fe->frames_r})
        for (auto& f : *v) {
            int rc = svo_image_create(ctx, c.width, c.height, fe->nlev - 1, &f);
            if (rc) {
                svo_frontend_destroy(fe);
                return rc;
            }
        }
    fe->desc_host.resize((size_t)fe->T * S);
    fe->desc_r_host.resize((size_t)fe->T * S);
    for (int t = 0; t < fe->T; t++)
        for (int s = 0; s < S; s++) {
            fe->desc_host[(size_t)t * S + s] = fe->frames[(size_t)s * fe->T + t]->desc;
            fe->desc_r_host[(size_t)t * S + s] = fe->frames_r[(size_t)s * fe->T + t]->desc;
        }
    // device state: one allocation, laid out by the carve sequence below (run once
    // on a null base to size it)
    size_t bytes = 0;
    char* const dbase0 = nullptr;
    for (int pass = 0; pass < 2; pass++) {
        if (pass == 1) {
            if (hipMalloc(&fe->dmem, bytes) != hipSuccess) {
                svo_frontend_destroy(fe);
                return set_error(ctx, SVO_ERR_HIP, "svo_frontend_create: hipMalloc(%zu)", bytes);
            }
        }
        char* p = pass == 0 ? dbase0 : (char*)fe->dmem;
        fe->d_desc = carve<PyrDesc>(p, (size_t)fe->T * S);
        fe->d_desc_r = carve<PyrDesc>(p, (size_t)fe->T * S);
        fe->xyA = carve<float>(p, 2 * (size_t)S * CAP);
        fe->next_xy = carve<float>(p, 2 * (size_t)S * CAP);
        fe->st_xy = carve<float>(p, 2 * (size_t)S * CAP);
        fe->st_next = carve<float>(p, 2 * (size_t)S * CAP);
        fe->st_status = carve<uint8_t>(p, (size_t)S * CAP);
        fe->st_X = carve<float4>(p, (size_t)S * CAP);
        fe->st_n = carve<int>(p, S);
        fe->pend0 = carve<int>(p, S);
        fe->pend_n = carve<int>(p, S);
        fe->spec_n = carve<int>(p, S);
        fe->kps = carve<float>(p, 3 * (size_t)S * fe->KCAP);
        fe->cand = carve<float>(p, 2 * (size_t)S * fe->BCAP);
        fe->midA = carve<int>(p, (size_t)S * CAP);
        fe->midB = carve<int>(p, (size_t)S * CAP);
        fe->iters = carve<int>(p, (size_t)S * CAP);
        fe->nA = carve<int>(p, S);
        fe->kn = carve<int>(p, S);
        fe->bn = carve<int>(p, S);
        fe->map_n = carve<int>(p, S);
        fe->added = carve<int>(p, S);
        fe->rowcnt = carve<int>(p, (size_t)S * c.height);
        fe->scr = carve<int>(p, fe->bscr * S);
        fe->status = carve<uint8_t>(p, (size_t)S * CAP);
        fe->fbits = carve<unsigned long long>(p, (size_t)S * c.height * ((c.width + 63) / 64));
        fe->rowoff = carve<int>(p, (size_t)S * c.height);
        fe->map = carve<double>(p, 3 * (size_t)S * fe->MAPCAP);
        fe->box_binned = carve<float>(p, 2 * (size_t)S * CAP);
        fe->box_band = carve<int>(p, (size_t)S * fast_box_cells(c.width, c.height));
        for (int k = 0; k < 2; k++) {
            fe->xyB_b[k] = carve<float>(p, 2 * (size_t)S * CAP);
            fe->obj_b[k] = carve<float>(p, 3 * (size_t)S * CAP);
            fe->nB_b[k] = carve<int>(p, S);
        }
        fe->xyB = fe->xyB_b[0];
        fe->obj = fe->obj_b[0];
        fe->nB = fe->nB_b[0];
        bytes = (size_t)(p - (pass == 0 ? dbase0 : (char*)fe->dmem)) + 256;
    }
    (void)hipMemsetAsync(fe->dmem, 0, bytes, ctx->stream);
    // host mirrors (pinned): both parities of the full point copies
    {
        const size_t hb = 2 * (((sizeof(float) * 2 * (size_t)S * CAP + 255) & ~(size_t)255) +
                               ((sizeof(float) * 3 * (size_t)S * CAP + 255) & ~(size_t)255)) + 4096;
        if (hipHostMalloc(&fe->hmem, hb, hipHostMallocDefault) != hipSuccess) {
            svo_frontend_destroy(fe);
            return set_error(ctx, SVO_ERR_HIP, "svo_frontend_create: hipHostMalloc");
        }
        char* p = (char*)fe->hmem;
        for (int k = 0; k < 2; k++) {
            fe->h_xyB_b[k] = carve<float>(p, 2 * (size_t)S * CAP);
            fe->h_obj_b[k] = carve<float>(p, 3 * (size_t)S * CAP);
        }
        fe->h_xyB = fe->h_xyB_b[0];
        fe->h_obj = fe->h_obj_b[0];
    }
    // zero-copy scoring buffers (coherent: the kernel's writes are visible to the
    // host once the stream is synchronised)
    {
        const size_t zb = ((sizeof(double) * 12 * (size_t)S * kRansacChunk + 255) & ~(size_t)255) +
                          ((sizeof(uint32_t) * (size_t)S * kRansacChunk * fe->WORDS + 255) & ~(size_t)255) +
                          sizeof(int) * (size_t)S * kRansacChunk + 256;
        if (hipHostMalloc(&fe->zmem, zb, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
            fe->zmem = nullptr;
            svo_frontend_destroy(fe);
            return set_error(ctx, SVO_ERR_HIP, "svo_frontend_create: host-coherent scoring buffers");
        }
        char* p = (char*)fe->zmem;
        fe->z_hyps = carve<double>(p, 12 * (size_t)S * kRansacChunk);
        fe->z_bits = carve<uint32_t>(p, (size_t)S * kRansacChunk * fe->WORDS);
        fe->z_cnt = carve<int>(p, (size_t)S * kRansacChunk);
    }
    // host-coherent outputs the kernels write directly (no D2H copies on the
    // critical path): post-LK counts / iteration sums / RANSAC subsets, the
    // keyframe's counts; the inlier bits the tail and the statistics read (parity
    // pair); the keyframe targets the keyframe kernels read
    {
        size_t zb = 0;
        auto add = [&](size_t b) { zb = ((zb + 255) & ~(size_t)255) + b; };
        for (int k = 0; k < 5; k++) add(sizeof(int) * S);  // h_nB, h_nA, h_added, h_target, h_over
        add(sizeof(long long) * S);
        add(sizeof(float) * kSampleFloats * kRansacPrefetch * (size_t)S);
        add(sizeof(uint32_t) * (size_t)S * fe->WORDS);
        add(sizeof(uint32_t) * (size_t)S * fe->WORDS);
        add(sizeof(double) * kSqpnpStats * (size_t)S);
        add(sizeof(double) * 12 * (size_t)S);
        add(sizeof(double) * 6 * (size_t)S);
        add(sizeof(SqpnpFitIn) * (size_t)S);
        add(1024);
        if (hipHostMalloc(&fe->zout, zb, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
            fe->zout = nullptr;
            svo_frontend_destroy(fe);
            return set_error(ctx, SVO_ERR_HIP, "svo_frontend_create: host-coherent alloc");
        }
        std::memset(fe->zout, 0, zb);
        char* p = (char*)fe->zout;
        fe->h_nB = carve<int>(p, S);
        fe->h_nA = carve<int>(p, S);
        fe->h_added = carve<int>(p, S);
        fe->h_target = carve<int>(p, S);
        fe->h_over = carve<int>(p, S);
        fe->h_itsum = carve<long long>(p, S);
        fe->h_samp = carve<float>(p, (size_t)kSampleFloats * kRansacPrefetch * S);
        fe->h_best_b[0] = carve<uint32_t>(p, (size_t)S * fe->WORDS);
        fe->h_best_b[1] = carve<uint32_t>(p, (size_t)S * fe->WORDS);
        fe->h_best = fe->h_best_b[0];
        fe->h_stats = carve<double>(p, kSqpnpStats * (size_t)S);
        fe->h_pose = carve<double>(p, 12 * (size_t)S);
        fe->h_pose6 = carve<double>(p, 6 * (size_t)S);
        fe->h_fitin = carve<SqpnpFitIn>(p, (size_t)S);
        for (int s = 0; s < S; s++) fe_set_pose(fe, s, false, nullptr, nullptr);
    }
    // derivative pyramids of three frames of every sequence (t - 1: LK's prev,
    // t, and t + 1, built beside LK(t))
    {
        size_t doff[kMaxLevels];
        int dpitch[kMaxLevels];
        const size_t dbytes = (deriv_layout(c.width, c.height, fe->nlev, doff, dpitch) + 255) & ~(size_t)255;
        if (hipMalloc(&fe->dermem, dbytes * 3 * S + 256 + sizeof(DerivDesc) * 3 * S) != hipSuccess) {
            svo_frontend_destroy(fe);
            return set_error(ctx, SVO_ERR_HIP, "svo_frontend_create: deriv alloc");
        }
        std::vector<DerivDesc> hd(3 * (size_t)S);
        char* base = (char*)fe->dermem + ((sizeof(DerivDesc) * 3 * S + 255) & ~(size_t)255);
        for (int k = 0; k < 3 * S; k++)
            for (int l = 0; l < kMaxLevels; l++) {
                hd[k].data[l] = l < fe->nlev ? (uint32_t*)(base + dbytes * k + doff[l]) : nullptr;
                hd[k].pitch[l] = l < fe->nlev ? dpitch[l] : 0;
            }
        fe->d_der = (DerivDesc*)fe->dermem;
        SVO_HIP(ctx, hipMemsetAsync(base, 0, dbytes * 3 * S, ctx->stream));  // zero borders, never rewritten
        SVO_HIP(ctx, hipMemcpyAsync(fe->d_der, hd.data(), sizeof(DerivDesc) * hd.size(), hipMemcpyHostToDevice,
                                    ctx->stream));
        SVO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    }
    fe->rs.resize(S);
    fe->pred_iters.assign(S, 0);
    fe->kf_prev.assign(S, 1);
    {
        const char* fp = std::getenv("SVO_FE_FAST_PRE");
        fe->fast_pre = fp && fp[0] == '0' ? 0 : 1;
        const char* pp = std::getenv("SVO_FE_PRE_AFTER_POST");
        fe->pre_after_post = pp && pp[0] == '0' ? 0 : 1;
        const char* sm = std::getenv("SVO_FE_SPEC_MARGIN");
        fe->spec_margin = sm ? std::atoi(sm) : 32;
        const char* se = std::getenv("SVO_FE_SPEC_EARLY");
        fe->spec_early = se && se[0] == '0' ? 0 : 1;
        fe->trace = trace_env();
        fe->device_fits = device_fits_env();
        if (c.use_orb) {  // ORB: detection at the keyframe, the serial keyframe path
            fe->fast_pre = 0;
            fe->spec_margin = -1;
            fe->spec_early = 0;
        }
    }
    if (fe->device_fits && hipMalloc(&fe->fit_work, sqpnp_fit_work_bytes(S)) != hipSuccess) {
        svo_frontend_destroy(fe);
        return set_error(ctx, SVO_ERR_HIP, "svo_frontend_create: fit workspace");
    }
    if (c.use_orb) {
        fe->orb = orb_batch_create(S, c.width, c.height, c.orb);
        if (!fe->orb) {
            svo_frontend_destroy(fe);
            return set_error(ctx, SVO_ERR_ARG, "svo_frontend_create: ORB parameters or workspace");
        }
        fe->orb_lv0.resize(S);
        fe->orb_over.assign(S, 0);
    }
    // (on the context stream: a first use of the null stream would take a fifth
    // hardware queue and serialise the step's streams)
    if (hipMalloc(&fe->score_map, fe->npx * S) != hipSuccess) {
        svo_frontend_destroy(fe);
        return set_error(ctx, SVO_ERR_HIP, "svo_frontend_create: score map alloc");
    }
    fe->pose.assign((size_t)S * 6, 0.0);
    // host pool: this rank's share of the node's cores (NUMA-local to its GPU),
    // at most 16 threads (the box's CPU share per GPU) and one per sequence
    const int world = local_world_env();
    {
        const int rank = local_rank_env();
        int ndev = 0;
        (void)hipGetDeviceCount(&ndev);
        std::vector<int> gnode(world, -1);
        for (int r = 0; r < world && ndev > 0; r++) gnode[r] = device_numa_node(r % ndev);
        // SVO_POOL_PIN: 1 pin always, 0 never; default: pin when several ranks share
        // the node (one process alone keeps the OS placement: pinning it to fixed
        // cores measured up to 4x slower host work on a shared box)
        const char* pe = std::getenv("SVO_POOL_PIN");
        const bool pin = pe ? pe[0] == '1' : world > 1;
        if (pin) fe->host_cpus = host_cpu_plan(std::min(rank, world - 1), world, gnode.data());
    }
    int nt = c.host_threads > 0 ? c.host_threads
                                : (fe->host_cpus.empty() ? (int)std::thread::hardware_concurrency() / world
                                                         : (int)fe->host_cpus.size());
    nt = std::max(1, std::min({nt, S, 16}));
    fe->pool = new Pool(nt - 1, fe->host_cpus);
    for (auto& e : fe->ev) (void)hipEventCreate(&e);
    {
        int least = 0, greatest = 0;
        (void)hipDeviceGetStreamPriorityRange(&least, &greatest);
        // the LK stream at the highest priority (its chain is the step's critical
        // path), the FAST stream at the lowest (FAST fills the CUs LK leaves idle
        // and the post-LK window; the speculative stereo LK behind it is ready
        // long before the keyframe needs it)
        // (the context's: created once, shared by every front end on it, svo_ctx)
        if ((!ctx->fe_lk && fe_make_stream(&ctx->fe_lk, greatest) != hipSuccess) ||
            (!ctx->fe_fast && fe_make_stream(&ctx->fe_fast, least) != hipSuccess) ||
            (!ctx->fe_copy && hipStreamCreateWithFlags(&ctx->fe_copy, hipStreamNonBlocking) != hipSuccess)) {
            svo_frontend_destroy(fe);
            return set_error(ctx, SVO_ERR_HIP, "svo_frontend_create: stream");
        }
        fe->st_lk = ctx->fe_lk;
        fe->st_fast = ctx->fe_fast;
        fe->st_copy = ctx->fe_copy;
        for (hipEvent_t* e : {&fe->ev_pyr, &fe->ev_fast, &fe->ev_lk, &fe->ev_post, &fe->ev_tail, &fe->ev_stats,
                              &fe->ev_pyr_r_b[0], &fe->ev_pyr_r_b[1], &fe->ev_pre, &fe->ev_fdone, &fe->ev_full_b[0],
                              &fe->ev_full_b[1]})
            (void)hipEventCreateWithFlags(e, hipEventDisableTiming);
        fe->ev_full = fe->ev_full_b[0];
    }
    SVO_HIP(ctx, hipMemcpyAsync(fe->d_desc, fe->desc_host.data(), sizeof(PyrDesc) * fe->desc_host.size(),
                                hipMemcpyHostToDevice, ctx->stream));
    SVO_HIP(ctx, hipMemcpyAsync(fe->d_desc_r, fe->desc_r_host.data(), sizeof(PyrDesc) * fe->desc_r_host.size(),
                                hipMemcpyHostToDevice, ctx->stream));
    SVO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    *out = fe;
    return SVO_OK;
}

void svo_frontend_destroy(svo_frontend* fe) {
    if (!fe) return;
    if (fe->ctx) (void)hipStreamSynchronize(fe->ctx->stream);
    // (the streams are the context's: finished here, destroyed with the context)
    for (hipStream_t st : {fe->st_lk, fe->st_fast, fe->st_copy, fe->st_up})
        if (st) (void)hipStreamSynchronize(st);
    delete fe->pool;
    for (auto* v : {&fe->frames, &fe->frames_r})
        for (auto* f : *v)
            if (f) svo_image_destroy(fe->ctx, f);
    if (fe->dmem) (void)hipFree(fe->dmem);
    if (fe->dermem) (void)hipFree(fe->dermem);
    if (fe->hmem) (void)hipHostFree(fe->hmem);
    if (fe->zmem) (void)hipHostFree(fe->zmem);
    if (fe->zout) (void)hipHostFree(fe->zout);
    for (auto& e : fe->ev)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : {fe->ev_pyr, fe->ev_fast, fe->ev_lk, fe->ev_post, fe->ev_tail, fe->ev_stats, fe->ev_pyr_r_b[0],
                         fe->ev_pyr_r_b[1], fe->ev_pre, fe->ev_fdone, fe->ev_full_b[0], fe->ev_full_b[1]})
        if (e) (void)hipEventDestroy(e);
    if (fe->score_map) (void)hipFree(fe->score_map);
    for (hipEvent_t e : fe->ev_up)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : fe->ev_free)
        if (e) (void)hipEventDestroy(e);
    if (fe->up_stage) (void)hipFree(fe->up_stage);
    orb_batch_destroy(fe->orb);
    if (fe->fit_work) (void)hipFree(fe->fit_work);
    delete fe;
}

// Let every stream finish and forget the work queued ahead (a prefetched first
// half, a pyramid built ahead, a pre-detection): their inputs are about to
// change (new frames, re-init).
static int fe_drain(svo_frontend* fe) {
    svo_ctx* ctx = fe->ctx;
    for (hipStream_t st : {fe->st_lk, fe->st_fast, fe->st_copy, ctx->stream, fe->st_up})
        if (st) SVO_HIP(ctx, hipStreamSynchronize(st));
    fe->front_t = -1;
    fe->spec_t = -1;
    return SVO_OK;
}

static int fe_set_frame(svo_frontend* fe, int seq, int t, const uint8_t* left, const uint8_t* right, int stride,
                        bool bgr) {
    if (!fe || seq < 0 || seq >= fe->S || t < 0 || t >= fe->T || !left || !right || stride < (bgr ? 3 : 1) * fe->W)
        return SVO_ERR_ARG;
    svo_ctx* ctx = fe->ctx;
    int rd = fe_drain(fe);
    if (rd) return rd;
    if (fe->pyr_ready >= 0 && fe->pyr_ready % fe->T == t) fe->pyr_ready = -1;  // built from the old image
    if (fe->pre_t >= 0 && fe->pre_t % fe->T == t) fe->pre_t = -1;  // detected on the old image
    if (fe->pyr_r_ready >= 0 && fe->pyr_r_ready % fe->T == t) fe->pyr_r_ready = -1;
    // the slot now holds frame t, resident (the drain above finished any streamed
    // upload into it): steps keep finding it in the ring
    if (!fe->up_t.empty()) {
        fe->up_t[t] = t;
        fe->free_rec[t] = 0;
    }
    for (int side = 0; side < 2; side++) {
        svo_image* im = (side ? fe->frames_r : fe->frames)[(size_t)seq * fe->T + t];
        const uint8_t* px = side ? right : left;
        uint8_t* l0 = const_cast<uint8_t*>(im->desc.lv[0].data);
        if (bgr) {
            int rc = ingest_bgr(ctx, px, stride, fe->W, fe->H, l0, im->desc.lv[0].pitch);
            if (rc) return rc;
        } else {
            SVO_HIP(ctx, hipMemcpy2DAsync(l0, im->desc.lv[0].pitch, px, stride, fe->W, fe->H, hipMemcpyHostToDevice,
                                          ctx->stream));
        }
    }
    SVO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return SVO_OK;
}

int svo_frontend_set_frame(svo_frontend* fe, int seq, int t, const uint8_t* left, const uint8_t* right, int stride) {
    return fe_set_frame(fe, seq, t, left, right, stride, false);
}

int svo_frontend_set_frame_bgr(svo_frontend* fe, int seq, int t, const uint8_t* left_bgr, const uint8_t* right_bgr,
                               int stride) {
    return fe_set_frame(fe, seq, t, left_bgr, right_bgr, stride, true);
}

// The pyramid builds of frame f (context stream) wait for its streamed upload.
static int fe_wait_upload(svo_frontend* fe, int f, hipStream_t st) {
    if (!fe->up_t.empty() && fe->up_t[f % fe->T] == f) SVO_HIP(fe->ctx, hipStreamWaitEvent(st, fe->ev_up[f % fe->T], 0));
    return SVO_OK;
}

// Frame f can be built ahead: resident frames are 0 .. n_frames - 1 (a caller
// that reuses slots with set_frame gets no ahead-builds past them); once frames
// are streamed (queue_frames), the ring holds the frames queued into it.
static bool fe_has_frame(const svo_frontend* fe, int f) {
    if (fe->up_t.empty()) return f < fe->T;
    return fe->up_t[f % fe->T] == f;
}

int svo_frontend_queue_frames(svo_frontend* fe, int t, const uint8_t* const* left, const uint8_t* const* right,
                              int stride, int bgr) {
    if (!fe || t < 0 || !left || !right || stride < (bgr ? 3 : 1) * fe->W) return SVO_ERR_ARG;
    svo_ctx* ctx = fe->ctx;
    const int S = fe->S, T = fe->T, W = fe->W, H = fe->H;
    if (T < 4) return set_error(ctx, SVO_ERR_ARG, "svo_frontend_queue_frames: needs a ring of n_frames >= 4");
    for (int s = 0; s < S; s++)
        if (!left[s] || !right[s]) return SVO_ERR_ARG;
    // ring discipline: frame t's pyramid is built at the end of step t - 2, so it is
    // queued before that step (t >= stepped + 3); its slot's previous frame t - T is
    // no longer read once step t - T + 1 returned (t <= stepped + T - 1)
    // a frame at or before the last step restarts the loop: everything queued and
    // built ahead is finished and forgotten, and the window opens as before init
    if (fe->stepped >= 0 && t <= fe->stepped) {
        int rd = fe_drain(fe);
        if (rd) return rd;
        fe->stepped = -1;
        fe->pyr_ready = fe->pyr_r_ready = fe->pre_t = -1;
        std::fill(fe->up_t.begin(), fe->up_t.end(), -1);
        std::fill(fe->free_rec.begin(), fe->free_rec.end(), 0);
    }
    if (fe->stepped >= 0 && (t < fe->stepped + 3 || t > fe->stepped + T - 1))
        return set_error(ctx, SVO_ERR_ARG, "svo_frontend_queue_frames: frame outside the ring window "
                                           "(stepped + 3 .. stepped + n_frames - 1)");
    if (fe->up_t.empty()) {
        if (!ctx->fe_up) SVO_HIP(ctx, hipStreamCreateWithFlags(&ctx->fe_up, hipStreamNonBlocking));
        fe->st_up = ctx->fe_up;
        fe->ev_up.assign(T, nullptr);
        for (auto& e : fe->ev_up) SVO_HIP(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        fe->up_t.assign(T, -1);
        fe->ev_free.assign(T, nullptr);
        for (auto& e : fe->ev_free) SVO_HIP(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        fe->free_rec.assign(T, 0);
    }
    // the staging block mirrors the host frames (rows `stride` apart, sequences
    // H rows apart): a run of sequences whose buffers follow each other in memory
    // is one contiguous H2D copy; grown (after the queued uploads) for a wider stride
    const size_t seq_bytes = (size_t)H * stride;
    if (seq_bytes > fe->up_cap) {
        SVO_HIP(ctx, hipStreamSynchronize(fe->st_up));
        if (fe->up_stage) SVO_HIP(ctx, hipFree(fe->up_stage));
        fe->up_stage = nullptr;
        fe->up_cap = seq_bytes;
        SVO_HIP(ctx, hipMalloc(&fe->up_stage, 2 * (size_t)S * fe->up_cap));
    }
    fe->up_seq = seq_bytes;  // (the conversion of earlier queued frames captured their own stride)
    const int slot = t % T;
    const size_t last_row = (size_t)(bgr ? 3 : 1) * W;  // bytes of a frame's last row (no stride padding after it)
    uint8_t* stage = fe->up_stage;
    // the slot's previous frame (t - T) is last read by LK(t - T + 1): the copy into
    // the slot waits for it on the device, not only by the host's window above
    if (fe->free_rec[slot]) SVO_HIP(ctx, hipStreamWaitEvent(fe->st_up, fe->ev_free[slot], 0));
    fe->free_rec[slot] = 0;
    for (int side = 0; side < 2; side++) {
        const uint8_t* const* src = side ? right : left;
        uint8_t* dst = stage + (size_t)side * S * fe->up_cap;
        for (int s0 = 0; s0 < S;) {
            int s1 = s0 + 1;
            while (s1 < S && src[s1] == src[s1 - 1] + seq_bytes) s1++;
            const size_t n = (size_t)(s1 - s0 - 1) * fe->up_seq + (size_t)(H - 1) * stride + last_row;
            SVO_HIP(ctx, hipMemcpyAsync(dst + (size_t)s0 * fe->up_seq, src[s0], n, hipMemcpyHostToDevice, fe->st_up));
            s0 = s1;
        }
        const PyrDesc* d = (side ? fe->d_desc_r : fe->d_desc) + (size_t)slot * S;
        SVO_HIP(ctx, launch_ingest_batched(dst, fe->up_seq, stride, d, S, W, H, bgr != 0, fe->st_up));
    }
    SVO_HIP(ctx, hipEventRecord(fe->ev_up[slot], fe->st_up));
    fe->up_t[slot] = t;
    // anything built ahead from the slot's previous frame is stale
    if (fe->pyr_ready == t) fe->pyr_ready = -1;
    if (fe->pyr_r_ready == t) fe->pyr_r_ready = -1;
    if (fe->pre_t == t) fe->pre_t = -1;
    return SVO_OK;
}

int svo_frontend_upload_wait(svo_frontend* fe, int t) {
    if (!fe || t < 0) return SVO_ERR_ARG;
    if (fe->up_t.empty() || fe->up_t[t % fe->T] != t) return SVO_OK;
    SVO_HIP(fe->ctx, hipEventSynchronize(fe->ev_up[t % fe->T]));
    return SVO_OK;
}

int svo_frontend_prebuild_pyramids(svo_frontend* fe) {
    if (!fe) return SVO_ERR_ARG;
    for (int t = 0; t < fe->T; t++) {
        if (!fe->up_t.empty() && fe->up_t[t] >= 0) SVO_HIP(fe->ctx, hipStreamWaitEvent(fe->ctx->stream, fe->ev_up[t], 0));
        SVO_HIP(fe->ctx, launch_pyramid_batched(fe->d_desc + (size_t)t * fe->S, fe->S, fe->W, fe->H, fe->nlev,
                                                fe->ctx->stream));
        SVO_HIP(fe->ctx, launch_pyramid_batched(fe->d_desc_r + (size_t)t * fe->S, fe->S, fe->W, fe->H, fe->nlev,
                                                fe->ctx->stream));
    }
    SVO_HIP(fe->ctx, hipStreamSynchronize(fe->ctx->stream));
    return SVO_OK;
}

// Tracking::startStereo's first frame (R:src/tracking.cpp:233-235): extractFeatures
// (FAST without a mask: prevFrame == frame has no features yet), stereo match,
// triangulation with the identity pose (Frame's default), capped at n_features.
// Frame t0 is a keyframe under either rule (nextFrame: lastFrameID == 0).
int svo_frontend_init(svo_frontend* fe, int t0) {
    if (!fe || t0 < 0) return SVO_ERR_ARG;
    int rd = fe_drain(fe);
    if (rd) return rd;
    fe->pyr_ready = -1;
    fe->pyr_r_ready = -1;
    fe->pre_t = -1;
    fe->fits_pending = false;
    fe->stats_pending = false;
    fe->boxes_binned = false;
    svo_ctx* ctx = fe->ctx;
    const int S = fe->S;
    for (int s = 0; s < S; s++) fe->h_target[s] = fe->cfg.n_features;
    std::fill(fe->kf_prev.begin(), fe->kf_prev.end(), 1);
    const PyrDesc* dcur = fe->d_desc + (size_t)(t0 % fe->T) * S;
    {
        int rw = fe_wait_upload(fe, t0, ctx->stream);
        if (rw) return rw;
    }
    SVO_HIP(ctx, launch_pyramid_scharr_batched(dcur, fe->d_der + (size_t)(t0 % 3) * S, S, fe->W, fe->H, fe->nlev,
                                               ctx->stream));
    SVO_HIP(ctx, launch_pyramid_batched(fe->d_desc_r + (size_t)(t0 % fe->T) * S, S, fe->W, fe->H, fe->nlev,
                                        ctx->stream));
    SVO_HIP(ctx, hipEventRecord(fe->ev_pyr_r_b[t0 & 1], ctx->stream));
    SVO_HIP(ctx, hipMemsetAsync(fe->nA, 0, sizeof(int) * S, ctx->stream));
    SVO_HIP(ctx, hipMemsetAsync(fe->map_n, 0, sizeof(int) * S, ctx->stream));
    SVO_HIP(ctx, hipMemsetAsync(fe->pend_n, 0, sizeof(int) * S, ctx->stream));
    int rc = fe->orb ? fe_orb_detect(fe, t0, false, ctx->stream) : fe_fast_and_bucket(fe, dcur, false, ctx->stream);
    if (rc) return rc;
    // n_in = nA (zero): nothing to compact, the candidates fill the set
    rc = fe_keyframe(fe, t0, fe->nA, nullptr, fe->xyA, fe->midA, fe->cfg.n_features, ctx->stream);
    if (rc) return rc;
    for (int s = 0; s < S; s++) fe_set_pose(fe, s, false, nullptr, nullptr);
    SVO_HIP(ctx, launch_finalize_map(fe_pending(fe), S, ctx->stream));
    SVO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    ph_collect(fe);
    std::fill(fe->pose.begin(), fe->pose.end(), 0.0);
    fe->stepped = t0;
    return SVO_OK;
}

// trackFrames' calcOpticalFlowPyrLK parameters (R:src/tracking.cpp:154-179)
static LKParams fe_temporal_params(const svo_frontend* fe) {
    const svo_frontend_config& c = fe->cfg;
    LKParams lp;
    lp.win_w = lp.win_h = c.win;
    lp.max_level = fe->ml;
    lp.max_count = std::min(std::max(c.lk_max_count, 0), 100);
    const double eps = std::min(std::max(c.lk_epsilon, 0.0), 10.0);
    lp.eps2 = eps * eps;
    lp.flags = c.lk_flags & ~(SVO_LK_USE_INITIAL_FLOW | SVO_LK_OPENCV_ORDER);
    lp.cv_order = (c.lk_flags & SVO_LK_OPENCV_ORDER) ? 1 : 0;
    lp.min_eig = (float)c.min_eig;
    lp.want_err = 0;
    lk_apply_env(lp);
    return lp;
}

static int fe_queue_pre_and_right(svo_frontend* fe, int tn);

// Post-LK of step t, queued once the previous step's poses are set
// (fe_finish_fits): its keyframe points go to the world frame first. The
// keyframe's stereo matches go out right behind it, speculatively, beside the
// host's RANSAC.
static int fe_post(svo_frontend* fe, int t) {
    const auto t0 = std::chrono::steady_clock::now();
    auto TP = [&](const char* label) {
        if (fe->trace)
            std::fprintf(stderr, "[fe post t=%d] %8.1f us  %s\n", t,
                         std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count(), label);
    };
    svo_ctx* ctx = fe->ctx;
    const int CAP = fe->CAP;
    hipStream_t sl = fe->st_lk;
    int slot;
    // the previous step's final fits (launch_sqpnp_fit) set the poses the post-LK
    // moves the previous keyframe's new map points with
    if (fe->device_fits) SVO_HIP(ctx, hipStreamWaitEvent(sl, fe->ev_stats, 0));
    PostLkBatch pb{fe->nA, fe->status, fe->next_xy, fe->midA, fe->iters, fe->xyB, fe->midB, fe->nB, fe_pending(fe),
                   fe->obj, CAP, kRansacPrefetch, fe->h_nB, fe->h_itsum, fe->h_samp};
    ph_begin(fe, PH_POST, sl, &slot);
    SVO_HIP(ctx, launch_post_lk(pb, fe->S, sl));
    ph_end(fe, sl, slot);
    SVO_HIP(ctx, hipEventRecord(fe->ev_post, sl));
    TP("post_lk launched");
    if (fe->pre_pending == t + 1) {
        // (SVO_FE_PRE_AFTER_POST) frame t+1's pre-detection and right pyramid, on the
        // context stream behind this post-LK: when LK runs long, the pre-detection
        // would otherwise be dispatched ahead of the critical post-LK
        SVO_HIP(ctx, hipStreamWaitEvent(ctx->stream, fe->ev_post, 0));
        int rc = fe_queue_pre_and_right(fe, t + 1);
        if (rc) return rc;
    }
    fe->pre_pending = -1;
    if (fe->spec_margin >= 0 && fe->spec_t != t) {
        int rq = fe_queue_spec(fe, t, false);
        if (rq) return rq;
    }
    TP("spec stereo launched");
    // the full point set for the final fits / long RANSAC runs, on the copy stream
    // (parity buffers: the previous step's fits still read theirs)
    return fe_queue_full(fe);
}

// First half of a step (enqueue only, no host waits): the previous step's side
// work if still pending, the pyramid of frame t if not built ahead, temporal LK,
// FAST, the right pyramid of frame t and frame t+1's left pyramid.
// svo_frontend_step enqueues the next step's first half right after its own
// keyframe, so the GPU goes on with LK while the caller is between steps.
// Split in two so that the step can put the next LK on the GPU right behind its
// keyframe (fe_front_lk) before the side work's launches (fe_front_rest).
static int fe_front_lk(svo_frontend* fe, int t);
static int fe_front_rest(svo_frontend* fe, int t);
static int fe_queue_next_image(svo_frontend* fe, int tn);
static int fe_front(svo_frontend* fe, int t) {
    int rc = fe_front_lk(fe, t);
    return rc ? rc : fe_front_rest(fe, t);
}

static int fe_front_lk(svo_frontend* fe, int t) {
    svo_ctx* ctx = fe->ctx;
    hipStream_t st0 = ctx->stream;
    // (resident frames: the caller keeps slot t % n_frames current, set_frame)
    if (!fe->up_t.empty() && (!fe_has_frame(fe, t) || !fe_has_frame(fe, t - 1)))
        return set_error(ctx, SVO_ERR_ARG, "svo_frontend_step: frame %d is not in the ring (queue_frames)", t);
    const int S = fe->S;
    const PyrDesc* dcur = fe->d_desc + (size_t)(t % fe->T) * S;
    int slot;
    // this step's parity buffers (the previous step's stay with its side work)
    fe->xyB = fe->xyB_b[t & 1];
    fe->obj = fe->obj_b[t & 1];
    fe->nB = fe->nB_b[t & 1];
    fe->h_best = fe->h_best_b[t & 1];
    fe->h_xyB = fe->h_xyB_b[t & 1];
    fe->h_obj = fe->h_obj_b[t & 1];
    fe->ev_full = fe->ev_full_b[t & 1];
    fe->full_queued = false;
    // 0. the previous step's SQPnP statistics and the binning of the FAST mask's
    //    box centres (frame t-1's features) normally went out at the end of that
    //    step, ahead of this step's LK; only after init / a reset are they queued here
    {
        int rq = fe_queue_stats(fe);
        if (rq) return rq;
    }
    // 1. pyramid of frame t and its Scharr derivative pyramid (used when frame
    //    t is the prev image of the next step; OpenCV recomputes it per call),
    //    normally built ahead by the previous step's front half
    if (fe->pyr_ready != t) {
        int rw = fe_wait_upload(fe, t, st0);
        if (rw) return rw;
        ph_begin(fe, PH_PYR, st0, &slot);
        SVO_HIP(ctx, launch_pyramid_scharr_batched(dcur, fe->d_der + (size_t)(t % 3) * S, S, fe->W, fe->H, fe->nlev,
                                                   st0));
        ph_end(fe, st0, slot);
        SVO_HIP(ctx, hipEventRecord(fe->ev_pyr, st0));
    }
    // 2. temporal LK (trackFrames, frame t-1 -> t) behind frame t's pyramid
    {
        const LKParams lp = fe_temporal_params(fe);
        const PyrDesc* dprev = fe->d_desc + (size_t)((t - 1) % fe->T) * S;
        hipStream_t sl = fe->st_lk;
        SVO_HIP(ctx, hipStreamWaitEvent(sl, fe->ev_pyr, 0));
        LKBatch lb{dprev, dcur, fe->d_der + (size_t)((t - 1) % 3) * S, fe->xyA, fe->next_xy, fe->status, nullptr,
                   fe->iters, fe->nA, 0, fe->CAP};
        ph_begin(fe, PH_LK, sl, &slot);
        // grid bound CAP: the host counts of the previous keyframe may not be back yet
        SVO_HIP(ctx, launch_lk(lb, S, fe->CAP, lp, sl));
        ph_end(fe, sl, slot);
        SVO_HIP(ctx, hipEventRecord(fe->ev_lk, sl));
        // frame t-1's images are not read after this LK (its stereo LK and keyframe
        // ran before it on this stream or were waited for there): its ring slot may
        // be streamed into once this event fires
        if (!fe->ev_free.empty()) {
            const int fs = (t - 1) % fe->T;
            SVO_HIP(ctx, hipEventRecord(fe->ev_free[fs], sl));
            fe->free_rec[fs] = 1;
        }
    }
    return SVO_OK;
}

static int fe_front_rest(svo_frontend* fe, int t) {
    svo_ctx* ctx = fe->ctx;
    hipStream_t st0 = ctx->stream;
    const int S = fe->S;
    const PyrDesc* dcur = fe->d_desc + (size_t)(t % fe->T) * S;
    int slot;
    if (!fe->boxes_binned)
        SVO_HIP(ctx, launch_box_bin(fe_fast_batch(fe, dcur, true), S, fe->W, fe->H, fe->st_fast));
    fe->boxes_binned = false;
    // 3. mask around frame t-1's features (the reference masks with prevFrame's
    //    features, R:src/tracking.cpp:77) + FAST/bucket on frame t, whole batch:
    //    independent of this step's LK and pose, so it is queued right behind the
    //    LK on the low-priority FAST stream, where it fills the CUs the LK's last
    //    waves leave idle and the post-LK window; the keyframe waits for it
    {
        hipStream_t sf = fe->st_fast;
        int stage = kFastAll;
        if (fe->fast_pre && fe->pre_t == t) {
            // frame t was detected (unmasked) during step t-1; only the box mask of
            // frame t-1's features, the recount, scan and emit remain
            SVO_HIP(ctx, hipStreamWaitEvent(sf, fe->ev_pre, 0));
            stage = kFastBoxes;
        }
        fe->pre_t = -1;
        if (!fe->orb) {  // (ORB detects at the keyframe, fe_orb_detect)
            int rc = fe_fast_and_bucket(fe, dcur, true, sf, true, stage);
            if (rc) return rc;
        }
        SVO_HIP(ctx, hipEventRecord(fe->ev_fast, sf));
        SVO_HIP(ctx, hipEventRecord(fe->ev_fdone, sf));
    }
    // 4. the right frame t's pyramid (no derivatives: it is the stereo LK's next
    //    image), normally built ahead in the previous step (6b); the stereo LK of
    //    frame t waits for ev_pyr_r_b[t & 1]
    if (fe->pyr_r_ready != t) {
        int rw = fe_wait_upload(fe, t, st0);
        if (rw) return rw;
        ph_begin(fe, PH_PYR_R, st0, &slot);
        SVO_HIP(ctx, launch_pyramid_batched(fe->d_desc_r + (size_t)(t % fe->T) * S, S, fe->W, fe->H, fe->nlev, st0));
        ph_end(fe, st0, slot);
        SVO_HIP(ctx, hipEventRecord(fe->ev_pyr_r_b[t & 1], st0));
    }
    fe->pyr_r_ready = -1;
    // 4b. early speculative stereo LK of frame t (fe_queue_spec), behind FAST(t)
    //     and this right pyramid
    if (fe->spec_early && fe->spec_margin >= 0 && fe->cfg.keyframe_rule == SVO_KF_EVERY) {
        for (int s = 0; s < S; s++) fe->h_target[s] = fe->cfg.n_features;
        int rc = fe_queue_spec(fe, t, true);
        if (rc) return rc;
    }
    // 5. frame t+1's pyramid + Scharr + borders, queued beside this LK: the
    //    derivative pyramids are triple-buffered (frame f in f % 3), so nothing
    //    this step reads is overwritten, and the memory-bound pyramid shares the
    //    GPU with the VALU-bound LK instead of the post-LK window
    if (fe_has_frame(fe, t + 1)) return fe_queue_next_image(fe, t + 1);
    return SVO_OK;
}

// Frame tn's left pyramid, its FAST pre-detection and its right pyramid on the
// context stream (steps 5-6b of the first half of step tn - 1).
static int fe_queue_next_image(svo_frontend* fe, int tn) {
    svo_ctx* ctx = fe->ctx;
    hipStream_t st0 = ctx->stream;
    const int S = fe->S;
    int slot;
    {
        int rw = fe_wait_upload(fe, tn, st0);
        if (rw) return rw;
        const PyrDesc* dnext = fe->d_desc + (size_t)(tn % fe->T) * S;
        ph_begin(fe, PH_PYR, st0, &slot);
        SVO_HIP(ctx, launch_pyramid_scharr_batched(dnext, fe->d_der + (size_t)(tn % 3) * S, S, fe->W, fe->H,
                                                   fe->nlev, st0));
        ph_end(fe, st0, slot);
        SVO_HIP(ctx, hipEventRecord(fe->ev_pyr, st0));
        fe->pyr_ready = tn;
        // (pre_after_post: 6 and 6b are queued by fe_post instead, behind the post-LK)
        if (fe->pre_after_post) {
            fe->pre_pending = tn;
            return SVO_OK;
        }
        fe->pre_pending = -1;
    }
    return fe_queue_pre_and_right(fe, tn);
}

// 6. FAST pre-detection of frame tn (fe_queue_pre), behind its pyramid: it fills
//    the CUs the latency-bound post-LK / stereo chain leaves; 6b. then frame tn's
//    right pyramid: ready when step tn begins, so its speculative stereo LK can
//    start right behind FAST(tn) beside LK(tn) (built beside LK(tn) instead, it was
//    starved until LK's end).
static int fe_queue_pre_and_right(svo_frontend* fe, int tn) {
    svo_ctx* ctx = fe->ctx;
    hipStream_t st0 = ctx->stream;
    const int S = fe->S;
    int slot;
    if (fe->fast_pre) {
        int rc = fe_queue_pre(fe, tn);
        if (rc) return rc;
    }
    ph_begin(fe, PH_PYR_R, st0, &slot);
    SVO_HIP(ctx, launch_pyramid_batched(fe->d_desc_r + (size_t)(tn % fe->T) * S, S, fe->W, fe->H, fe->nlev, st0));
    ph_end(fe, st0, slot);
    SVO_HIP(ctx, hipEventRecord(fe->ev_pyr_r_b[tn & 1], st0));
    fe->pyr_r_ready = tn;
    return SVO_OK;
}

// Keyframe targets of step t (read by the speculative stereo prep and the
// keyframe kernels of this step): n_features on a keyframe, 0 otherwise.
// SVO_KF_EVERY: every frame. SVO_KF_REFERENCE: Tracking::nextFrame
// (R:src/tracking.cpp:68-69) -- the previous frame was no keyframe and kept fewer
// than features_to_track features (h_nA: the count after the previous step).
static int64_t fe_keyframe_targets(svo_frontend* fe) {
    const svo_frontend_config& c = fe->cfg;
    int64_t nkf = 0;
    for (int s = 0; s < fe->S; s++) {
        const bool kf = c.keyframe_rule == SVO_KF_EVERY || (!fe->kf_prev[s] && fe->h_nA[s] < c.features_to_track);
        fe->h_target[s] = kf ? c.n_features : 0;
        fe->kf_prev[s] = kf ? 1 : 0;
        nkf += kf ? 1 : 0;
    }
    return nkf;
}

int svo_frontend_step(svo_frontend* fe, int t, svo_frontend_stats* stats) {
    if (!fe || t < 1) return SVO_ERR_ARG;
    // per-round RANSAC inputs / scores on stderr (SVO_FE_DEBUG=1)
    static const bool debug_on = [] {
        const char* e = std::getenv("SVO_FE_DEBUG");
        return e && e[0] == '1';
    }();
    const bool tr = fe->trace;
    const auto trace_t0 = std::chrono::steady_clock::now();
    std::vector<std::pair<const char*, double>> trace;
    auto TP = [&](const char* label) {
        if (tr)
            trace.push_back({label, std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() -
                                                                               trace_t0).count()});
    };
    svo_ctx* ctx = fe->ctx;
    const int S = fe->S, CAP = fe->CAP;
    const svo_frontend_config& c = fe->cfg;
    int slot;
    using clk = std::chrono::steady_clock;
    auto ms_since = [](clk::time_point t0) {
        return std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    };
    const auto t_call = clk::now();
    double ms_enqueue = 0, ms_wait_post = 0, ms_wait_score = 0, ms_wait_kf = 0, ms_orb = 0;
    int64_t rounds = 0;

    if (fe->front_t != t) {
        int rf = fe_front(fe, t);
        if (rf) return rf;
    }
    fe->front_t = -1;
    TP("front enqueued");
    const int64_t n_keyframes = fe_keyframe_targets(fe);
    // the previous step's final pose fits: the host does them while the GPU tracks
    // this frame; they set the poses that move the previous keyframe's new map
    // points to the world frame, so this step's post-LK is queued right after
    // (with device_fits they ran on the device and the post-LK waits there)
    ms_enqueue += ms_since(t_call);
    double ms_fit = fe->device_fits ? 0.0 : fe_finish_fits(fe);
    TP("fits done");
    {
        const auto te = clk::now();
        int rp = fe_post(fe, t);
        if (rp) return rp;
        ms_enqueue += ms_since(te);
    }
    TP("post-lk queued");
    hipStream_t sl = fe->st_lk, sf = fe->st_fast;
    int rc = SVO_OK;
    const PyrDesc* dcur = fe->d_desc + (size_t)(t % fe->T) * S;

    double ms_hyp = 0;
    const float thr = (float)((double)c.pnp_reproj * (double)c.pnp_reproj);
    int64_t nhyp = 0, inl = 0;
    std::vector<int> ms(S, 0);
    std::vector<int> flat;  // (sequence, hypothesis) pairs of a chunk round
    flat.reserve((size_t)S * kRansacChunk);

    // calculatePose (RANSAC per sequence, hypotheses scored on the GPU), drop
    // outliers (R:src/tracking.cpp:218-229), keyframe
    TP("ransac begin");
    auto tw = clk::now();
    {
        // wait for the post-LK results, priming the pool (its workers sleep after
        // an idle spin window, and a futex wake-up of 15 threads cost ~40 us on the
        // critical path) shortly before they are predicted to land
        const double lead_ms = fe->post_wait_ms - 0.08;
        bool primed = false;
        for (;;) {
            const hipError_t q = hipEventQuery(fe->ev_post);
            if (q == hipSuccess) break;
            if (q != hipErrorNotReady) SVO_HIP(ctx, q);
            if (!primed && ms_since(tw) >= lead_ms) {
                fe->pool->prime();
                primed = true;
            }
        }
        const double w = ms_since(tw);
        fe->post_wait_ms = fe->post_wait_ms > 0 ? 0.75 * fe->post_wait_ms + 0.25 * w : w;
    }
    TP("lk results on host");
    ms_wait_post = ms_since(tw);
    // the speculative stereo LK went out early (fe_front) or with the post-LK (fe_post)
    const bool spec = fe->spec_margin >= 0 && fe->spec_t == t;
    const bool spec_early = spec && fe->spec_was_early;
    fe->spec_t = -1;
    int lk_loss = 0, ransac_drop = 0;
    bool need_full = false;
    for (int s = 0; s < S; s++) {
        RansacSeq& r = fe->rs[s];
        r.begin(fe->h_obj + 3 * (size_t)s * CAP, fe->h_xyB + 2 * (size_t)s * CAP, fe->h_nB[s], c.pnp_iterations);
        r.samp = fe->h_samp + (size_t)kSampleFloats * kRansacPrefetch * s;
        r.nsamp = kRansacPrefetch;
        // first chunk sized by the hypotheses the previous frame's outlier ratio
        // implies (a prediction only: a short chunk costs one more scoring round)
        r.first_chunk = std::max(kChunk0, fe->pred_iters[s]);
        need_full |= r.direct && !r.done;  // n <= 5: EPnP on all points
    }
    bool have_full = false;
    auto ensure_full = [&]() -> int {
        if (have_full) return SVO_OK;
        int rf = fe_queue_full(fe);
        if (rf) return rf;
        SVO_HIP(ctx, hipEventSynchronize(fe->ev_full));
        have_full = true;
        return SVO_OK;
    };
    if (need_full) {
        int rf = ensure_full();
        if (rf) return rf;
    }
    for (;;) {
        // sequences still sampling (no pool dispatch once all are done)
        bool any = false;
        for (int s = 0; s < S; s++) {
            any |= !fe->rs[s].done && !fe->rs[s].direct;
            need_full |= fe->rs[s].next_end() > fe->rs[s].nsamp;
        }
        if (!any) break;
        if (need_full) {  // past the prefetched subsets (> 26 hypotheses): rare
            const auto tfw = clk::now();
            int rf = ensure_full();
            if (rf) return rf;
            ms_wait_score += ms_since(tfw);
        }
        rounds++;
        auto th = clk::now();
        // the chunks' subsets are drawn per sequence (the RNG's order), their EPnP
        // solves shared out one hypothesis per pool task: a sequence predicted to
        // need 5 hypotheses no longer keeps one thread busy for 5 solves while
        // others idle (forward / occluder scene: ~320 solves a step)
        flat.clear();
        for (int s = 0; s < S; s++) {
            ms[s] = fe->rs[s].draw_chunk();
            for (int j = 0; j < ms[s]; j++) flat.push_back(s * kRansacChunk + j);
        }
        // one pool task per group of kEpnpLanes hypotheses (epnp_pixels_batch: their
        // 12 x 12 SVDs in SIMD lanes), groups taken in flat order across sequences
        const int ntask = ((int)flat.size() + kEpnpLanes - 1) / kEpnpLanes;
        auto solve_task = [&](int k) {
            RansacSeq* seqs[kEpnpLanes];
            int js[kEpnpLanes];
            const int k0 = k * kEpnpLanes;
            const int cnt = std::min(kEpnpLanes, (int)flat.size() - k0);
            for (int q = 0; q < cnt; q++) {
                seqs[q] = &fe->rs[flat[k0 + q] / kRansacChunk];
                js[q] = flat[k0 + q] % kRansacChunk;
            }
            solve_hypotheses(seqs, js, cnt, c.K);
        };
        if (tr) {
            // per-task attribution (trace only): which threads ran the solves, how long each took
            std::vector<std::pair<size_t, double>> tk(ntask);
            const auto tb = clk::now();
            fe->pool->run(ntask, [&](int k) {
                const auto a = clk::now();
                solve_task(k);
                tk[k] = {std::hash<std::thread::id>{}(std::this_thread::get_id()),
                         std::chrono::duration<double, std::micro>(clk::now() - a).count()};
                (void)tb;
            });
            std::vector<size_t> ids;
            double sum = 0, mx = 0;
            for (auto& e : tk) {
                if (std::find(ids.begin(), ids.end(), e.first) == ids.end()) ids.push_back(e.first);
                sum += e.second;
                mx = std::max(mx, e.second);
            }
            std::fprintf(stderr,
                         "[fe t=%d] pool: %zu solves in %zu tasks on %zu threads, mean %.1f us, max %.1f us per task, "
                         "wall %.1f us\n",
                         t, flat.size(), tk.size(), ids.size(), tk.empty() ? 0.0 : sum / tk.size(), mx,
                         std::chrono::duration<double, std::micro>(clk::now() - tb).count());
        } else {
            fe->pool->run(ntask, solve_task);
        }
        for (int s = 0; s < S; s++) fe->rs[s].nh += ms[s];
        ms_hyp += ms_since(th);
        TP("hyps generated");
        int mmax = 0;
        for (int s = 0; s < S; s++) mmax = std::max(mmax, ms[s]);
        if (mmax == 0) break;
        for (int s = 0; s < S; s++) {
            double* dst = fe->z_hyps + 12 * (size_t)s * kRansacChunk;
            std::memcpy(dst, fe->rs[s].hyp, sizeof(double) * 12 * ms[s]);
            for (int j = ms[s]; j < mmax; j++) std::memset(dst + 12 * j, 0, sizeof(double) * 12);
            nhyp += ms[s];
        }
        // hypotheses live at stride kRansacChunk; score only the mmax rows of this
        // round (rows beyond a sequence's own count are ignored). The kernel reads
        // the hypotheses and writes bits / counts in host-coherent memory.
        PnpBatch pb{fe->obj, fe->xyB, fe->nB, 0, CAP, fe->z_hyps, mmax, nullptr, fe->z_bits, fe->WORDS, fe->z_cnt};
        pb.mstride = kRansacChunk;
        ph_begin(fe, PH_PNP, sl, &slot);
        SVO_HIP(ctx, launch_pnp_score(pb, S, c.K[0], c.K[4], c.K[2], c.K[5], thr, sl));
        ph_end(fe, sl, slot);
        TP("scoring enqueued");
        const auto tsw = clk::now();
        SVO_HIP(ctx, hipStreamSynchronize(sl));
        ms_wait_score += ms_since(tsw);
        TP("scores on host");
        // consume is a few compares per hypothesis: cheaper here than a pool dispatch
        for (int s = 0; s < S; s++) {
            if (ms[s] <= 0) continue;
            const int* cnts = fe->z_cnt + (size_t)s * kRansacChunk;
            const uint32_t* bits = fe->z_bits + (size_t)s * kRansacChunk * fe->WORDS;
            if (debug_on) {
                const RansacSeq& r = fe->rs[s];
                unsigned hs = 0;
                for (int k = 0; k < kSampleFloats * ms[s]; k++) {
                    unsigned u;
                    std::memcpy(&u, r.samp + (size_t)kSampleFloats * (r.nh - ms[s]) + k, 4);
                    hs = hs * 31u + u;
                }
                std::fprintf(stderr, "[fe dbg t=%d s=%d] n=%d nh=%d m=%d samp=%08x cnt=", t, s, r.n, r.nh, ms[s], hs);
                for (int j = 0; j < ms[s]; j++) std::fprintf(stderr, "%d(%d,%.17g) ", cnts[j], (int)r.valid[j], r.hyp[12 * j]);
                std::fprintf(stderr, "\n");
            }
            fe->rs[s].consume(cnts, bits, fe->WORDS, c.pnp_confidence);
        }
    }
    // the RANSAC inlier set is the output (R:src/tracking.cpp:218-229); the final
    // SQPnP-objective fit only refines the pose, from statistics summed on the GPU
    TP("consumed");
    auto tf = clk::now();
    int max_take = 0;  // the keyframe's candidates per sequence are at most target - kept
    bool spec_ok = spec;  // every sequence dropped at most spec_margin points
    for (int s = 0; s < S; s++) {
        RansacSeq& r = fe->rs[s];
        r.select(c.K, false);
        // the device's final fit starts from this outcome (fe_queue_stats)
        SqpnpFitIn& fi = fe->h_fitin[s];
        fi.mode = !r.ok ? 0 : (r.fitted ? 2 : 1);
        std::memcpy(fi.R, r.bestR, sizeof(fi.R));
        std::memcpy(fi.t, r.fitted ? r.tvec : r.bestt, sizeof(fi.t));
        std::memcpy(fi.rv, r.rvec, sizeof(fi.rv));
        const int kept = r.ok ? r.maxGood : (r.n < 4 ? r.n : 0);
        max_take = std::max(max_take, fe->h_target[s] - kept);
        // (a sequence without a keyframe takes nothing: nothing to cover)
        // (early: h_nA still holds the count before LK; the keyframe rewrites it)
        const int n_ref = spec_early ? fe->h_nA[s] : fe->h_nB[s];
        spec_ok &= fe->h_target[s] == 0 || n_ref - kept <= fe->spec_m;
        lk_loss = std::max(lk_loss, fe->h_nA[s] - fe->h_nB[s]);
        ransac_drop = std::max(ransac_drop, fe->h_nB[s] - kept);
        uint32_t* b = fe->h_best + (size_t)s * fe->WORDS;
        std::memset(b, 0, sizeof(uint32_t) * fe->WORDS);
        if (r.ok) {
            std::memcpy(b, r.best.data(), sizeof(uint32_t) * r.best.size());
        } else if (r.n < 4) {
            // solvePnPRansac would throw (CV_Assert npoints >= 4); keep the frame's
            // features untouched instead of aborting the batch
            for (int k = 0; k < r.n; k++) b[k >> 5] |= 1u << (k & 31);
        }
        inl += r.ok ? (int64_t)r.maxGood : r.n;
        fe->pred_iters[s] = (r.ok && r.n > 0)
                                ? std::max(1, RansacSeq::predict_iters(c.pnp_confidence,
                                                                       (double)(r.n - r.maxGood) / r.n,
                                                                       c.pnp_iterations))
                                : 0;
    }
    fe->lk_loss = lk_loss;
    fe->ransac_drop = ransac_drop;
    ms_fit += ms_since(tf);
    TP("selected");
    // the SQPnP statistics of these inliers feed the pose fits the host runs during
    // the next step's LK. They are computed by the keyframe's outlier compaction
    // (the same workgroup reads the same points and bits: suffstats.hpp), so they
    // are done when the keyframe is, ahead of the next LK on the same queue. As a
    // kernel of their own on the copy stream they were at times dispatched only
    // after the next LK had filled the GPU -- in a process that had run other front
    // ends first, every step (host_ms_fit 2.25 ms instead of 0.33: the headline
    // 12 % slower, profiles/r06/c_legs_order_cause.txt)
    fe->stats_pending = true;
    fe->stats_parity = t & 1;
    fe->stats_in_tail = true;
    // ORB: the keyframe's detection, on the steps that take a keyframe
    if (fe->orb) {
        bool any = false;
        for (int s = 0; s < S; s++) any |= fe->h_target[s] > 0;
        if (any) {
            const auto to = clk::now();
            rc = fe_orb_detect(fe, t, true, sf);
            if (rc) return rc;
            ms_orb += ms_since(to);
        } else {
            SVO_HIP(ctx, hipMemsetAsync(fe->kn, 0, sizeof(int) * S, sf));
        }
        SVO_HIP(ctx, hipEventRecord(fe->ev_fast, sf));
    }
    // the mask (reads xyA) and FAST (writes kps) must be done before xyA is
    // rewritten / kps read
    SVO_HIP(ctx, hipStreamWaitEvent(sl, fe->ev_fast, 0));
    // drop the outliers (the kernel reads the inlier bits from host-coherent
    // memory), then the keyframe: candidates, stereo LK, triangulation, append
    const auto tkq = clk::now();
    rc = fe_keyframe(fe, t, fe->nB, fe->h_best, fe->xyB, fe->midB, max_take, sl, spec_ok);
    if (rc) return rc;
    SVO_HIP(ctx, hipEventRecord(fe->ev_tail, sl));
    if (!fe->stats_in_tail) {  // (fe_keyframe took them: done with the compaction)
        SVO_HIP(ctx, hipEventRecord(fe->ev_stats, sl));
        if (fe->device_fits) {  // the device's SQPnP fits from them, on the copy stream
            const int p = fe->stats_parity;
            SVO_HIP(ctx, hipStreamWaitEvent(fe->st_copy, fe->ev_stats, 0));
            SVO_HIP(ctx, launch_sqpnp_fit(fe->h_stats, fe->h_fitin, fe->obj_b[p], fe->nB_b[p], fe->CAP,
                                          fe->h_best_b[p], fe->WORDS, fe->S, fe->h_pose6, fe->h_pose, fe->fit_work,
                                          fe->st_copy));
            SVO_HIP(ctx, hipEventRecord(fe->ev_stats, fe->st_copy));
        }
        fe->stats_pending = false;
    }
    TP("tail queued");
    {
        int mt = fe->CAP;
        for (int s = 0; s < S; s++) mt = std::min(mt, fe->h_nB[s]);
        fe->min_tracked = mt;
    }
    fe->fits_pending = true;  // statistics land with the stream syncs below
    fe->fit_parity = t & 1;
    // The critical path goes on with the next step's LK right behind this
    // keyframe; only the SQPnP statistics of these inliers go to the GPU ahead of
    // it (the pose fits need them at the next step's start).
    SVO_HIP(ctx, hipStreamWaitEvent(sf, fe->ev_tail, 0));
    // this step's counts, before the next step's first half re-fills the mirrors
    int64_t lk_its = 0, tracked = 0;
    for (int s = 0; s < S; s++) {
        lk_its += fe->h_itsum[s];
        tracked += fe->h_nB[s];
    }
    rc = fe_queue_stats(fe);
    if (rc) return rc;
    // the next step's first half goes out now, behind this step's keyframe, so
    // the GPU moves on to its LK while the host returns to the caller: its LK
    // first (the keyframe -> LK hand-off is on the critical path), then the
    // binning of these features as the next frame's mask boxes (FAST stream,
    // ahead of the next step's FAST) and the rest of the first half
    // (streamed frames: the next frame was queued before this step, or the next
    // step finds it missing and fails loudly in its own first half)
    const bool next_ok = fe_has_frame(fe, t + 1);
    if (next_ok) {
        rc = fe_front_lk(fe, t + 1);
        if (rc) return rc;
    }
    SVO_HIP(ctx, launch_box_bin(fe_fast_batch(fe, dcur, true), S, fe->W, fe->H, sf));
    fe->boxes_binned = true;
    if (next_ok) {
        rc = fe_front_rest(fe, t + 1);
        if (rc) return rc;
        fe->front_t = t + 1;
    }
    TP("next front queued");
    ms_enqueue += ms_since(tkq);
    // wait for this step's keyframe only (the statistics, the next frame's
    // pyramid and the prefetched first half keep running into the next step)
    tw = clk::now();
    SVO_HIP(ctx, hipEventSynchronize(fe->ev_tail));
    ms_wait_kf = ms_since(tw);
    TP("synced");
    ph_collect(fe);
    if (tr) {
        for (auto& e : trace) std::fprintf(stderr, "[fe t=%d] %8.1f us  %s\n", t, e.second, e.first);
    }
    if (stats) {
        std::memset(stats, 0, sizeof(*stats));
        stats->lk_iterations = lk_its;
        stats->tracked = tracked;
        for (int s = 0; s < S; s++) {
            stats->added += fe->h_added[s];
            stats->features += fe->h_nA[s];
        }
        stats->inliers = inl;
        stats->hypotheses = nhyp;
        stats->host_ms_hyp = ms_hyp;
        stats->host_ms_fit = ms_fit;
        stats->host_ms_wait = ms_wait_post + ms_wait_score + ms_wait_kf;
        stats->keyframes = n_keyframes;
        stats->host_ms_wait_post = ms_wait_post;
        stats->host_ms_wait_score = ms_wait_score;
        stats->host_ms_wait_kf = ms_wait_kf;
        stats->host_ms_enqueue = ms_enqueue;
        stats->host_ms_step = ms_since(t_call);
        stats->ransac_rounds = rounds;
        int64_t mh = 0;
        for (int s = 0; s < S; s++) mh = std::max<int64_t>(mh, fe->rs[s].nh);
        stats->max_hypotheses = mh;
        stats->serial_keyframe = spec_ok ? 0 : 1;
        stats->full_copy = have_full ? 1 : 0;
        // Tracking::nextFrame's rule: a keyframe takes every masked corner, so a
        // corner left out for lack of capacity (n_features) is a deviation
        int64_t over = 0;
        if (c.keyframe_rule == SVO_KF_REFERENCE)
            for (int s = 0; s < S; s++)
                if (fe->h_target[s] > 0)  // a keyframe: this step's detection ran (ORB: orb_over)
                    over += fe->h_over[s] + (fe->orb ? fe->orb_over[s] : 0);
        stats->kf_overflow = over;
        stats->host_ms_orb = ms_orb;
        stats->spec_margin = fe->spec_m;
    }
    fe->stepped = t;
    return SVO_OK;
}

int svo_frontend_synchronize(svo_frontend* fe) {
    if (!fe) return SVO_ERR_ARG;
    svo_ctx* ctx = fe->ctx;
    int rq = fe_queue_stats(fe);
    if (rq) return rq;
    for (hipStream_t st : {fe->st_lk, fe->st_fast, fe->st_copy, ctx->stream}) SVO_HIP(ctx, hipStreamSynchronize(st));
    fe_finish_fits(fe);
    // the last keyframe's map points to the world frame (the next post-LK finds
    // nothing pending then)
    SVO_HIP(ctx, launch_finalize_map(fe_pending(fe), fe->S, ctx->stream));
    SVO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return SVO_OK;
}

int svo_frontend_pose(svo_frontend* fe, int seq, double rvec[3], double tvec[3]) {
    if (!fe || seq < 0 || seq >= fe->S) return SVO_ERR_ARG;
    int rq = fe_queue_stats(fe);
    if (rq) return rq;
    fe_finish_fits(fe);
    std::memcpy(rvec, &fe->pose[6 * (size_t)seq], sizeof(double) * 3);
    std::memcpy(tvec, &fe->pose[6 * (size_t)seq + 3], sizeof(double) * 3);
    return SVO_OK;
}

int svo_frontend_features(svo_frontend* fe, int seq, float* xy, int cap, int* n) {
    if (!fe || seq < 0 || seq >= fe->S) return SVO_ERR_ARG;
    svo_ctx* ctx = fe->ctx;
    int cnt = 0;
    SVO_HIP(ctx, hipMemcpyAsync(&cnt, fe->nA + seq, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    SVO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    const int k = std::min(cnt, cap);
    if (k > 0 && xy) {
        SVO_HIP(ctx, hipMemcpyAsync(xy, fe->xyA + 2 * (size_t)seq * fe->CAP, sizeof(float) * 2 * k,
                                    hipMemcpyDeviceToHost, ctx->stream));
        SVO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    }
    if (n) *n = cnt;
    return SVO_OK;
}

int svo_frontend_map_points(svo_frontend* fe, int seq, double* xyz, int cap, int* n) {
    if (!fe || seq < 0 || seq >= fe->S || cap < 0 || (cap > 0 && !xyz)) return SVO_ERR_ARG;
    int rc = svo_frontend_synchronize(fe);
    if (rc) return rc;
    svo_ctx* ctx = fe->ctx;
    int cnt = 0, mn = 0;
    SVO_HIP(ctx, hipMemcpyAsync(&cnt, fe->nA + seq, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    SVO_HIP(ctx, hipMemcpyAsync(&mn, fe->map_n + seq, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    SVO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    std::vector<int> mid((size_t)cnt);
    std::vector<double> map(3 * (size_t)mn);
    if (cnt > 0)
        SVO_HIP(ctx, hipMemcpyAsync(mid.data(), fe->midA + (size_t)seq * fe->CAP, sizeof(int) * cnt,
                                    hipMemcpyDeviceToHost, ctx->stream));
    if (mn > 0)
        SVO_HIP(ctx, hipMemcpyAsync(map.data(), fe->map + 3 * (size_t)seq * fe->MAPCAP, sizeof(double) * 3 * mn,
                                    hipMemcpyDeviceToHost, ctx->stream));
    SVO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    for (int i = 0; i < std::min(cnt, cap); i++) {
        if (mid[i] < 0 || mid[i] >= mn) return set_error(ctx, SVO_ERR_HIP, "svo_frontend_map_points: bad map id");
        std::memcpy(xyz + 3 * (size_t)i, &map[3 * (size_t)mid[i]], sizeof(double) * 3);
    }
    if (n) *n = cnt;
    return SVO_OK;
}

int svo_frontend_scharr_level(svo_frontend* fe, int seq, int t, int level, int16_t* ix, int16_t* iy, int stride) {
    if (!fe || seq < 0 || seq >= fe->S || t < 0 || level < 0 || level >= fe->nlev) return SVO_ERR_ARG;
    int rc = svo_frontend_synchronize(fe);
    if (rc) return rc;
    svo_ctx* ctx = fe->ctx;
    const ImgLevel& L = fe->desc_host[(size_t)(t % fe->T) * fe->S + seq].lv[level];
    if (stride < L.w) return set_error(ctx, SVO_ERR_ARG, "svo_frontend_scharr_level: stride");
    DerivDesc dd;
    SVO_HIP(ctx, hipMemcpy(&dd, fe->d_der + (size_t)(t % 3) * fe->S + seq, sizeof(dd), hipMemcpyDeviceToHost));
    return download_deriv_level(ctx, dd, level, L.w, L.h, ix, iy, stride);
}

int svo_frontend_pyramid_level(svo_frontend* fe, int seq, int t, int right, int level, uint8_t* out, int stride) {
    static_assert(SVO_PYR_PAD == kPyrPad, "header border width");
    if (!fe || seq < 0 || seq >= fe->S || t < 0 || level < 0 || level >= fe->nlev || !out) return SVO_ERR_ARG;
    int rc = svo_frontend_synchronize(fe);
    if (rc) return rc;
    svo_ctx* ctx = fe->ctx;
    const ImgLevel& L = (right ? fe->desc_r_host : fe->desc_host)[(size_t)(t % fe->T) * fe->S + seq].lv[level];
    const int bw = L.w + 2 * kPyrPad;
    if (stride < bw) return set_error(ctx, SVO_ERR_ARG, "svo_frontend_pyramid_level: stride");
    SVO_HIP(ctx, hipMemcpy2D(out, stride, L.data - (ptrdiff_t)kPyrPad * L.pitch - kPyrPad, L.pitch, bw,
                             L.h + 2 * kPyrPad, hipMemcpyDeviceToHost));
    return SVO_OK;
}

int svo_frontend_time_pyramid(svo_frontend* fe, int t, int reps, double* ms_per_launch) {
    if (!fe || t < 0 || reps <= 0 || !ms_per_launch) return SVO_ERR_ARG;
    int rc = svo_frontend_synchronize(fe);
    if (rc) return rc;
    svo_ctx* ctx = fe->ctx;
    const int S = fe->S;
    const PyrDesc* d = fe->d_desc + (size_t)(t % fe->T) * S;
    const DerivDesc* dd = fe->d_der + (size_t)(t % 3) * S;
    hipEvent_t e0, e1;
    SVO_HIP(ctx, hipEventCreate(&e0));
    SVO_HIP(ctx, hipEventCreate(&e1));
    // one untimed rebuild first (caches warm, identical contents)
    SVO_HIP(ctx, launch_pyramid_scharr_batched(d, dd, S, fe->W, fe->H, fe->nlev, ctx->stream));
    SVO_HIP(ctx, hipEventRecord(e0, ctx->stream));
    for (int i = 0; i < reps; i++)
        SVO_HIP(ctx, launch_pyramid_scharr_batched(d, dd, S, fe->W, fe->H, fe->nlev, ctx->stream));
    SVO_HIP(ctx, hipEventRecord(e1, ctx->stream));
    SVO_HIP(ctx, hipEventSynchronize(e1));
    float ms = 0.f;
    SVO_HIP(ctx, hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    *ms_per_launch = ms / reps;
    fe->pyr_ready = -1;
    return SVO_OK;
}

int svo_frontend_time_fast(svo_frontend* fe, int t, int reps, double* ms_per_launch) {
    if (!fe || t < 0 || reps <= 0 || !ms_per_launch) return SVO_ERR_ARG;
    int rc = svo_frontend_synchronize(fe);
    if (rc) return rc;
    svo_ctx* ctx = fe->ctx;
    const PyrDesc* d = fe->d_desc + (size_t)(t % fe->T) * fe->S;
    const FastDetBatch fb = fe_fast_batch(fe, d, false);
    auto launch = [&]() {
        return launch_fast_detect(fb, fe->S, fe->W, fe->H, fe->cfg.fast_threshold, fe->cfg.fast_nonmax, ctx->stream,
                                  kFastDetect);
    };
    hipEvent_t e0, e1;
    SVO_HIP(ctx, hipEventCreate(&e0));
    SVO_HIP(ctx, hipEventCreate(&e1));
    SVO_HIP(ctx, launch());  // warm-up
    SVO_HIP(ctx, hipEventRecord(e0, ctx->stream));
    for (int i = 0; i < reps; i++) SVO_HIP(ctx, launch());
    SVO_HIP(ctx, hipEventRecord(e1, ctx->stream));
    SVO_HIP(ctx, hipEventSynchronize(e1));
    float ms = 0.f;
    SVO_HIP(ctx, hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    *ms_per_launch = ms / reps;
    fe->pre_t = -1;  // the row words now hold frame t's unmasked detection, not a queued one
    return SVO_OK;
}

int svo_host_cpu_plan(int local_rank, int local_world, const int* gpu_node, int* cpus, int cap, int* n) {
    if (local_world <= 0 || local_rank < 0 || local_rank >= local_world || cap < 0 || (cap > 0 && !cpus))
        return SVO_ERR_ARG;
    const std::vector<int> v = host_cpu_plan(local_rank, local_world, gpu_node);
    for (int i = 0; i < (int)v.size() && i < cap; i++) cpus[i] = v[i];
    if (n) *n = (int)v.size();
    return SVO_OK;
}

int svo_frontend_host_cpus(svo_frontend* fe, int* cpus, int cap, int* n) {
    if (!fe || cap < 0 || (cap > 0 && !cpus)) return SVO_ERR_ARG;
    for (int i = 0; i < (int)fe->host_cpus.size() && i < cap; i++) cpus[i] = fe->host_cpus[i];
    if (n) *n = (int)fe->host_cpus.size();
    return SVO_OK;
}

int svo_frontend_streams(svo_frontend* fe, void** streams, int cap, int* n) {
    if (!fe || cap < 0 || (cap > 0 && !streams)) return SVO_ERR_ARG;
    const hipStream_t st[3] = {fe->st_lk, fe->st_fast, fe->st_copy};
    for (int i = 0; i < 3 && i < cap; i++) streams[i] = (void*)st[i];
    if (n) *n = 3;
    return SVO_OK;
}

int svo_frontend_phase_times(svo_frontend* fe, double* ms, int64_t* launches, int cap) {
    if (!fe) return SVO_ERR_ARG;
    ph_fold(fe, true);
    for (int i = 0; i < kPhases && i < cap; i++) {
        if (ms) ms[i] = fe->phase_ms[i];
        if (launches) launches[i] = fe->phase_n[i];
    }
    return kPhases;
}

void svo_frontend_reset_times(svo_frontend* fe) {
    if (!fe) return;
    ph_fold(fe, true);
    for (int i = 0; i < kPhases; i++) {
        fe->phase_ms[i] = 0;
        fe->phase_n[i] = 0;
    }
}

int svo_pool_selftest(int threads, int jobs, int64_t* bad) {
    if (threads < 1 || jobs < 1 || !bad) return SVO_ERR_ARG;
    // jobs of alternating, growing and shrinking sizes with primes between them
    // (the front end's pattern: per-hypothesis jobs whose size changes every
    // round): every task of every job must run exactly once, and no task of an
    // older job may run after its job returned
    Pool pool(threads - 1);
    std::vector<std::atomic<int>> hits(4096);
    std::atomic<int64_t> errors{0};
    uint64_t rng = 0x9e3779b97f4a7c15ull;
    for (int j = 0; j < jobs; j++) {
        rng = rng * 6364136223846793005ull + 1442695040888963407ull;
        const int n = (j & 1) ? 1 + (int)((rng >> 33) % 4096) : 1 + (int)((rng >> 33) % 8);
        for (int i = 0; i < n; i++) hits[i].store(0, std::memory_order_relaxed);
        const int tag = j;
        std::atomic<int> live{1};
        pool.run(n, [&, tag](int i) {
            if (i < 0 || i >= n || !live.load(std::memory_order_acquire) || tag != j) errors.fetch_add(1);
            if (i >= 0 && i < n) hits[i].fetch_add(1, std::memory_order_relaxed);
        });
        live.store(0, std::memory_order_release);
        for (int i = 0; i < n; i++)
            if (hits[i].load(std::memory_order_relaxed) != 1) errors.fetch_add(1);
        if ((rng >> 20) & 1) pool.prime();
    }
    *bad = errors.load();
    return SVO_OK;
}

}  // extern "C"
