#!/usr/bin/env python3
"""Benchmark: the reference's per-frame tracking step on MI355X.

Metric (BASELINE.json): frames/sec @1241x376, 2000 feats; LK iters/sec; achieved
HBM GB/s. A "step" = one stereo frame of every sequence in the batch through
pyramids (left + Scharr, right) -> temporal LK (21x21, maxLevel 3, 50 it,
MIN_EIGENVALS) -> status compaction -> solvePnPRansac (100 it, 8 px, 0.999: host
EPnP + GPU scoring, host SQPnP-objective fit) -> outlier removal -> keyframe:
mask + FAST(20, NMS), the first (2000 - n) corners stereo-matched (11x11 LK,
maxLevel 3, 30 it), |yR - yL| < 40, DLT triangulation, z > 0, world frame by the
estimated pose (R:src/tracking.cpp:240-269; every frame a keyframe that tops the
set up to 2000 features). Frames are synthetic KITTI-sized stereo renders
(svo_amd/scene.py), uploaded to HBM before the timed region. Multi-GPU: one
process per GPU, each advancing its own batch of independent sequences (weak
scaling, no collective on the data path).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--seq S] [--config kitti|1080p|4k]
"""
from __future__ import annotations

import argparse
import json
import re
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (W, H, n_features, max_level, workload label)   -- BASELINE.json configs[1..3]
    "kitti": (1241, 376, 2000, 3, "1241x376 KITTI-size synthetic, 2000 feats, 3-level (maxLevel 3) pyr-LK 21x21"),
    "1080p": (1920, 1080, 8000, 4, "1920x1080 synthetic, 8000 feats, maxLevel 4 pyr-LK 21x21"),
    "4k": (3840, 2160, 16000, 3, "3840x2160 synthetic, 16000 feats, 21x21 LK, maxLevel 3"),
}
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (guides/MI355X_MICROARCH.md)


def level_sizes(W: int, H: int, max_level: int):
    sizes = [(W, H)]
    for _ in range(max_level):
        w, h = sizes[-1]
        sizes.append(((w + 1) // 2, (h + 1) // 2))
    return sizes


def lk_bytes_per_feature(levels: int, win: int = 21) -> int:
    """B_lk per feature = L((win+3)^2 + (win+1)^2) + 21."""
    return levels * ((win + 3) ** 2 + (win + 1) ** 2) + 21


def pyr_bytes_per_frame(W: int, H: int, max_level: int) -> int:
    """B_pyr = sum_{l<L} w_l h_l (reads) + sum_{l>=1} w_l h_l (writes)."""
    sizes = level_sizes(W, H, max_level)
    return sum(w * h for w, h in sizes[:-1]) + sum(w * h for w, h in sizes[1:])


def deriv_bytes_per_frame(W: int, H: int, max_level: int) -> int:
    """The Scharr derivative pyramid the same launch writes (int16 Ix, Iy per pixel
    of every level; not in SURVEY's B_pyr, stated separately)."""
    return sum(4 * w * h for w, h in level_sizes(W, H, max_level))


def frame_bytes(W: int, H: int, n: int, max_level: int, win: int = 21) -> int:
    """B = B_pyr + B_fast + B_lk per frame."""
    return pyr_bytes_per_frame(W, H, max_level) + W * H + n * lk_bytes_per_feature(max_level + 1, win)


def dist_setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist  # plumbing only: barrier + max over ranks
        dist.init_process_group("gloo")
    return world, rank, local, dist


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int, argv) -> int:
    """`bench.py --gpus N` started without a launcher (no WORLD_SIZE in the env):
    start N child processes of this script, one per GPU, with the env
    torch.distributed.run would give them (RANK / LOCAL_RANK / WORLD_SIZE /
    LOCAL_WORLD_SIZE / MASTER_*; rendezvous on 127.0.0.1), and exit with the
    worst child status. This process never touches the GPU (no HIP call before
    the children start, no exec), so the children own the devices."""
    import subprocess
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    # a rank that fails leaves the others waiting in a barrier: end them too
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 1
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


def sequence_seeds(rank: int, per_gpu: int):
    """Seeds of the independent sequences this rank owns (disjoint across ranks)."""
    return [rank * per_gpu + s + 1 for s in range(per_gpu)]


def barrier(dist):
    if dist is not None:
        dist.barrier()


def allreduce_max(dist, v: float) -> float:
    if dist is None:
        return v
    import torch
    t = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allreduce_sum(dist, v: float) -> float:
    if dist is None:
        return v
    import torch
    t = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def kernel_key(name: str):
    """(bare name, template arguments) of a demangled kernel name as rocprofv3 lists it:
    'void svo::pyr_chain_kernel<3, true, 2>' -> ('pyr_chain_kernel', ('3', 'true', '2'))."""
    m = re.match(r"^(?:void\s+)?(?:[A-Za-z_]\w*::)*([A-Za-z_]\w*)\s*(?:<(.*)>)?", name.strip())
    if not m:
        return name, ()
    targs = tuple(a.strip() for a in m.group(2).split(",")) if m.group(2) else ()
    return m.group(1), targs


def pmc_select(kernels: dict, name: str, targs=None):
    """The one entry of a PMC summary's `kernels` whose bare name is `name` and whose
    first template arguments equal `targs` position by position (None in `targs` = any;
    `targs` None = no constraint). Exact keys, not substrings: the left chain's
    pyr_scharr_kernel<true, true, true> and the right pyramid's <true, false, true>
    share every prefix. More than one match is an error (ambiguous selection)."""
    hits = []
    for k, v in kernels.items():
        n, a = kernel_key(k)
        if n != name:
            continue
        # (trailing arguments beyond `targs` are free: round 6 appended LOOP to lk_multi_kernel)
        if targs is not None and (len(a) < len(targs) or any(t is not None and t != x for t, x in zip(targs, a))):
            continue
        hits.append((k, v))
    if len(hits) > 1:
        raise ValueError(f"PMC selection {name}<{targs}> is ambiguous: {[k for k, _ in hits]}")
    return hits[0] if hits else (None, None)


def pmc_traffic(cfg_name: str, name: str, seqs: int = 0, targs=None):
    """Per-launch HBM bytes of one kernel instance (bare name + template arguments,
    pmc_select) from the rocprofv3 PMC summary measured on THIS config's workload
    (profiles/pmc_summary.json configs[cfg_name], written by tools/pmc_summary.py
    --config), scaled from the sequences per launch it was measured at (the source's
    --seq) to `seqs`; None when that config or instance was not measured."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    c = d.get("configs", {}).get(cfg_name, {})
    m = re.search(r"--seq (\d+)", c.get("source", ""))
    scale = seqs / int(m.group(1)) if (m and seqs) else 1.0
    _, v = pmc_select(c.get("kernels", {}), name, targs)
    b = None if v is None else v.get("hbm_bytes_per_launch")
    return None if b is None else int(b * scale)


# template arguments of the instances the rooflines price (pmc_select): the temporal
# 21 x 21 LK (lk_multi_kernel<FPW 4, QJM 1, MINW 3, KKS 2, 21, 21, NR 7, LOOP false>;
# MINW free: A/B builds vary it; the stereo 11 x 11 instance is
# <4, 1, 6, 1, 11, 11, 11, true>), the left pyramid's Scharr kernels (second argument
# SCH = true; the right pyramid's instances have false there)
LK_TEMPORAL_TARGS = ("4", "1", None, "2", "21", "21", "7")
PYR_LEFT_TARGS = (None, "true", None)
CHAIN_LEFT_TARGS = (None, "true", None)

VALU_PEAK_G = 256 * 4 * 2.4 / 2  # G wave64 VALU instructions/s: 256 CUs x 4 SIMD-32, 2 cycles each at 2.4 GHz


def pmc_valu(kernel_prefix: str, seqs: int, cfg_name: str = "kitti"):
    """VALU wave-instructions per launch of a kernel from the committed SQ mix pass
    (profiles/valu_summary.json, written by tools/gpu.sh mix: SQ_INSTS_VALU per
    dispatch), scaled from the sequences per launch it was measured at to `seqs`;
    None when absent or measured at another config (its features per sequence and
    levels differ)."""
    path = os.path.join(ROOT, "profiles", "valu_summary.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None
    mc = re.search(r"--config (\w+)", d.get("source", ""))
    if (mc.group(1) if mc else "kitti") != cfg_name:
        return None, None
    m = re.search(r"--seq (\d+)", d.get("source", ""))
    measured = int(m.group(1)) if m else 128
    parts = (kernel_prefix,) if isinstance(kernel_prefix, str) else kernel_prefix
    for k, v in d.get("kernels", {}).items():
        if all(x in k for x in parts):
            return v["valu_per_dispatch"] * seqs / measured, d.get("source")
    return None, None


def roofline_valu(lk_name: str, seqs: int, lk_avg_s: float, cfg_name: str = "kitti"):
    """LK against the bound that binds it, VALU issue (SURVEY.md 8(d) prices it by
    bytes; rocprof shows the kernel issue-bound): the mix pass's VALU
    instructions per launch over this run's live average launch time."""
    # the mix pass keys kernels with their template arguments (the 21 x 21 and the
    # stereo 11 x 11 instances of lk_multi_kernel are separate entries)
    kname = ("lk_multi_kernel<4, 1, ", ", 2, 21, 21, 7") if lk_name.startswith("lk_multi") else "lk_fast_kernel<21, 21"
    valu, src = pmc_valu(kname, seqs, cfg_name)
    if valu is None or lk_avg_s <= 0:
        return None
    ach = valu / lk_avg_s / 1e9
    out = {"kernel": lk_name + ">", "bound": "valu", "achieved": round(ach, 1), "peak": VALU_PEAK_G,
           "unit": "G wave-instr/s", "frac": round(ach / VALU_PEAK_G, 4), "valu_per_launch": int(valu),
           "source": src, "timing": "live average launch time (the roofline's)"}
    # gfx950 issues most of LK's instructions (dot2, perm, DPP, cndmask, cmp, cvt, left
    # shifts) at half the rate of the 1,228.8 G/s peak: the issue rate its own mix
    # allows (tools/lk_mix_model.py over the compiled ISA, measured per-class rates)
    try:
        with open(os.path.join(ROOT, "profiles", "lk_issue_model.json")) as f:
            mdl = json.load(f)
        if lk_name.startswith("lk_multi"):
            out["peak_mix_weighted"] = mdl["peak_mix_G"]
            out["frac_mix_weighted"] = round(ach / mdl["peak_mix_G"], 4)
            out["slow_class_share"] = mdl["slow_share"]
            out["mix_model"] = mdl["source"]
    except (OSError, ValueError, KeyError):
        pass
    return out


def cpu_baseline(cfg_name: str, seconds: float):
    """The oracle (CPU restatement of the reference's OpenCV path) timed on this
    host on a bounded sample of the same workload: one sequence, frames until
    `seconds` of CPU work, twice: LK over all host threads (OpenMP, as OpenCV's
    parallel_for_) and single-threaded; FAST and PnP are
    single-threaded in both, as in OpenCV."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle as O  # noqa: E402  (oracle: cpu_baseline leg only)
    from oracle_loop import OracleLoop  # noqa: E402
    from svo_amd.scene import Scene
    W, H, N, _, _ = CONFIGS[cfg_name]
    # every CPU this process may use: the affinity mask, capped by OMP_NUM_THREADS
    # where the machine sets it -- the GPU box exports its per-GPU CPU share there
    # (16) while its affinity mask and nproc show the whole node (256); SURVEY
    # §8(d) asks for LK over all the host cores the process has
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        cores = min(cores, int(omp))

    def run(threads, secs):
        O.set_threads(threads)
        sc = Scene(W, H, seed=101)
        loop = OracleLoop(sc, N).init(0)
        dt, n = 0.0, 0
        while dt < secs and n < 5000:
            left, right = sc.frame(n + 1), sc.right(n + 1)  # rendered outside the timed region
            t0 = time.perf_counter()
            loop.step(n + 1, left, right)
            dt += time.perf_counter() - t0
            n += 1
        return n, dt

    n, dt = run(cores, seconds)
    n1, dt1 = run(1, seconds)
    O.set_threads(cores)
    return {"value": round(n / dt, 3), "unit": "frames/s", "cores": cores, "kind": "port",
            "nproc": os.cpu_count(), "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"),
            "sample": f"{n} stereo frames of one {W}x{H} sequence, {N} feats, {dt:.1f} s; oracle/ C restatement "
                      f"of the OpenCV path (LK OpenMP over {cores} threads, FAST/PnP/triangulation single-thread)",
            "single_thread": {"value": round(n1 / dt1, 3), "cores": 1,
                              "sample": f"{n1} frames, {dt1:.1f} s, everything on one thread"}}


def slowest_step(step_s, diag, warmup):
    """The slowest timed step with the library's own account of it: host waits
    split by what was waited for (post-LK results, RANSAC scoring rounds, the
    keyframe), launch issue time, RANSAC rounds, the serial keyframe fallback
    and the full point copy (svo_frontend_stats)."""
    if not step_s:
        return None
    i = int(np.argmax(step_s))
    d = diag[i]
    keys = ("host_ms_step", "host_ms_wait_post", "host_ms_wait_score", "host_ms_wait_kf", "host_ms_enqueue",
            "host_ms_hyp", "host_ms_fit", "ransac_rounds", "max_hypotheses", "hypotheses", "serial_keyframe",
            "full_copy", "added", "tracked", "inliers")
    out = {"index": i, "frame": warmup + 1 + i, "wall_ms": round(step_s[i] * 1e3, 3)}
    out.update({k: (round(d[k], 3) if isinstance(d[k], float) else d[k]) for k in keys})
    # the part of the step's wall time spent outside the library call (Python, ctypes)
    out["outside_call_ms"] = round(step_s[i] * 1e3 - d["host_ms_step"], 3)
    return out


def forward_workload(S, SceneForward, ctx, W, H, N, ML, Sq, K, Wm, threads):
    """The harder sequence (svo_amd.scene.SceneForward: forward translation with
    parallax + a textured occluder sliding against the static world, 5-20 % RANSAC
    outliers, several times more keyframe points) timed like the headline: Sq
    sequences per launch, Wm warm-up + K timed steps. 16 distinct sequences are
    rendered (the general renderer's host cost) and each fills Sq / 16 batch slots."""
    n_dist = min(Sq, 16)
    T = Wm + K + 2  # as the headline: the last timed step queues the next LK
    scs = [SceneForward(W, H, seed=1000 + i) for i in range(n_dist)]
    P = min(T, 2 * scs[0].period)
    pairs = [[(sc.frame(t), sc.right(t)) for t in range(P)] for sc in scs]
    fef = S.Frontend(ctx, S.FrontendConfig(W, H, scs[0].K, n_seq=Sq, n_frames=T, n_features=N, max_level=ML,
                                           host_threads=threads, timing=0))
    for s in range(Sq):
        for t in range(T):
            fef.set_frame(s, t, *pairs[s % n_dist][t % P])
    fef.init(0)
    for t in range(1, Wm + 1):
        fef.step(t)
    tot = {"tracked": 0, "inliers": 0, "added": 0, "hypotheses": 0}
    t1 = time.perf_counter()
    for t in range(Wm + 1, Wm + K + 1):
        st = fef.step(t).as_dict()
        for k in tot:
            tot[k] += st[k]
    fef.synchronize()
    dt = time.perf_counter() - t1
    fef.close()
    return {"value": round(Sq * K / dt, 2), "unit": "frames/s", "ms_per_step": round(dt / K * 1e3, 4),
            "steps": K, "warmup": Wm, "distinct_sequences": n_dist,
            "outlier_ratio": round(1 - tot["inliers"] / max(tot["tracked"], 1), 4),
            "stats_per_step": {k: round(v / K, 2) for k, v in tot.items()},
            "scene": "SceneForward: 0.04 m/frame forward (ping-pong), occluder at 8 m sliding 22 px/frame"}


def stream_workload(S, Scene, ctx, W, H, N, ML, Sq, K, Wm, threads, bgr, Kmat, pairs=None):
    """Ingest inside the timed window (the reference's loader hands each frame to
    Tracking as it is read, R:include/async_image_loader.h:36-69): the headline's
    loop, but every step's stereo pairs travel over PCIe -- svo_frontend_queue_frames:
    page-locked host frames, asynchronous H2D on the front end's upload stream into a
    4-slot ring, level 0 written by the batched ingest kernel (grey copy, or
    cv::cvtColor(BGR2GRAY) on the device when bgr) -- frame t + 2 queued before step
    t, overlapped with the step. 16 distinct sequences (the headline's first 16, or
    rendered) fill the Sq slots; every slot gets its own copy (Sq x 2 images per
    step cross the link). Also reported: the same uploads alone, back to back (the
    link + conversion ceiling)."""
    n_dist = min(Sq, 16)
    T = Wm + K + 3  # frames 0 .. Wm + K + 2 (frame t + 2 queued before step t)
    if pairs is None:
        scs = [Scene(W, H, seed=sequence_seeds(0, n_dist)[i]) for i in range(n_dist)]
        P = min(T, 2 * scs[0].period)
        pairs = [[(sc.frame(t), sc.right(t)) for t in range(P)] for sc in scs]
    P = min(T, len(pairs[0]))
    shape = (P, n_dist, H, W, 3) if bgr else (P, n_dist, H, W)
    pl, pr = S.PinnedBuffer(shape), S.PinnedBuffer(shape)
    for p in range(P):
        for d in range(n_dist):
            a, b = pairs[d][p]
            # BGR with equal channels: its grey is the frame itself (the tracking is
            # the grey run's; the conversion's arithmetic runs all the same)
            pl.array[p, d] = a[..., None] if bgr else a
            pr.array[p, d] = b[..., None] if bgr else b

    def queue(fe, t):
        fe.queue_frames(t, [pl.array[t % P, s % n_dist] for s in range(Sq)],
                        [pr.array[t % P, s % n_dist] for s in range(Sq)])

    K_img = Sq * 2 * W * H * (3 if bgr else 1)  # bytes over the link per step
    fe = S.Frontend(ctx, S.FrontendConfig(W, H, Kmat, n_seq=Sq, n_frames=4, n_features=N, max_level=ML,
                                          host_threads=threads, timing=0))
    # the link + conversion alone: 8 uploads back to back before init (no step reads the ring yet)
    for t in range(2):
        queue(fe, t)
    fe.upload_wait(1)
    t1 = time.perf_counter()
    for t in range(8):
        queue(fe, t)
    fe.upload_wait(7)
    alone = 8 * K_img / (time.perf_counter() - t1) / 1e9
    print(f"[bench] stream {'bgr' if bgr else 'grey'}: uploads alone {alone:.1f} GB/s", file=sys.stderr, flush=True)
    for t in range(3):
        queue(fe, t)
    fe.init(0)
    for t in range(1, Wm + 1):
        queue(fe, t + 2)
        fe.step(t)
    t1 = time.perf_counter()
    for t in range(Wm + 1, Wm + K + 1):
        queue(fe, t + 2)
        fe.step(t)
    fe.synchronize()
    dt = time.perf_counter() - t1
    fe.close()
    pl.close()
    pr.close()
    return {"value": round(Sq * K / dt, 2), "unit": "frames/s", "ms_per_step": round(dt / K * 1e3, 4),
            "steps": K, "warmup": Wm, "input": "BGR 8UC3" if bgr else "grey",
            "h2d_bytes_per_step": K_img, "h2d_GBps_in_loop": round(K_img * K / dt / 1e9, 2),
            "h2d_GBps_alone": round(alone, 2), "distinct_sequences": n_dist, "ring_slots": 4}


def orb_workload(S, SceneForward, ctx, W, H, ML, Sq, K, Wm, threads):
    """The reference's shipped configuration (R:configs/config.yaml:15,19-27): ORB
    keyframe detector (150 features, scale 1.2, 8 levels, HARRIS), Tracking::nextFrame's
    keyframe rule with features_to_track 70 (R:src/tracking.cpp:68-69), on the forward
    / occluder scene so that tracks are lost and keyframes recur; timed like the
    headline (Sq sequences per launch, Wm warm-up + K timed steps)."""
    n_dist = min(Sq, 16)
    T = Wm + K + 2
    scs = [SceneForward(W, H, seed=2000 + i) for i in range(n_dist)]
    P = min(T, 2 * scs[0].period)
    pairs = [[(sc.frame(t), sc.right(t)) for t in range(P)] for sc in scs]
    feo = S.Frontend(ctx, S.FrontendConfig(W, H, scs[0].K, n_seq=Sq, n_frames=T, n_features=2000, max_level=ML,
                                           host_threads=threads, timing=0, use_orb=1,
                                           keyframe_rule=S.KF_REFERENCE, features_to_track=70))
    for s in range(Sq):
        for t in range(T):
            feo.set_frame(s, t, *pairs[s % n_dist][t % P])
    feo.init(0)
    for t in range(1, Wm + 1):
        feo.step(t)
    tot = {"tracked": 0, "inliers": 0, "added": 0, "keyframes": 0}
    t1 = time.perf_counter()
    for t in range(Wm + 1, Wm + K + 1):
        st = feo.step(t).as_dict()
        for k in tot:
            tot[k] += st[k]
    feo.synchronize()
    dt = time.perf_counter() - t1
    feo.close()
    return {"value": round(Sq * K / dt, 2), "unit": "frames/s", "ms_per_step": round(dt / K * 1e3, 4),
            "steps": K, "warmup": Wm, "distinct_sequences": n_dist,
            "keyframe_ratio": round(tot["keyframes"] / (Sq * K), 4),
            "stats_per_step": {k: round(v / K, 2) for k, v in tot.items()},
            "config": "use_orb 1 (150 features, 1.2, 8 levels, HARRIS), SVO_KF_REFERENCE, features_to_track 70, "
                      "SceneForward"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults: a steady-state window (the first steps run while clocks ramp and the
    # RANSAC chunk predictions settle); every sequence frame is resident in HBM
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    # 256 independent sequences per GPU: the post-LK chain (post-LK kernel, host
    # EPnP, scoring, keyframe: ~0.16 ms, mostly latency) is paid once per step for the
    # whole batch, so frames/s rises with the batch -- round 4, driver window: 128:
    # 88.3k-89.1k, 256: 94.6k-94.9k (profiles/r04/e_seqcurve.txt); a step takes ~2.7 ms
    # at 256 (each sequence still advances ~370 frames/s)
    ap.add_argument("--seq", type=int, default=256, help="independent sequences per GPU (batched launches)")
    ap.add_argument("--config", default="kitti", choices=sorted(CONFIGS))
    ap.add_argument("--threads", type=int, default=0, help="host RANSAC threads (0 = auto)")
    ap.add_argument("--timing", type=int, default=2, choices=(1, 2, 3),
                    help="phase events: 1 all phases, 2 only LK/pyramid/FAST (lighter host tail), "
                         "3 the LK launches only (the roofline's)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-single", action="store_true")
    ap.add_argument("--no-orb", action="store_true", help="skip the shipped-config (ORB, reference keyframe rule) workload")
    ap.add_argument("--no-stream", action="store_true",
                    help="skip the streamed-ingest workloads (frames over PCIe inside the window, grey and BGR)")
    ap.add_argument("--no-opencv-order", action="store_true",
                    help="skip the headline batch timed again with LK in OpenCV's float order (SVO_LK_OPENCV_ORDER)")
    ap.add_argument("--no-bucketed", action="store_true",
                    help="skip the second measurement with bucketed selection in the loop")
    ap.add_argument("--scene", default="rot", choices=("rot", "forward"),
                    help="rot: the rotation-only scene (the headline); forward: SceneForward (translation "
                         "parallax + a moving occluder: 5-20%% RANSAC outliers) as the timed workload")
    ap.add_argument("--no-forward", action="store_true",
                    help="skip the extra timed pass over the forward/occluder scene (`workloads.forward`)")
    ap.add_argument("--legs", default="after", choices=("first", "after"),
                    help="after (default): the side workloads (single stream, bucketed, forward, ORB, "
                         "streamed) run behind the headline; first: before it -- measured 12 %% slower for the "
                         "headline (other front ends created and closed in the process first: "
                         "profiles/r05/l_legs_order_ab.txt)")
    ap.add_argument("--dry-run", action="store_true",
                    help="set up the ranks, print each rank's shard and exit (no GPU call)")
    args = ap.parse_args()

    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world, rank, local, dist = dist_setup()
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} ranks")
    if args.dry_run:
        seeds = sequence_seeds(rank, args.seq)
        barrier(dist)
        tot = allreduce_sum(dist, float(len(seeds)))
        print(json.dumps({"rank": rank, "local_rank": local, "world": world, "seeds": seeds,
                          "total_sequences": int(tot)}), flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return
    import svo_amd as S
    from svo_amd.scene import Scene, SceneForward

    W, H, N, ML, label = CONFIGS[args.config]
    Sq, K, Wm = args.seq, args.steps, args.warmup
    # frames 0 .. Wm + K + 1: the last timed step (Wm + K) queues the next step's
    # first half (its LK) as every step does, so the timed window holds K steps'
    # worth of work -- the LK of step Wm + 1, queued by the last warm-up step, runs
    # at the window's start, and that of step Wm + K + 1 is waited for at its end
    T = Wm + K + 2
    device = local
    if world > 1:
        # One rank per GPU; ranks beyond the visible devices (a multi-rank rehearsal on a
        # one-GPU box) share them round-robin. device_count() does not initialise HIP.
        import torch
        n_dev = torch.cuda.device_count()
        if n_dev > 0:
            device = local % n_dev
    ctx = S.Context(device)
    seeds = sequence_seeds(rank, Sq)
    scene_cls = SceneForward if args.scene == "forward" else Scene
    scenes = [scene_cls(W, H, seed=sd) for sd in seeds]
    # the synthetic camera ping-pongs with period 2 * scene.period (32 frames), so
    # P rendered stereo pairs per sequence are reused cyclically (frame t = pair
    # t mod P; rendering is host work outside the timing, all T frames resident)
    P = min(T, 2 * scenes[0].period)
    cfg = S.FrontendConfig(W, H, scenes[0].K, n_seq=Sq, n_frames=T, n_features=N, max_level=ML,
                           host_threads=args.threads, timing=args.timing)
    fe = S.Frontend(ctx, cfg)
    pairs0 = None
    keep_pairs = not (args.no_bucketed and args.no_opencv_order) and world == 1
    all_pairs = []
    for s, sc in enumerate(scenes):
        pairs = [(sc.frame(t), sc.right(t)) for t in range(P)]
        for t in range(T):
            fe.set_frame(s, t, *pairs[t % P])
        if s == 0:
            pairs0 = pairs
        if keep_pairs:
            all_pairs.append(pairs)
        if s % 16 == 15:
            print(f"[bench] rank {rank}: {s + 1}/{Sq} sequences rendered and uploaded", file=sys.stderr, flush=True)
    side = {"single": None, "bucketed": None, "forward": None, "orb": None, "stream": None, "opencv_order": None}

    def side_legs(close_fe):
        """The side workloads of the line (each its own front end and timed window)."""
        print("[bench] side measurements", file=sys.stderr, flush=True)
        close_fe()  # (legs after the headline: its front end is done with)
        single = None
        if not args.no_single and world == 1:
            fe1 = S.Frontend(ctx, S.FrontendConfig(W, H, scenes[0].K, n_seq=1, n_frames=T, n_features=N, max_level=ML))
            for t in range(T):
                fe1.set_frame(0, t, *pairs0[t % P])
            fe1.init(0)
            for t in range(1, Wm + 1):
                fe1.step(t)
            t1 = time.perf_counter()
            for t in range(Wm + 1, Wm + K + 1):
                fe1.step(t)
            fe1.synchronize()
            single = K / (time.perf_counter() - t1)
            fe1.close()
        forward = None
        if not args.no_forward and args.scene == "rot" and world == 1:
            print("[bench] forward / occluder workload", file=sys.stderr, flush=True)
            forward = forward_workload(S, SceneForward, ctx, W, H, N, ML, Sq, K, Wm, args.threads)
        orb = None
        if not args.no_orb and args.scene == "rot" and world == 1:
            print("[bench] shipped ORB configuration workload", file=sys.stderr, flush=True)
            orb = orb_workload(S, SceneForward, ctx, W, H, ML, Sq, K, Wm, args.threads)
        stream = None
        if not args.no_stream and args.scene == "rot" and world == 1:
            print("[bench] streamed-ingest workloads (grey, BGR)", file=sys.stderr, flush=True)
            firsts = all_pairs[:16] if all_pairs else None
            stream = {kind: stream_workload(S, Scene, ctx, W, H, N, ML, Sq, K, Wm, args.threads, kind == "bgr",
                                            scenes[0].K, firsts) for kind in ("grey", "bgr")}
        # (last when the legs run first: the headline's own workload, so the GPU
        # goes into the headline's warm-up busy)
        # SURVEY §8(d) lists "FAST + bucket" in the frame metric, but the reference's loop
        # never buckets (its call site is a TODO, R:src/tracking.cpp:88), so `value` is the
        # reference's loop; the same batch is timed again with bucketed selection
        # (bucket.hip, 50-px cells x 4 per cell) between FAST and the keyframe's take
        def headline_variant(**kw):
            """The headline batch (same frames) under another configuration: frames/s, ms/step."""
            fev = S.Frontend(ctx, S.FrontendConfig(W, H, scenes[0].K, n_seq=Sq, n_frames=T, n_features=N, max_level=ML,
                                                   host_threads=args.threads, timing=0, **kw))
            for s, pairs in enumerate(all_pairs):
                for t in range(T):
                    fev.set_frame(s, t, *pairs[t % P])
            fev.init(0)
            for t in range(1, Wm + 1):
                fev.step(t)
            t1 = time.perf_counter()
            for t in range(Wm + 1, Wm + K + 1):
                fev.step(t)
            fev.synchronize()
            dtv = time.perf_counter() - t1
            fev.close()
            return {"value": round(Sq * K / dtv, 2), "unit": "frames/s", "ms_per_step": round(dtv / K * 1e3, 4),
                    "steps": K, "warmup": Wm}

        bucketed = opencv_order = None
        if all_pairs:
            BS, PB = 50, 4
            if not args.no_bucketed:
                bucketed = dict(headline_variant(bucket_size=BS, per_bucket=PB), bucket_size=BS, per_bucket=PB)
            if not args.no_opencv_order:
                # both LK calls summed in OpenCV's own float order (SVO_LK_OPENCV_ORDER: the
                # drop-in Tracking mirror's default, bit-identical to cv::calcOpticalFlowPyrLK's
                # x86 build) instead of exactly (the headline): four features per wave
                print("[bench] OpenCV-order LK workload", file=sys.stderr, flush=True)
                opencv_order = dict(headline_variant(lk_flags=S.LK_GET_MIN_EIGENVALS | S.LK_OPENCV_ORDER),
                                    lk="SVO_LK_OPENCV_ORDER (lk_cvq_kernel, four features per wave)")
        side.update(single=single, bucketed=bucketed, forward=forward, orb=orb, stream=stream,
                    opencv_order=opencv_order)

    legs_after = args.legs == "after" or world > 1
    if not legs_after:
        side_legs(close_fe=lambda: None)
    fe.init(0)
    try:
        host_cpus = fe.host_cpus()  # this rank's pinned share of the node (svo_host_cpu_plan)
    except (AttributeError, S.SvoError):  # an older library under SVO_GPU_LIB A/B
        host_cpus = []
    feats_after = {}  # features after step t = the inputs of LK(t + 1)
    for t in range(1, Wm + 1):
        if t == Wm:
            # the phase timers restart before the last warm-up step: resetting
            # folds the pending event pairs, which waits for the GPU, so it must
            # not sit between the warm-up and the timed window (the window would
            # start on an idle GPU with LK(Wm + 1) already done)
            fe.reset_times()
        st = fe.step(t).as_dict()
        feats_after[t] = st["features"]
    tot = {"lk_iterations": 0, "tracked": 0, "inliers": 0, "added": 0, "hypotheses": 0,
           "host_ms_hyp": 0.0, "host_ms_fit": 0.0, "host_ms_wait": 0.0, "host_ms_wait_post": 0.0,
           "host_ms_wait_score": 0.0, "host_ms_wait_kf": 0.0, "host_ms_enqueue": 0.0, "ransac_rounds": 0,
           "serial_keyframe": 0, "full_copy": 0}
    step_s = []  # host wall time of each timed step (a slow run shows whether one step or all were slow)
    step_diag = []  # the library's per-step diagnostics of each timed step
    barrier(dist)
    t0 = time.perf_counter()
    tp = t0
    for t in range(Wm + 1, Wm + K + 1):
        st = fe.step(t).as_dict()
        now = time.perf_counter()
        step_s.append(now - tp)
        tp = now
        for k in tot:
            tot[k] += st[k]
        step_diag.append(st)
        feats_after[t] = st["features"]
    fe.synchronize()  # the last step's pose fits / prefetched pyramid belong to the timed work
    barrier(dist)
    dt = time.perf_counter() - t0
    dt_max = allreduce_max(dist, dt)
    frames = Sq * K * world
    fps = frames / dt_max
    lk_iters_total = allreduce_sum(dist, float(tot["lk_iterations"]))
    phases = fe.phase_times()

    if rank != 0:
        return
    # roofline of the dominant kernel (by device time): LK. The event pairs folded
    # since reset_times (before step Wm) bracket the LK launches of steps Wm + 1 ..
    # Wm + K + 1 (each queued by the step before it); LK(t) tracks the features
    # left after step t-1, so those launches processed feats_after[t-1] each.
    lk_ms, lk_n = phases["lk"]
    L = ML + 1
    last = Wm + K + 1
    lk_units = sum(feats_after[t - 1] for t in range(last - lk_n + 1, last + 1)) if lk_n > 0 else 0
    assert lk_n <= K + 1, "LK launches timed do not match the steps"
    units_per_launch = lk_units / max(lk_n, 1)
    bytes_per_launch = units_per_launch * lk_bytes_per_feature(L)
    lk_avg_s = lk_ms / max(lk_n, 1) / 1e3
    achieved = bytes_per_launch / lk_avg_s / 1e9 if lk_avg_s > 0 else 0.0
    # the 21x21 temporal call runs lk_multi_kernel<4, 1 (four features per wave)
    # unless SVO_LK_QUAD=0 (lk_fast_kernel, one per wave; svo_amd/csrc/lk.hip launch_lk)
    if os.environ.get("SVO_LK_QUAD", "1")[:1] == "0":
        lk_name, lk_desc, lk_targs = "lk_fast_kernel<21, 21", "one feature per wave", ("21", "21", None)
    else:
        lk_name, lk_desc, lk_targs = "lk_multi_kernel<4, 1", "four features per wave", LK_TEMPORAL_TARGS
    traffic = pmc_traffic(args.config, lk_name.split("<")[0], Sq, lk_targs)
    dominant = max(phases, key=lambda k: phases[k][0])
    # pyramid + Scharr of one new left frame per sequence per step (the launch
    # chain pyr_scharr_kernel x levels + the coarsest Scharr + borders)
    # (in the step it runs beside LK, which stretches it: its roofline is taken
    # from the same chain timed alone, 20 rebuilds of the last frame, after the
    # timed region; the in-step average is reported beside it)
    pyr_ms, pyr_n = phases.get("pyramid", (0.0, 0))
    pyr_instep_s = pyr_ms / max(pyr_n, 1) / 1e3
    pyr_avg_s = fe.time_pyramid(Wm + K, 20) / 1e3
    pyr_bytes = Sq * pyr_bytes_per_frame(W, H, ML)
    der_bytes = Sq * deriv_bytes_per_frame(W, H, ML)
    # the chain's HBM bytes. Fused (SVO_PYR_FUSED=1, the default; c = the coarsest
    # level, max(ML, stereo maxLevel 3)): c - 1 pyr_scharr launches (their average
    # over the levels x the count = the sum) + pyr_chain_kernel (last two levels,
    # derivatives, borders). Per level: c pyr_scharr + the coarsest scharr + borders.
    c_lev = max(ML, 3)
    if os.environ.get("SVO_PYR_FUSED", "1")[:1] == "0":
        t_ps, t_sc, t_pad = (pmc_traffic(args.config, k, Sq, a) for k, a in
                             (("pyr_scharr_kernel", PYR_LEFT_TARGS), ("scharr_kernel", None),
                              ("pad_batched_kernel", None)))
        pyr_traffic = c_lev * t_ps + t_sc + t_pad if None not in (t_ps, t_sc, t_pad) else None
        pyr_kernels = "pyr_scharr_kernel x levels + scharr_kernel (coarsest) + pad_batched_kernel (borders)"
    else:
        # the left chain (Scharr on): pyr_scharr_kernel<NT, true, XT> + pyr_chain_kernel<c, true, s>
        t_ps = pmc_traffic(args.config, "pyr_scharr_kernel", Sq, PYR_LEFT_TARGS)
        t_ch = pmc_traffic(args.config, "pyr_chain_kernel", Sq, CHAIN_LEFT_TARGS)
        pyr_traffic = (c_lev - 1) * t_ps + t_ch if None not in (t_ps, t_ch) else None
        pyr_kernels = (f"pyr_scharr_kernel x {c_lev - 1} (pyrDown + Scharr + the source level's border) + "
                       "pyr_chain_kernel (last two levels, their derivatives and borders)")
    # FAST detection (the pre-detection stage: FAST-9 + cornerScore + NMS, unmasked)
    # of the last frame of every sequence, timed alone the same way; algorithmic
    # bytes = one read of each W x H u8 frame (one raster pass)
    fast_avg_s = fe.time_fast(Wm + K, 20) / 1e3 if hasattr(fe, "time_fast") else 0.0
    fast_bytes = Sq * W * H
    fast_traffic = pmc_traffic(args.config, "fast_detect_q_kernel", Sq)  # one instance per config
    print("[bench] timed window done", file=sys.stderr, flush=True)
    if legs_after:
        side_legs(close_fe=fe.close)
    single, bucketed, forward, orb, stream, opencv_order = (
        side[k] for k in ("single", "bucketed", "forward", "orb", "stream", "opencv_order"))
    out = {
        "metric": "frames/sec @1241x376, 2000 feats; LK iters/sec; achieved HBM GB/s",
        "value": round(fps, 2),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": K,
        "warmup": Wm,
        "ms_per_step": round(dt_max / K * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8/int32 fixed-point (LK sums exact int, solve f32), f64 PnP",
        "data": "synthetic (rendered KITTI-size frames, seeded; no dataset on the box)"
                + ("; SceneForward (translation + moving occluder)" if args.scene == "forward" else ""),
        "config": {"workload": label, "sequences_per_gpu": Sq, "global_batch": Sq * world,
                   "features": N, "win": 21, "max_level": ML, "parallelism": f"{world} x independent sequences",
                   "host_cpus_rank0": len(host_cpus)},
        "lk_iters_per_s": round(lk_iters_total / dt_max, 1),
        "achieved_GBps_algorithmic": round(frames * frame_bytes(W, H, N, ML) / dt_max / 1e9, 2),
        "side_legs": "after" if legs_after else "first",
        "single_stream_fps": round(single, 2) if single else None,
        "bucketed": bucketed,
        "workloads": {"forward": forward, "orb_reference": orb, "stream": stream, "opencv_order": opencv_order},
        "phase_ms_per_step": {k: round(v[0] / K, 4) for k, v in phases.items()},
        "stats_per_step": {k: round(v / K, 3) for k, v in tot.items()},
        "step_ms": {"mean": round(float(np.mean(step_s)) * 1e3, 4),
                    "median": round(float(np.median(step_s)) * 1e3, 4), "p90": round(float(np.percentile(step_s, 90)) * 1e3, 4),
                    "max": round(max(step_s) * 1e3, 4), "min": round(min(step_s) * 1e3, 4),
                    "all": [round(x * 1e3, 3) for x in step_s]},
        "slowest_step": slowest_step(step_s, step_diag, Wm),
        "roofline": {
            "kernel": f"{lk_name}> (temporal LK 21x21, all levels, {lk_desc})",
            "dominant_phase": dominant,
            "bound": "hbm",
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "traffic": traffic,
            "algorithmic_bytes_per_launch": int(bytes_per_launch),
            "units_per_launch": round(units_per_launch, 1),
            "bytes_per_unit": lk_bytes_per_feature(L),
            "avg_launch_us": round(lk_avg_s * 1e6, 3),
            "launches_timed": lk_n,
        },
        "roofline_valu": roofline_valu(lk_name, Sq, lk_avg_s, args.config),
        "roofline_pyramid": {
            "kernel": f"pyramid chain: {pyr_kernels}; one new left frame of {Sq} sequences per launch",
            "bound": "hbm",
            "achieved": round(pyr_bytes / pyr_avg_s / 1e9, 2) if pyr_avg_s > 0 else 0.0,
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(pyr_bytes / pyr_avg_s / 1e9 / HBM_PEAK_GBPS, 4) if pyr_avg_s > 0 else 0.0,
            "traffic": pyr_traffic,
            "algorithmic_bytes_per_launch": pyr_bytes,
            "derivative_bytes_per_launch": der_bytes,
            "achieved_incl_derivatives": round((pyr_bytes + der_bytes) / pyr_avg_s / 1e9, 2) if pyr_avg_s > 0 else 0.0,
            # PMC bytes over the algorithmic bytes: SURVEY's B_pyr counts the image levels
            # only; the chain also writes each level's Scharr pair (int16 Ix, Iy per pixel),
            # the plane OpenCV's calcOpticalFlowPyrLK computes per call and per level
            # (lkpyramid.cpp: calcSharrDeriv into derivIBuf) -- written once per frame here
            # and read by both of the reference's LK calls on that frame (stereo, and the
            # next step's temporal call)
            "traffic_over_algorithmic": round(pyr_traffic / pyr_bytes, 3) if pyr_traffic else None,
            "traffic_over_algorithmic_incl_derivatives": (round(pyr_traffic / (pyr_bytes + der_bytes), 3)
                                                          if pyr_traffic else None),
            "avg_launch_us": round(pyr_avg_s * 1e6, 3),
            "timing": "alone, 20 launches (HIP events on the launch stream)",
            "in_step_avg_launch_us": round(pyr_instep_s * 1e6, 3),
        },
        "roofline_fast": {
            "kernel": f"fast_detect_q_kernel<32> (FAST-9 + cornerScore + NMS, 64x32 tiles), {Sq} frames per launch",
            "bound": "hbm",
            "achieved": round(fast_bytes / fast_avg_s / 1e9, 2) if fast_avg_s > 0 else 0.0,
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(fast_bytes / fast_avg_s / 1e9 / HBM_PEAK_GBPS, 4) if fast_avg_s > 0 else 0.0,
            "traffic": fast_traffic,
            "algorithmic_bytes_per_launch": fast_bytes,
            "avg_launch_us": round(fast_avg_s * 1e6, 3),
            "timing": "alone, 20 launches (HIP events on the launch stream; includes the row-count reset)",
        },
    }
    if not args.no_cpu_baseline and world == 1:  # rank 0 at N = 1 only
        print("[bench] CPU baseline (oracle loop)", file=sys.stderr, flush=True)
        out["cpu_baseline"] = cpu_baseline(args.config, args.cpu_seconds)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
