#!/usr/bin/env python3
"""Probe: the sequences of one GPU split into G front ends stepped alternately.

While the host runs one group's RANSAC / keyframe hand-off, the GPU runs the
other groups' LK, so the host's critical chain after LK overlaps device work.

    python tools/groups_probe.py --seq 256 --groups 1 2 4 --steps 20 --warmup 5
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (CONFIGS, sequence_seeds)
import svo_amd as S  # noqa: E402
from svo_amd.scene import Scene  # noqa: E402


def run(G, Sq, K, Wm, threads, pairs_all, W, H, N, ML, Kmat, shared_ctx):
    T = Wm + K + 2
    P = len(pairs_all[0])
    per = Sq // G
    ctxs = [S.Context(0)] if shared_ctx else [S.Context(0) for _ in range(G)]
    fes = []
    for g in range(G):
        ctx = ctxs[0 if shared_ctx else g]
        fe = S.Frontend(ctx, S.FrontendConfig(W, H, Kmat, n_seq=per, n_frames=T, n_features=N, max_level=ML,
                                              host_threads=threads, timing=0))
        for s in range(per):
            pairs = pairs_all[g * per + s]
            for t in range(T):
                fe.set_frame(s, t, *pairs[t % P])
        fe.init(0)
        fes.append(fe)
    for t in range(1, Wm + 1):
        for fe in fes:
            fe.step(t)
    for fe in fes:
        fe.synchronize()
    t0 = time.perf_counter()
    for t in range(Wm + 1, Wm + K + 1):
        for fe in fes:
            fe.step(t)
    for fe in fes:
        fe.synchronize()
    dt = time.perf_counter() - t0
    for fe in fes:
        fe.close()
    return Sq * K / dt, dt / K * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seq", type=int, default=256)
    ap.add_argument("--groups", type=int, nargs="+", default=[1, 2])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--shared-ctx", action="store_true")
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    W, H, N, ML, _ = bench.CONFIGS["kitti"]
    seeds = bench.sequence_seeds(0, a.seq)
    scenes = [Scene(W, H, seed=sd) for sd in seeds]
    P = min(a.warmup + a.steps + 2, 2 * scenes[0].period)
    pairs_all = []
    for i, sc in enumerate(scenes):
        pairs_all.append([(sc.frame(t), sc.right(t)) for t in range(P)])
        if i % 64 == 63:
            print(f"[probe] {i + 1} sequences rendered", flush=True)
    for r in range(a.reps):
        for G in a.groups:
            fps, ms = run(G, a.seq, a.steps, a.warmup, a.threads, pairs_all, W, H, N, ML, scenes[0].K, a.shared_ctx)
            print(f"groups {G} x {a.seq // G} seq: {fps:10.1f} frames/s  {ms:.3f} ms per step", flush=True)


if __name__ == "__main__":
    main()
