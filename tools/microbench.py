#!/usr/bin/env python3
"""Kernel micro-benchmarks through the C ABI (for rocprofv3 runs).

    python tools/microbench.py lk --points 128000 --reps 5 [--cv]
    python tools/microbench.py pyr --reps 20
    python tools/microbench.py fast --reps 20
    python tools/microbench.py fepyr --reps 20 --seq 64   (the front end's batched pyramid chain)
    python tools/microbench.py fefast --reps 20 --seq 64  (the front end's batched FAST detection)
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import svo_amd as S  # noqa: E402
from svo_amd.scene import Scene  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["lk", "pyr", "fast", "stereo", "fepyr", "fefast", "epnp"])
    ap.add_argument("--seq", type=int, default=64)
    ap.add_argument("--points", type=int, default=128000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--w", type=int, default=1241)
    ap.add_argument("--h", type=int, default=376)
    ap.add_argument("--count", type=int, default=0, help="override the LK iteration cap")
    ap.add_argument("--cv", action="store_true", help="LK in OpenCV's float order (SVO_LK_OPENCV_ORDER)")
    args = ap.parse_args()
    ctx = S.Context(0)
    sc = Scene(args.w, args.h, seed=0)
    A, B = sc.frame(0), sc.frame(1)
    ga, gb = ctx.image(A, 4), ctx.image(B, 4)
    if args.what in ("lk", "stereo"):
        kp = ctx.fast_detect(ga, 20, True)[:, :2]
        reps = -(-args.points // len(kp))
        rng = np.random.default_rng(0)
        pts = np.concatenate([kp + rng.uniform(-0.5, 0.5, kp.shape).astype(np.float32) * (i > 0)
                              for i in range(reps)])[: args.points]
        win, crit, flags = ((21, 21), (3, 50, 1e-3), S.LK_GET_MIN_EIGENVALS) if args.what == "lk" else \
            ((11, 11), (3, 30, 1e-3), 0)
        if args.count:
            crit = (crit[0], args.count, crit[2])
        if args.cv:
            flags |= S.LK_OPENCV_ORDER
        for r in range(args.reps):
            t = time.perf_counter()
            ctx.calc_optical_flow_pyr_lk(ga, gb, pts, win_size=win, max_level=3, criteria=crit, flags=flags)
            dt = time.perf_counter() - t
            print(f"{args.what} {len(pts)} pts: {dt*1e3:.3f} ms (host incl. copies), iters {ctx.lk_last_iterations()}")
    elif args.what == "pyr":
        for r in range(args.reps):
            ga.upload(A)
        print("pyr done")
    elif args.what == "fefast":
        cfg = S.FrontendConfig(args.w, args.h, sc.K, n_seq=args.seq, n_frames=2, n_features=2000, max_level=3)
        fe = S.Frontend(ctx, cfg)
        for s_ in range(args.seq):
            sq = Scene(args.w, args.h, seed=s_)
            fe.set_frame(s_, 0, sq.frame(0), sq.right(0))
            fe.set_frame(s_, 1, sq.frame(1), sq.right(1))
        for r in range(3):
            ms = fe.time_fast(1, args.reps)
            print(f"fefast {args.seq} x {args.w}x{args.h}: {ms * 1e3:.1f} us per launch")
    elif args.what == "fepyr":
        cfg = S.FrontendConfig(args.w, args.h, sc.K, n_seq=args.seq, n_frames=2, n_features=2000, max_level=3)
        fe = S.Frontend(ctx, cfg)
        for s_ in range(args.seq):
            for t in range(2):
                fe.set_frame(s_, t, A if t == 0 else B, B)
        ms = fe.time_pyramid(1, args.reps)
        print(f"fepyr {args.seq} x {args.w}x{args.h}: {ms * 1e3:.1f} us per chain")
    elif args.what == "epnp":
        # RANSAC's EPnP: device 6 (a GPU lane per subset) vs device 0 (host SIMD
        # lanes + pool); host wall per call, the kernel time from rocprof
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
        from test_epnp_cpu import K as KE, subsets
        for m in (64, 256, 512, 4096):
            subs = subsets(7, m, 0.5)[0]
            for dev in (0, 6):
                ctx.epnp_subsets(subs, KE, device=dev)
                t = time.perf_counter()
                for r in range(args.reps):
                    ctx.epnp_subsets(subs, KE, device=dev)
                dt = (time.perf_counter() - t) / args.reps
                print(f"epnp m={m} device={dev}: {dt * 1e6:.1f} us per call ({dt * 1e6 / m:.2f} us per subset)")
    elif args.what == "fast":
        for r in range(args.reps):
            kp = ctx.fast_detect(ga, 20, True)
        print("fast", len(kp))


if __name__ == "__main__":
    main()
