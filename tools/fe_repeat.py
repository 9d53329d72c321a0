#!/usr/bin/env python3
"""Repeatability check of the batched frontend against the oracle loop: the
oracle's steps are computed once, then the frontend runs them REPS times under
each environment variant (one process), reporting the first mismatching step of
every run. For hunting schedule-dependent results (races).

    python tools/fe_repeat.py [--reps 3] [--probe] VAR=VAL[,VAR=VAL] ...
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import svo_amd as S  # noqa: E402
from oracle_loop import OracleLoop  # noqa: E402  (checker only)
from svo_amd.scene import Scene  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="*", default=[""])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--probe", action="store_true", help="read pose + map points after every step (as the tests)")
    a = ap.parse_args()
    W, H, N, T = 640, 376, 800, a.frames
    ref = OracleLoop(Scene(W, H, seed=3), N).init(0)
    want = []
    for t in range(1, T):
        rs = ref.step(t)
        want.append((rs, ref.pts.copy(), ref.X.copy()))
    sc = Scene(W, H, seed=3)
    frames = [(sc.frame(t), sc.right(t)) for t in range(T)]
    ctx = S.Context(0)
    for var in a.variants:
        env = dict(kv.split("=", 1) for kv in var.split(",") if kv)
        for k, v in env.items():
            os.environ[k] = v
        for rep in range(a.reps):
            fe = S.Frontend(ctx, S.FrontendConfig(W, H, sc.K, n_seq=1, n_frames=T, n_features=N))
            for t in range(T):
                fe.set_frame(0, t, *frames[t])
            fe.init(0)
            bad = None
            log = []
            for t in range(1, T):
                st = fe.step(t).as_dict()
                rs, pts, X = want[t - 1]
                if a.probe:
                    fe.pose(0)
                    Xg = fe.map_points(0)
                    if Xg.shape == X.shape:
                        rel = np.abs(Xg - X).max(axis=1) / np.abs(X).max(axis=1)
                        worst = int(rel.argmax())
                        log.append(f"t={t} maxrel={rel.max():.2e}@{worst} n>1e-6:{int((rel > 1e-6).sum())}")
                diff = [k for k in ("tracked", "lk_iterations", "inliers", "added", "features") if st[k] != rs[k]]
                if diff or not np.array_equal(fe.features(0), pts):
                    bad = f"t={t} " + " ".join(f"{k}:{st[k]}/{rs[k]}" for k in diff)
                    break
            fe.close()
            print(f"[{var or 'default'}] rep {rep}: {'OK' if bad is None else 'MISMATCH ' + bad} | " + "; ".join(log),
                  flush=True)
        for k in env:
            del os.environ[k]


if __name__ == "__main__":
    main()
