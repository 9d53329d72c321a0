#!/usr/bin/env python3
"""Per-step view of the bench's headline front end after init (round 5 diagnosis of
the first ~15 steps running slower than the steady state; profiles/r05/l_warmup_ab.txt):
for every step after init, the host wall time and the library's per-step statistics
(svo_frontend_stats), so that what converges over the steps shows.

    python tools/step_ramp.py [--seq 256] [--steps 40]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import svo_amd as S  # noqa: E402
from svo_amd.scene import Scene  # noqa: E402

KEYS = ("lk_iterations", "tracked", "inliers", "added", "hypotheses", "ransac_rounds", "max_hypotheses",
        "host_ms_wait_post", "host_ms_hyp", "host_ms_fit", "host_ms_wait_score", "host_ms_wait_kf",
        "host_ms_enqueue", "serial_keyframe", "spec_margin")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seq", type=int, default=256)
    ap.add_argument("--steps", type=int, default=40)
    a = ap.parse_args()
    W, H, N, ML = 1241, 376, 2000, 3
    T = a.steps + 2
    ctx = S.Context(0)
    scenes = [Scene(W, H, seed=s + 1) for s in range(a.seq)]
    P = min(T, 2 * scenes[0].period)
    fe = S.Frontend(ctx, S.FrontendConfig(W, H, scenes[0].K, n_seq=a.seq, n_frames=T, n_features=N, max_level=ML))
    for s, sc in enumerate(scenes):
        pairs = [(sc.frame(t), sc.right(t)) for t in range(P)]
        for t in range(T):
            fe.set_frame(s, t, *pairs[t % P])
        if s % 32 == 31:
            print(f"[ramp] {s + 1}/{a.seq} sequences", file=sys.stderr, flush=True)
    fe.init(0)
    print("step  wall_ms " + " ".join(KEYS))
    tp = time.perf_counter()
    for t in range(1, a.steps + 1):
        st = fe.step(t).as_dict()
        now = time.perf_counter()
        vals = []
        for k in KEYS:
            v = st.get(k)
            vals.append("-" if v is None else (f"{v:.3f}" if isinstance(v, float) else str(v)))
        print(f"{t:4d} {1e3 * (now - tp):8.3f} " + " ".join(vals), flush=True)
        tp = now
    fe.synchronize()
    fe.close()


if __name__ == "__main__":
    main()
