"""How much of each derivative level the temporal LK reads (CPU only).

The pyramid chain writes the x4 Scharr pairs (Ix | Iy << 16, 4 B per pixel) of every
level of every new left frame, full frame; the temporal LK of the NEXT step reads them
only inside its features' windows: at level L the 22 x 22 block (21 x 21 window + the
bilinear column / row) whose corner is floor(p / 2^L - 10) for every tracked feature p
of the frame (R:src/tracking.cpp:160-165 -> lkpyramid.cpp: the derivative window is
sampled at the PREVIOUS position, which does not move during the iterations).

This replays the benchmark's loop (tests/oracle_loop.py: every frame a keyframe topping
the set up to 2,000) on the bench scene and the forward / occluder scene and prints, per
level, the fraction of the level's pixels inside the union of the windows, and the
derivative bytes a density-exact writer would have written against the full-frame ones.

    python tools/deriv_coverage.py [--steps 8]
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

from oracle_loop import OracleLoop  # noqa: E402
from svo_amd.scene import Scene, SceneForward  # noqa: E402

WIN, MAX_LEVEL = 21, 3


def coverage(pts, w, h):
    out = []
    for lv in range(MAX_LEVEL + 1):
        # level sizes as cv::buildOpticalFlowPyramid: (w + 1) / 2 per level
        lw, lh = w, h
        for _ in range(lv):
            lw, lh = (lw + 1) // 2, (lh + 1) // 2
        m = np.zeros((lh, lw), bool)
        p = pts.astype(np.float32) * np.float32(1.0 / (1 << lv)) - np.float32((WIN - 1) * 0.5)
        ix = np.floor(p[:, 0]).astype(int)
        iy = np.floor(p[:, 1]).astype(int)
        for x, y in zip(ix, iy):
            x0, y0 = max(x, 0), max(y, 0)
            x1, y1 = min(x + WIN + 1, lw), min(y + WIN + 1, lh)
            if x1 > x0 and y1 > y0:
                m[y0:y1, x0:x1] = True
        out.append((lw * lh, int(m.sum())))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=8)
    a = ap.parse_args()
    for name, sc in (("Scene(1241x376, seed 0)", Scene(1241, 376, seed=0)),
                     ("SceneForward(1241x376, seed 1)", SceneForward(1241, 376, seed=1))):
        loop = OracleLoop(sc).init(0)
        acc = np.zeros((MAX_LEVEL + 1, 2))
        for t in range(1, a.steps + 1):
            cov = coverage(loop.pts, 1241, 376)  # the windows LK(t) reads in frame t - 1
            acc += np.array(cov, float)
            loop.step(t)
        print(name, f"({a.steps} steps, {len(loop.pts)} features at the end)")
        full = read = 0.0
        for lv in range(MAX_LEVEL + 1):
            n, c = acc[lv]
            print(f"  level {lv}: {c / n:6.3f} of the level's pixels inside the windows")
            full += n
            read += c
        print(f"  derivative bytes: read-density writer {read / full:.3f} of the full-frame writer's "
              f"({4 * full / a.steps / 1e6:.2f} MB per frame full)")


if __name__ == "__main__":
    main()
