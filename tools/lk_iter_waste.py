#!/usr/bin/env python3
"""Iteration waste of four features per wave (CPU only, oracle).

lk_multi_kernel runs the features of a sequence four to a wave, in list order
(features pt0 .. pt0 + 3 of block pt0 / 4), and a wave iterates a level until its
slowest feature has converged: the trip count of a wave at a level is the max of its
four features' iteration counts there. This replays the temporal LK of the loop with
the oracle's per-level iteration counts (identical to the GPU's: the LK parity tests
compare them) and reports, per level and overall,

  waste = 1 - (sum of feature iterations) / (4 x sum over waves of the max),

i.e. the share of the trip loop's lane-groups that idle, for the product's grouping
(list order), for features sorted by their own previous step's total count (a schedule
the front end could compute: the kernel writes per-feature counts) and for an
oracle-ideal grouping (sorted by that step's own counts: a bound on what any regrouping
could recover, not a schedule the kernel could know).

    python tools/lk_iter_waste.py [--steps 60] > profiles/r05/i_lk_iter_waste.txt
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import oracle as O  # noqa: E402  (checker: test infrastructure)
from oracle_loop import OracleLoop, TEMPORAL  # noqa: E402
from svo_amd.scene import Scene, SceneForward  # noqa: E402

FPW = 4


def group_max(it, order=None):
    """sum over groups of FPW consecutive features (after `order`) of the max count"""
    if order is not None:
        it = it[order]
    n = len(it)
    pad = (-n) % FPW
    g = np.concatenate([it, np.zeros(pad, it.dtype)]).reshape(-1, FPW)
    return int(g.max(axis=1).sum())


def run(sc, steps, n=2000):
    E = OracleLoop(sc, n, acc=O.ACC_EXACT).init(0)
    L = E.max_level + 1
    feat = np.zeros(L)
    wave = np.zeros(L)
    ideal = np.zeros(L)
    pred = np.zeros(L)
    key = None  # each feature's iterations (all levels) at the previous step; -1: new
    for t in range(1, steps + 1):
        nx, _, _, it = O.lk(E.img, sc.frame(t), E.pts, TEMPORAL["win"], E.max_level, TEMPORAL["criteria"],
                            TEMPORAL["flags"], acc=O.ACC_EXACT, level_iters=True)
        # it: (levels, n), row l = pyramid level l (level max_level runs first)
        order = None if key is None else np.argsort(key, kind="stable")
        for lv in range(L):
            row = it[lv].astype(np.int64)
            feat[lv] += row.sum()
            wave[lv] += group_max(row)
            ideal[lv] += group_max(row, np.argsort(row, kind="stable"))
            pred[lv] += group_max(row, order)
        tot = it.sum(axis=0)
        at = {nx[i].tobytes(): i for i in range(len(nx))}
        E.step(t)
        # the kept features lead the new list in their old order; the keyframe's new ones follow
        key = np.array([tot[at[p.tobytes()]] if p.tobytes() in at else -1 for p in E.pts], np.int64)
        key[key < 0] = int(np.median(tot))
    return feat, wave, ideal, pred


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=60)
    a = ap.parse_args()
    print(__doc__.split("\n\n")[0])
    print(f"(FPW = {FPW}; {a.steps} steps per scene; level 0 = full resolution)")
    for name, sc in (("Scene(1241x376, seed 0)", Scene(1241, 376, seed=0)),
                     ("SceneForward(1241x376, seed 1)", SceneForward(1241, 376, seed=1))):
        feat, wave, ideal, pred = run(sc, a.steps)
        print(name)
        for lv in range(len(feat)):
            print(f"  level {lv}: feature iterations {feat[lv] / a.steps:9.0f}/step, wave trips x {FPW} "
                  f"{FPW * wave[lv] / a.steps:9.0f}/step, waste {1 - feat[lv] / (FPW * wave[lv]):.3f}, "
                  f"grouped by the previous step's counts {1 - feat[lv] / (FPW * pred[lv]):.3f}, "
                  f"ideal-grouping waste {1 - feat[lv] / (FPW * ideal[lv]):.3f}")
        tf, tw, ti, tp = feat.sum(), wave.sum(), ideal.sum(), pred.sum()
        print(f"  all levels: {tf / a.steps:.0f} feature iterations per step, waste {1 - tf / (FPW * tw):.3f} "
              f"(grouped by the previous step's counts {1 - tf / (FPW * tp):.3f}, ideal grouping "
              f"{1 - tf / (FPW * ti):.3f}); mean iterations per feature and level "
              f"{tf / a.steps / 2000 / len(feat):.2f}")
        sys.stdout.flush()


if __name__ == "__main__":
    main()
