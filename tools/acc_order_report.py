#!/usr/bin/env python3
"""LK accumulation order at loop level (CPU only, oracle): OpenCV's SSE float
order (oracle ACC_SSE) against the exact integer sums the product's kernels
compute (ACC_EXACT, which the GPU path equals bit for bit).

  lockstep:     every step both orders run from the SAME state (the EXACT loop's),
                so each step's numbers are the per-call deviation;
  free-running: two independent loops, one per order, over the whole sequence.

    python tools/acc_order_report.py [--rot-steps 200] [--fwd-steps 40] > profiles/r05/acc_order.txt
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import oracle as O  # noqa: E402  (checker: test infrastructure)
from oracle_loop import OracleLoop, TEMPORAL  # noqa: E402
from svo_amd.scene import Scene, SceneForward  # noqa: E402

COUNTS = ("tracked", "inliers", "added", "features", "hypotheses")


def lockstep(sc, steps, n=2000):
    E = OracleLoop(sc, n, acc=O.ACC_EXACT).init(0)
    rows = []
    for t in range(1, steps + 1):
        B = sc.frame(t)
        res = {}
        for acc in (O.ACC_EXACT, O.ACC_SSE):
            res[acc] = O.lk(E.img, B, E.pts, TEMPORAL["win"], E.max_level, TEMPORAL["criteria"], TEMPORAL["flags"],
                            acc=acc, level_iters=True)
        (ne, se, _, ie), (ns, ss, _, is_) = res[O.ACC_EXACT], res[O.ACC_SSE]
        both = (se == 1) & (ss == 1)
        d = np.abs(ne - ns).max(axis=1)
        d[~both] = 0
        capped = (ie == TEMPORAL["criteria"][1]).any(axis=0) | (is_ == TEMPORAL["criteria"][1]).any(axis=0)
        r = {"t": t, "n": len(E.pts), "differ": int(((ne != ns).any(axis=1) & both).sum()), "max_d": float(d.max()),
             "max_d_converged": float(d[~capped].max()) if (~capped).any() else 0.0,
             "over_01": int((d > 0.1).sum()), "over_01_uncapped": int(((d > 0.1) & ~capped).sum()),
             "flips": int((se != ss).sum())}
        sets, poses, hyps = [], [], []
        for nx, st in ((ne, se), (ns, ss)):
            k = st == 1
            rc, rv, tv, inl, nh = O.solve_pnp_ransac(E.X[k], nx[k], sc.K)
            sets.append(set(np.flatnonzero(k)[inl].tolist()) if rc == 1 else set())
            poses.append(np.r_[rv, tv])
            hyps.append(nh)
        r["inlier_symdiff"] = len(sets[0] ^ sets[1])
        r["hyp_equal"] = hyps[0] == hyps[1]
        r["pose_d"] = float(np.abs(poses[0] - poses[1]).max())
        rows.append(r)
        E.step(t)
    return rows


def free_running(sc, steps, n=2000):
    E = OracleLoop(sc, n, acc=O.ACC_EXACT).init(0)
    S = OracleLoop(sc, n, acc=O.ACC_SSE).init(0)
    rows = []
    for t in range(1, steps + 1):
        a, b = E.step(t), S.step(t)
        rows.append({"t": t, "count_d": {k: (a.get(k), b.get(k)) for k in COUNTS if a.get(k) != b.get(k)},
                     "pose_d": float(max(np.abs(E.pose[0] - S.pose[0]).max(), np.abs(E.pose[1] - S.pose[1]).max())),
                     "same_list": len(E.pts) == len(S.pts) and bool(np.array_equal(E.pts, S.pts))})
    return rows


def summarize_lockstep(name, rows):
    a = lambda k: np.array([r[k] for r in rows])  # noqa: E731
    return (f"{name} lockstep {len(rows)} steps, {a('n').mean():.0f} features/step: positions differing "
            f"{a('differ').sum()} ({a('differ').mean():.1f}/step); max |d| {a('max_d').max():.3g} px, over converged "
            f"features {a('max_d_converged').max():.3g} px; > 0.1 px: {a('over_01').sum()} (of them without a level at "
            f"the iteration cap: {a('over_01_uncapped').sum()}); status flips {a('flips').sum()}; RANSAC inlier-set "
            f"symmetric difference {a('inlier_symdiff').sum()}; steps with different hypothesis counts "
            f"{int((~a('hyp_equal')).sum())}; max pose |d| {a('pose_d').max():.3g}")


def summarize_free(name, rows):
    diff = [r for r in rows if r["count_d"]]
    first = next((r["t"] for r in rows if not r["same_list"]), None)
    worst = max((abs(x - y) for r in diff for k, (x, y) in r["count_d"].items() if k != "hypotheses"), default=0)
    return (f"{name} free-running {len(rows)} frames: feature lists bitwise equal through frame "
            f"{(first - 1) if first else len(rows)}; frames with any differing count {len(diff)} (first "
            f"{diff[0]['t'] if diff else None}, largest count difference {worst}); max pose |d| "
            f"{max(r['pose_d'] for r in rows):.3g}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rot-steps", type=int, default=200)
    ap.add_argument("--fwd-steps", type=int, default=40)
    args = ap.parse_args()
    print(__doc__.strip().splitlines()[0])
    for name, mk, steps in (("Scene(1241x376, seed 0)", lambda: Scene(1241, 376, seed=0), args.rot_steps),
                            ("SceneForward(1241x376, seed 1)", lambda: SceneForward(1241, 376, seed=1), args.fwd_steps)):
        t0 = time.time()
        print(summarize_lockstep(name, lockstep(mk(), steps)), flush=True)
        fr = free_running(mk(), steps)
        print(summarize_free(name, fr), flush=True)
        for r in fr:
            if r["count_d"]:
                print(f"   frame {r['t']}: " + ", ".join(f"{k} {x} vs {y}" for k, (x, y) in r["count_d"].items()))
        print(f"   ({time.time() - t0:.0f} s)", flush=True)


if __name__ == "__main__":
    main()
