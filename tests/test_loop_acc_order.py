"""LK accumulation order through the loop (CPU only, oracle vs oracle).

The product's LK has two summation modes. SVO_LK_OPENCV_ORDER (the drop-in
Tracking mirror's default) sums the normal equations in OpenCV's own float
SSE-lane order and equals the oracle's ACC_SSE bit for bit -- per call and
through 200 frames of the loop, with no exemption (tests/test_lk_opencv_order_gpu.py).
The batched benchmark front end's default sums exactly (integers, one rounding:
lk.hip) and equals the oracle's ACC_EXACT bit for bit (the GPU suite). This file
characterises only that second, documented choice: what exact sums instead of
OpenCV's float order do to the reference's loop
(R:src/tracking.cpp:154-179 trackFrames, :181-230 calculatePose) on the
KITTI-size bench scene and the forward / occluder scene:

* lockstep -- both orders from the same state every step (per-call deviation):
  no status flips, identical RANSAC inlier index sets and hypothesis counts,
  poses within 1e-5, and every tracked point within 0.1 px unless the point ran
  into the 50-iteration cap at some level (non-converging, oscillating windows --
  there the two orders may stop at different points of the oscillation);
* free-running -- two independent loops: the feature lists stay close and the
  poses within 1e-3.

The full 200-frame record is profiles/r05/acc_order.txt (tools/acc_order_report.py).
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
from acc_order_report import free_running, lockstep, summarize_free, summarize_lockstep  # noqa: E402

from svo_amd.scene import Scene, SceneForward  # noqa: E402


def _check_lockstep(rows):
    for r in rows:
        assert r["flips"] == 0, r
        assert r["inlier_symdiff"] == 0, r
        assert r["hyp_equal"], r
        assert r["pose_d"] <= 1e-5, r
        assert r["over_01_uncapped"] == 0, r
        assert r["max_d_converged"] <= 0.1, r


def test_lockstep_sse_order_kitti_scene():
    rows = lockstep(Scene(1241, 376, seed=0), 40)
    print(summarize_lockstep("Scene(1241x376, seed 0)", rows))
    _check_lockstep(rows)
    # the orders do differ (this is not a vacuous comparison)
    assert sum(r["differ"] for r in rows) > 1000


def test_lockstep_sse_order_forward_scene():
    rows = lockstep(SceneForward(1241, 376, seed=1), 20)
    print(summarize_lockstep("SceneForward(1241x376, seed 1)", rows))
    _check_lockstep(rows)


def test_free_running_sse_order_stays_close():
    rows = free_running(Scene(1241, 376, seed=0), 50)
    print(summarize_free("Scene(1241x376, seed 0)", rows))
    for r in rows:
        assert r["pose_d"] <= 1e-3, r
        for k, (x, y) in r["count_d"].items():
            if k != "hypotheses":
                assert abs(x - y) <= 5, r
    assert np.mean([bool(r["count_d"]) for r in rows]) <= 0.25
