"""RANSAC's EPnP minimal solver in GPU lanes (svo_epnp_subsets device = 6,
epnp_lane.hip): each lane runs the front end's host solver (epnp.hpp, OpenCV's
epnp.cpp with its Jacobi SVDs restated) on one 5-point subset. Bit for bit the
oracle's EPnP (oracle/pnp.c + cvsvd.c) -- on ordinary and on degenerate subsets
(coplanar, collinear, repeated, one depth, identical pixels: non-finite models
included) -- so hypotheses solved on the device score and accept exactly as the
host's (R:src/tracking.cpp:191-196, ptsetreg.cpp's RANSAC)."""
import time

import numpy as np
import pytest

import oracle as O
import svo_amd as S
from test_epnp_cpu import K, degenerate_subsets, subsets

pytestmark = pytest.mark.gpu


def test_epnp_device_lanes_are_the_oracle():
    ctx = S.Context(0)
    subs = np.r_[subsets(41, 331, 0.5)[0], subsets(42, 130, 3.0)[0], degenerate_subsets(43, 140)]
    t0 = time.perf_counter()
    Rt, ok = ctx.epnp_subsets(subs, K, device=6)
    dt = time.perf_counter() - t0
    Rh, okh = ctx.epnp_subsets(subs, K, device=0)
    ctx.epnp_subsets(subs, K, device=6)  # (first launch: code object load)
    t0 = time.perf_counter()
    ctx.epnp_subsets(subs, K, device=6)
    dt2 = time.perf_counter() - t0
    differ = nonfinite = 0
    for k in range(len(subs)):
        rc, Ro, to = O.epnp(subs[k, :15].reshape(5, 3), subs[k, 15:].reshape(5, 2), K)
        nonfinite += rc != 0
        if rc != 0:  # a non-finite model: rejected (ok 0) -- its NaN payload bits are the ALU's own
            differ += ok[k] != 0
        else:
            differ += ok[k] != 1 or not np.array_equal(np.r_[Ro.ravel(), to].view(np.uint64), Rt[k].view(np.uint64))
    print(f"device EPnP (a lane per subset): {len(subs)} subsets in {dt * 1e3:.2f} ms first call, "
          f"{dt2 * 1e3:.2f} ms second (incl. copies), "
          f"{differ} differ from the oracle, {nonfinite} non-finite models")
    assert differ == 0
    assert nonfinite > 0
    fin = ok == 1
    assert np.array_equal(ok, okh) and np.array_equal(Rt[fin].view(np.uint64), Rh[fin].view(np.uint64))


def test_epnp_device_lanes_batch_edges():
    """Counts that leave a wave partly idle (1, 63, 64, 65) and m = 0."""
    ctx = S.Context(0)
    subs = subsets(44, 130, 0.3)[0]
    for m in (0, 1, 63, 64, 65, 130):
        Rt, ok = ctx.epnp_subsets(subs[:m], K, device=6)
        Rh, okh = ctx.epnp_subsets(subs[:m], K, device=0)
        assert ok.all() and np.array_equal(ok, okh) and np.array_equal(Rt.view(np.uint64), Rh.view(np.uint64)), m
