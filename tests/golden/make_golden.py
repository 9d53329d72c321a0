#!/usr/bin/env python3
"""Regenerate the committed golden fixtures (tests/golden/*.npz) from the oracle.

The reference has no tests and OpenCV is absent, so these fixtures are the
oracle's outputs on seeded synthetic inputs: they pin the
oracle against drift and give the GPU tests a stored answer. Inputs are
rendered by svo_amd's host-side synthetic generator (deterministic C code).

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import oracle as O  # noqa: E402
from svo_amd.scene import Scene  # noqa: E402


def main():
    sc = Scene(160, 120, seed=11)
    A, B = sc.frame(0), sc.frame(1)
    pyr = O.build_pyramid(A, (21, 21), 3)
    kp_nms = O.fast(A, 20, True)
    kp_all = O.fast(A, 20, False)
    mask = O.mask_boxes(160, 120, kp_nms[::4, :2] + np.float32(0.5), 10.0)
    kp_mask = O.fast(A, 20, True, mask)
    pts = kp_nms[:, :2].copy()
    t_n, t_s, t_e, _ = O.lk(A, B, pts, (21, 21), 3, (3, 50, 1e-3), O.LK_GET_MIN_EIGENVALS)
    s_n, s_s, s_e, _ = O.lk(A, B, pts, (11, 11), 3, (3, 30, 1e-3), 0)
    bx, ba = O.bucket(kp_all[:, :2], 160, 120, 50, 2)
    X = sc.map_points(pts, 0)
    rc, rv, tv, inl, _ = O.solve_pnp_ransac(X, t_n, sc.K)
    np.savez_compressed(os.path.join(HERE, "small_160x120.npz"), A=A, B=B,
                        **{f"pyr{l}": pyr[l] for l in range(1, len(pyr))},
                        kp_nms=kp_nms, kp_all=kp_all, mask=mask, kp_mask=kp_mask,
                        pts=pts, t_next=t_n, t_status=t_s, t_err=t_e,
                        s_next=s_n, s_status=s_s, s_err=s_e,
                        bucket_xy=bx, X=X, K=sc.K, pnp_rvec=rv, pnp_tvec=tv, pnp_inliers=inl)
    print("wrote small_160x120.npz:", len(kp_nms), "kps,", int(t_s.sum()), "tracked,", len(inl), "inliers")

    # colour ingest + ORB: a BGR frame whose channels differ,
    # its grey conversion, and ORB(150 and 500 features) with and without a box mask
    sc2 = Scene(320, 240, seed=12)
    g0 = sc2.frame(0)
    bgr = np.ascontiguousarray(np.stack([g0, np.roll(g0, 3, axis=1), 255 - g0], axis=2))
    gray = O.bgr2gray(bgr)
    kq = O.fast(gray, 20, True)[::5, :2]
    omask = O.mask_boxes(320, 240, kq, 10.0)
    orb150, oct150 = O.orb_detect(gray, None, nfeatures=150)
    orb500m, oct500m = O.orb_detect(gray, omask, nfeatures=500)
    np.savez_compressed(os.path.join(HERE, "orb_ingest_320x240.npz"), bgr=bgr, gray=gray, mask=omask,
                        orb150=orb150, oct150=oct150, orb500m=orb500m, oct500m=oct500m)
    print("wrote orb_ingest_320x240.npz:", len(orb150), "/", len(orb500m), "ORB keypoints")


if __name__ == "__main__":
    main()
