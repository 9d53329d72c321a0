"""The reference's per-frame tracking loop composed from oracle pieces (TEST
INFRASTRUCTURE / CPU baseline only).

Mirrors Tracking::startStereo (R:src/tracking.cpp:232-276) as the batched
frontend runs it, keyframe-every-frame top-up mode:
  trackFrames     :154-179  temporal LK 21x21, maxLevel 3, {COUNT+EPS,50,1e-3}, MIN_EIGENVALS; keep status
  calculatePose   :181-230  solvePnPRansac(100, 8.0, 0.999, SQPNP); drop outliers
  extractFeatures :74-92    mask = boxes(+-10) around prevFrame's features; FAST(20, NMS) with mask
  (top-up)                  append the first n_features - n keypoints (optionally bucketed)
Map points of new features come from the synthetic scene's depth (the
frontend's stand-in for triangulateNewMapPoints, :120-152).
"""
from __future__ import annotations

import numpy as np

import oracle as O


class OracleLoop:
    def __init__(self, scene, n_features=2000, bucket=(0, 0), depth_seed=0, acc=O.ACC_EXACT):
        self.sc, self.N, self.bucket, self.acc = scene, n_features, bucket, acc
        self.depth_seed = depth_seed

    def _candidates(self, img, mask):
        kp = O.fast(img, 20, True, mask)[:, :2]
        if self.bucket[0] > 0:
            kp, _ = O.bucket(kp, img.shape[1], img.shape[0], self.bucket[0], self.bucket[1])
        return kp

    def init(self, t0=0):
        self.t = t0
        self.img = self.sc.frame(t0)
        cand = self._candidates(self.img, None)
        self.pts = cand[: self.N].astype(np.float32)
        self.X = self._map_points(self.pts, t0)
        return self

    def _map_points(self, pts, t):
        saved = self.sc.seed
        self.sc.seed = self.depth_seed
        try:
            return self.sc.map_points(pts, t)
        finally:
            self.sc.seed = saved

    def step(self, t, frame=None):
        B = self.sc.frame(t) if frame is None else frame
        nx, st, _, it = O.lk(self.img, B, self.pts, (21, 21), 3, (3, 50, 1e-3), O.LK_GET_MIN_EIGENVALS,
                             acc=self.acc, want_err=False)
        keep = st == 1
        p2, X2 = nx[keep], self.X[keep]
        stats = {"lk_iterations": int(it.sum()), "tracked": int(keep.sum())}
        if len(p2) >= 4:
            rc, rv, tv, inl, nh = O.solve_pnp_ransac(X2, p2, self.sc.K)
            if rc == 1:
                p2, X2 = p2[inl], X2[inl]
            self.pose = (rv, tv)
            stats["hypotheses"] = nh
        stats["inliers"] = len(p2)
        mask = O.mask_boxes(B.shape[1], B.shape[0], self.pts, 10.0)
        cand = self._candidates(B, mask)
        need = max(self.N - len(p2), 0)
        new = cand[:need].astype(np.float32)
        self.pts = np.concatenate([p2, new]).astype(np.float32)
        self.X = np.concatenate([X2, self._map_points(new, t)]) if len(new) else X2
        stats["added"] = len(new)
        stats["features"] = len(self.pts)
        self.img = B
        self.t = t
        return stats
