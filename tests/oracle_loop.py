"""The reference's per-frame tracking loop composed from oracle pieces (TEST
INFRASTRUCTURE / CPU baseline only).

Mirrors Tracking::startStereo (R:src/tracking.cpp:232-276) as the batched
frontend runs it, every frame a keyframe that tops the feature set up:
  trackFrames     :154-179  temporal LK 21x21, maxLevel 3, {COUNT+EPS,50,1e-3}, MIN_EIGENVALS; keep status
  calculatePose   :181-230  solvePnPRansac(100, 8.0, 0.999, SQPNP); drop outliers;
                            pose = inverse([R(rvec) | tvec]) (identity without a model)
  extractFeatures :74-92    mask = boxes(+-10) around prevFrame's features; FAST(20, NMS) with mask
  (top-up)                  the first n_features - n keypoints (optionally bucketed)
  findLeftFeaturesInRight :94-118  stereo LK 11x11, maxLevel 3, {COUNT+EPS,30,1e-3}; status && |yR-yL| < 40
  triangulateNewMapPoints :120-152 DLT(P_left, P_right), z > 0, world = pose * p
"""
from __future__ import annotations

import numpy as np

import oracle as O

TEMPORAL = dict(win=(21, 21), max_level=3, criteria=(3, 50, 1e-3), flags=O.LK_GET_MIN_EIGENVALS)
STEREO = dict(win=(11, 11), max_level=3, criteria=(3, 30, 1e-3), flags=0)
Y_THRESHOLD = np.float32(40.0)  # R:configs/config.yaml:16 (float, R:include/config_reader.h:41)


def pose_inverse(rv, tv):
    """Frame::pose() from the solvePnPRansac model: [R(rvec) | tvec]^-1 as
    svo::SE3d::inverse evaluates it (R^T, -(R^T t)), operation by operation."""
    R = O.rodrigues(np.asarray(rv, np.float64))
    T = R.T.copy()
    t = np.array([-(T[i, 0] * tv[0] + T[i, 1] * tv[1] + T[i, 2] * tv[2]) for i in range(3)])
    return T, t


def transform(T, t, X):
    """T * p for float32 camera points (as Eigen::Vector3d{p.x, p.y, p.z}), left to right."""
    x, y, z = (X[:, k].astype(np.float64) for k in range(3))
    return np.stack([T[i, 0] * x + T[i, 1] * y + T[i, 2] * z + t[i] for i in range(3)], axis=1)


class OracleLoop:
    def __init__(self, scene, n_features=2000, bucket=(0, 0), acc=O.ACC_EXACT, max_level=TEMPORAL["max_level"],
                 rule="every", features_to_track=70, detector="fast", orb=None, nonmax=True):
        """max_level: the temporal LK's (BASELINE configs: 3 at KITTI and 4K, 4 at
        1080p); the stereo LK keeps the reference's maxLevel 3.
        rule: "every" -- every frame a keyframe topping the set up to n_features
        (the benchmark's loop); "reference" -- Tracking::nextFrame's rule
        (R:src/tracking.cpp:68-69): a keyframe iff the previous frame was not one
        and kept fewer than features_to_track features; a keyframe takes every
        masked corner (extractFeatures, :74-92) -- n_features is only the
        capacity, and stats["kf_overflow"] counts the corners it had no room for
        (the reference's loop has no cap: a test sizes the capacity so that this
        stays 0).
        nonmax: FAST's nonmaxSuppression. The struct default is true
        (R:include/config_reader.h:37); the shipped YAML spells the key
        `nonmaxsuppression` (R:configs/config.yaml:31) while the reader looks up
        `nonMaxSuppression` (R:include/config_reader.h:80), so with use_orb: 0 the
        shipped config runs FAST WITHOUT suppression."""
        self.sc, self.N, self.bucket, self.acc = scene, n_features, bucket, acc
        self.nonmax = nonmax
        self.max_level = max_level
        self.rule, self.features_to_track = rule, features_to_track
        self.detector, self.orb = detector, dict(orb or {})
        self.P_left, self.P_right = scene.projections()

    def _candidates(self, img, mask):
        """extractFeatures' detect (R:src/tracking.cpp:82): FAST(20, nonmax) or, with
        detector="orb", cv::ORB (R:src/tracking.cpp:35-52: the shipped config's
        150 features, scale 1.2, 8 levels, patch / edge 31, FAST 20, HARRIS)."""
        if self.detector == "orb":
            return O.orb_detect(img, mask, **self.orb)[0][:, :2]
        kp = O.fast(img, 20, self.nonmax, mask)[:, :2]
        if self.bucket[0] > 0:
            kp, _ = O.bucket(kp, img.shape[1], img.shape[0], self.bucket[0], self.bucket[1])
        return kp

    def _keyframe(self, left, right, cand, T, t):
        """findLeftFeaturesInRight + triangulateNewMapPoints of the candidate points."""
        new = np.ascontiguousarray(cand, np.float32)
        if len(new) == 0:
            return new.reshape(0, 2), np.zeros((0, 3))
        nr, st, _, _ = O.lk(left, right, new, STEREO["win"], STEREO["max_level"], STEREO["criteria"],
                            STEREO["flags"], acc=self.acc, want_err=False)
        keep = (st == 1) & (np.abs(nr[:, 1] - new[:, 1]) < Y_THRESHOLD)
        newL, newR = new[keep], nr[keep]
        _, xyz = O.triangulate(self.P_left, self.P_right, newL, newR)
        front = xyz[:, 2] > 0
        return newL[front], transform(T, t, xyz[front])

    def init(self, t0=0, left=None, right=None):
        self.t = t0
        self.img = self.sc.frame(t0) if left is None else left
        right = self.sc.right(t0) if right is None else right
        cand = self._candidates(self.img, None)
        self.init_overflow = max(len(cand) - self.N, 0)
        cand = cand[: self.N]
        self.pose_T = (np.eye(3), np.zeros(3))
        self.pts, self.X = self._keyframe(self.img, right, cand, *self.pose_T)
        self.pose = (np.zeros(3), np.zeros(3))
        self.kf_prev = True  # frame t0 is a keyframe (lastFrameID == 0)
        return self

    def step(self, t, left=None, right=None):
        B = self.sc.frame(t) if left is None else left
        Br = self.sc.right(t) if right is None else right
        nx, st, _, it = O.lk(self.img, B, self.pts, TEMPORAL["win"], self.max_level, TEMPORAL["criteria"],
                             TEMPORAL["flags"], acc=self.acc, want_err=False)
        keep = st == 1
        p2, X2 = nx[keep], self.X[keep]
        stats = {"lk_iterations": int(it.sum()), "tracked": int(keep.sum())}
        rv, tv = np.zeros(3), np.zeros(3)
        self.last_pnp = (X2, p2, 0)  # the RANSAC's inputs (tests replay its hypotheses)
        if len(p2) >= 4:
            rc, rv_, tv_, inl, nh = O.solve_pnp_ransac(X2, p2, self.sc.K)
            self.last_pnp = (X2, p2, nh)
            if rc == 1:
                p2, X2 = p2[inl], X2[inl]
                rv, tv = rv_, tv_
            else:  # no model: every feature is an outlier (R:src/tracking.cpp:218-229)
                p2, X2 = p2[:0], X2[:0]
            stats["hypotheses"] = nh
        self.pose = (rv, tv)
        self.pose_T = pose_inverse(rv, tv)
        stats["inliers"] = len(p2)
        kf = self.rule == "every" or (not self.kf_prev and len(self.pts) < self.features_to_track)
        self.kf_prev = kf
        stats["keyframe"] = int(kf)
        mask = O.mask_boxes(B.shape[1], B.shape[0], self.pts, 10.0)
        cand = self._candidates(B, mask)
        need = max(self.N - len(p2), 0) if kf else 0
        stats["kf_overflow"] = max(len(cand) - need, 0) if kf and self.rule == "reference" else 0
        newL, newX = self._keyframe(B, Br, cand[:need], *self.pose_T)
        self.pts = np.concatenate([p2, newL]).astype(np.float32)
        self.X = np.concatenate([X2, newX]) if len(newL) else X2
        stats["added"] = len(newL)
        stats["features"] = len(self.pts)
        self.img = B
        self.t = t
        return stats
