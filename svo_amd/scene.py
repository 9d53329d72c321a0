"""Deterministic synthetic scenes for the parity tests and the bench.

The reference reads KITTI sequence 00 (R:configs/config.yaml:2-4); KITTI is not
available here, so frames are rendered from a textured canvas (random
rectangles, 3x3 box blur, +-3 noise) by a pinhole camera that only rotates.
Per frame the camera turns so that the image moves by about (+1.37, -0.82) px
and rolls 0.25 deg (ping-pong over `period` frames so the view stays on the
canvas): frame-to-frame motion is the homography K R K^-1, the same order of
motion as the survey's similarity warp, and a 3D point placed at ANY depth on
a canvas ray reprojects exactly. The canvas surface sits on a smooth depth
field, and a rectified right view (`right`) renders it with the disparity
fx * b / depth, so stereo LK + triangulation recover the depth.
"""
from __future__ import annotations

import ctypes as C
import math
import os

import numpy as np

from . import SvoError

_u8p = C.POINTER(C.c_uint8)
_f64p = C.POINTER(C.c_double)
_SYNTH = None
# include/svo_synth.h (libsvo_synth.so: host code, tests and bench only)
_SYNTH_SIGS = [
    ("svo_synth_canvas", C.c_int, [C.c_uint64, C.c_int, C.c_int, C.c_int, _u8p]),
    ("svo_synth_frame", C.c_int, [_u8p, C.c_int, C.c_int, C.c_int, C.c_int, _f64p, _f64p,
                                  C.c_uint64, C.c_int, _u8p, C.c_int, C.c_int]),
    ("svo_synth_frame_right", C.c_int, [_u8p, C.c_int, C.c_int, C.c_int, C.c_int, _f64p, _f64p,
                                        C.c_double, C.c_int, C.c_uint64, C.c_int, _u8p, C.c_int, C.c_int]),
    ("svo_synth_view", C.c_int, [_u8p, C.c_int, C.c_int, C.c_int, C.c_int, _f64p, _f64p, _f64p, C.c_int, _f64p,
                                 C.c_int, _u8p, C.c_int, C.c_int, C.c_uint64, C.c_int, _u8p, C.c_int, C.c_int]),
]
SYNTH_SYMBOLS = [s[0] for s in _SYNTH_SIGS]


def synth_lib_path() -> str:
    return os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libsvo_synth.so")


def _synth_lib():
    global _SYNTH
    if _SYNTH is None:
        path = synth_lib_path()
        if not os.path.exists(path):
            raise SvoError(f"synthetic input library not built: {path} missing (run __graft_entry__.build())")
        L = C.CDLL(path)
        for name, res, args in _SYNTH_SIGS:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _SYNTH = L
    return _SYNTH


def _p(a, t):
    return a.ctypes.data_as(t)


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


def synth_canvas(seed: int, cw: int, ch: int, n_rect: int) -> np.ndarray:
    out = np.empty((ch, cw), np.uint8)
    if _synth_lib().svo_synth_canvas(seed, cw, ch, n_rect, _p(out, _u8p)) != 0:
        raise SvoError("svo_synth_canvas failed")
    return out


def synth_frame(canvas: np.ndarray, margin: tuple, R, K, noise_seed: int, noise: int, w: int,
                h: int) -> np.ndarray:
    canvas = _c(canvas, np.uint8)
    R = _c(R, np.float64).reshape(9)
    K = _c(K, np.float64).reshape(9)
    out = np.empty((h, w), np.uint8)
    ch, cw = canvas.shape
    if _synth_lib().svo_synth_frame(_p(canvas, _u8p), cw, ch, int(margin[0]), int(margin[1]), _p(R, _f64p),
                             _p(K, _f64p), noise_seed, noise, _p(out, _u8p), w, h) != 0:
        raise SvoError("svo_synth_frame failed")
    return out


def synth_view(canvas: np.ndarray, margin: tuple, R, Cw, K, depth_seed: int, occ, occ_tex, noise_seed: int,
               noise: int, w: int, h: int) -> np.ndarray:
    """svo_synth_view: the depth-field surface from camera (R, centre Cw) in front of
    the rectangles occ ((n, 5): x0, y0, x1, y1, z) textured by occ_tex."""
    canvas = _c(canvas, np.uint8)
    R = _c(R, np.float64).reshape(9)
    Cw = _c(Cw, np.float64).reshape(3)
    K = _c(K, np.float64).reshape(9)
    occ = _c(np.zeros((0, 5)) if occ is None else occ, np.float64).reshape(-1, 5)
    tex = _c(np.zeros((2, 2), np.uint8) if occ_tex is None else occ_tex, np.uint8)
    out = np.empty((h, w), np.uint8)
    ch, cw = canvas.shape
    th, tw = tex.shape
    if _synth_lib().svo_synth_view(_p(canvas, _u8p), cw, ch, int(margin[0]), int(margin[1]), _p(R, _f64p), _p(Cw, _f64p),
                            _p(K, _f64p), int(depth_seed), _p(occ, _f64p), len(occ), _p(tex, _u8p), tw, th,
                            noise_seed, noise, _p(out, _u8p), w, h) != 0:
        raise SvoError("svo_synth_view failed")
    return out


def synth_frame_right(canvas: np.ndarray, margin: tuple, R, K, bf: float, depth_seed: int, noise_seed: int,
                      noise: int, w: int, h: int) -> np.ndarray:
    canvas = _c(canvas, np.uint8)
    R = _c(R, np.float64).reshape(9)
    K = _c(K, np.float64).reshape(9)
    out = np.empty((h, w), np.uint8)
    ch, cw = canvas.shape
    if _synth_lib().svo_synth_frame_right(_p(canvas, _u8p), cw, ch, int(margin[0]), int(margin[1]), _p(R, _f64p),
                                   _p(K, _f64p), float(bf), int(depth_seed), noise_seed, noise, _p(out, _u8p),
                                   w, h) != 0:
        raise SvoError("svo_synth_frame_right failed")
    return out

KITTI_W, KITTI_H = 1241, 376
# R:configs/config.yaml:8-11 (fx, fy, cx, cy), held as float32 like the
# reference's cv::Matx33f K (R:include/tracking.h:55)
KITTI_FX, KITTI_FY, KITTI_CX, KITTI_CY = 718.8560, 718.8560, 607.1928, 185.2157
# fx * baseline of the synthetic stereo rig. KITTI's is 386.1448 (P1[0,3]); a
# quarter of it keeps the disparities of the 3-21 m depth field (5-32 px) in
# the range an 11x11, maxLevel-3 LK recovers, as on KITTI's far field.
STEREO_BF = 386.1448 / 4


def intrinsics(w: int, h: int) -> np.ndarray:
    """Camera matrix for a w x h synthetic frame: KITTI's, scaled; float32-rounded."""
    sx, sy = w / KITTI_W, h / KITTI_H
    K = np.array([[KITTI_FX * sx, 0, KITTI_CX * sx], [0, KITTI_FY * sx, KITTI_CY * sy], [0, 0, 1]],
                 np.float32)
    return K.astype(np.float64)


def stereo_projections(K, bf: float = STEREO_BF):
    """KITTI-style calib rows of the rectified rig (R:src/main.cpp:25-32) as float32
    3x4: left P = K[I|0], right P = K[I|0] with P[0, 3] = -fx * b."""
    P0 = np.zeros((3, 4), np.float32)
    P0[:, :3] = np.asarray(K, np.float64)
    P1 = P0.copy()
    P1[0, 3] = -bf
    return P0, P1


def rot(axis: str, a: float) -> np.ndarray:
    c, s = math.cos(a), math.sin(a)
    if axis == "x":
        return np.array([[1, 0, 0], [0, c, -s], [0, s, c]])
    if axis == "y":
        return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])


class Scene:
    """A synthetic sequence: canvas + per-frame camera rotation."""

    def __init__(self, w: int, h: int, seed: int = 0, period: int = 16, noise: int = 3,
                 shift=(1.37, -0.82), roll_deg: float = 0.25, density: float = 1 / 250.0):
        self.w, self.h, self.seed, self.period, self.noise = w, h, seed, period, noise
        self.K = intrinsics(w, h)
        fx, fy = self.K[0, 0], self.K[1, 1]
        self.yaw_rate = math.atan(shift[0] / fx)
        self.pitch_rate = math.atan(-shift[1] / fy)
        self.roll_rate = math.radians(roll_deg)
        diag = math.hypot(w, h) / 2
        span = period * max(abs(shift[0]), abs(shift[1])) + diag * math.sin(period * self.roll_rate) + 16
        self.margin = int(math.ceil(span)) + 8
        self.cw, self.ch = w + 2 * self.margin, h + 2 * self.margin
        n_rect = int(self.cw * self.ch * density)
        self.canvas = synth_canvas(seed, self.cw, self.ch, n_rect)

    def phase(self, t: int) -> float:
        p = self.period
        m = t % (2 * p)
        return float(m if m <= p else 2 * p - m)

    def R(self, t: int) -> np.ndarray:
        """World -> camera rotation of frame t."""
        s = self.phase(t)
        return rot("z", s * self.roll_rate) @ rot("x", s * self.pitch_rate) @ rot("y", s * self.yaw_rate)

    def frame(self, t: int) -> np.ndarray:
        return synth_frame(self.canvas, (self.margin, self.margin), self.R(t), self.K,
                           (self.seed << 20) + t + 1, self.noise, self.w, self.h)

    def right(self, t: int, bf: float = STEREO_BF) -> np.ndarray:
        """Right image of the rectified stereo pair at frame t (depth field surface)."""
        return synth_frame_right(self.canvas, (self.margin, self.margin), self.R(t), self.K, bf, self.seed,
                                 (self.seed << 20) + t + (1 << 19), self.noise, self.w, self.h)

    def projections(self, bf: float = STEREO_BF):
        """KITTI-style calib rows P0 (left) and P1 (right) as float32 3x4 (R:src/main.cpp:25-32)."""
        return stereo_projections(self.K, bf)

    def depth(self, cu: np.ndarray, cv: np.ndarray) -> np.ndarray:
        """Smooth positive depth field over canvas coordinates (metres)."""
        return 12.0 + 5.0 * np.sin(cu / 97.0 + self.seed) + 4.0 * np.cos(cv / 61.0 - 0.5 * self.seed)

    def map_points(self, pts: np.ndarray, t: int) -> np.ndarray:
        """World points (float64, (n,3)) of pixels `pts` observed in frame t."""
        pts = np.asarray(pts, np.float64).reshape(-1, 2)
        Ki = np.linalg.inv(self.K)
        rays = (Ki @ np.c_[pts, np.ones(len(pts))].T)          # camera rays
        rw = self.R(t).T @ rays                                 # world rays
        cu = self.K[0, 0] * rw[0] / rw[2] + self.K[0, 2]
        cv = self.K[1, 1] * rw[1] / rw[2] + self.K[1, 2]
        rho = self.depth(cu, cv)
        return (rw / rw[2] * rho).T.copy()

    def project(self, X: np.ndarray, t: int) -> np.ndarray:
        Xc = (self.R(t) @ np.asarray(X, np.float64).T)
        uv = self.K @ Xc
        return (uv[:2] / uv[2]).T


class SceneForward(Scene):
    """A harder sequence: the rotating camera of `Scene` also
    moves forward along the world z axis (ping-pong, `speed` m per frame), so the
    frames carry depth-dependent parallax (no homography maps one onto the next)
    and the depth field comes within 3 m; and a textured rectangle in the world
    plane z = `occ_z` slides sideways at `occ_px` image pixels per frame against
    the static world, so the map points on it turn into RANSAC outliers as soon
    as it has moved (defaults: 8-26 % of the tracked points dropped per frame). Both views are rendered by svo_synth_view (the right camera
    is the left one shifted by the baseline along its x axis). Frame 0: R = I,
    C = 0 (the world frame is camera 0's, as the reference's first frame)."""

    def __init__(self, w: int, h: int, seed: int = 0, period: int = 16, speed: float = 0.04,
                 occ_z: float = 8.0, occ_px: float = 22.0, occ_size=(0.35, 0.60), **kw):
        super().__init__(w, h, seed=seed, period=period, **kw)
        self.speed, self.occ_z = speed, occ_z
        fx, fy = self.K[0, 0], self.K[1, 1]
        self.occ_step = occ_px * occ_z / fx  # world metres per frame at the occluder's depth
        hw, hh = occ_z * (w / 2) / fx, occ_z * (h / 2) / fy
        self.occ_w, self.occ_h = occ_size[0] * 2 * hw, occ_size[1] * 2 * hh
        self.occ_x0, self.occ_y0 = -0.85 * hw, -0.5 * self.occ_h
        tw, th = 256, 160
        self.occ_tex = synth_canvas(seed + 7919, tw, th, tw * th // 40)

    def C(self, t: int) -> np.ndarray:
        """Camera centre of frame t (world)."""
        return np.array([0.0, 0.0, self.speed * self.phase(t)])

    def occluders(self, t: int) -> np.ndarray:
        x0 = self.occ_x0 + self.occ_step * self.phase(t)
        return np.array([[x0, self.occ_y0, x0 + self.occ_w, self.occ_y0 + self.occ_h, self.occ_z]])

    def _view(self, t: int, centre, noise_seed: int) -> np.ndarray:
        return synth_view(self.canvas, (self.margin, self.margin), self.R(t), centre, self.K, self.seed,
                          self.occluders(t), self.occ_tex, noise_seed, self.noise, self.w, self.h)

    def frame(self, t: int) -> np.ndarray:
        return self._view(t, self.C(t), (self.seed << 20) + t + 1)

    def right(self, t: int, bf: float = STEREO_BF) -> np.ndarray:
        centre = self.C(t) + self.R(t).T @ np.array([bf / self.K[0, 0], 0.0, 0.0])
        return self._view(t, centre, (self.seed << 20) + t + (1 << 19))

    def map_points(self, pts, t):  # noqa: D102 -- not a single-ray lookup any more
        raise NotImplementedError("SceneForward: 3D points come from stereo triangulation")
