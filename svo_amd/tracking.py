"""ctypes binding of libsvo_tracking.so (include/svo_tracking.h): the host C++
mirror of the reference's Tracking (R:include/tracking.h) driven frame by frame.

    tr = Tracking(calib24, features_to_track=70)
    tr.push(left, right); tr.step()        # initial keyframe
    tr.push(left, right); tr.step()        # trackFrames -> calculatePose (-> keyframe path)
    tr.frame_info(), tr.features(), tr.trace("lk_next")
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import SvoError, lib as _gpu_lib

_LIB = None
_u8p = C.POINTER(C.c_uint8)
_f32p = C.POINTER(C.c_float)
_f64p = C.POINTER(C.c_double)
_i64p = C.POINTER(C.c_int64)
_i32p = C.POINTER(C.c_int)
_vp = C.c_void_p


class TrackingConfig(C.Structure):
    _fields_ = [("fast_threshold", C.c_int), ("fast_nonmax", C.c_int), ("y_threshold", C.c_float),
                ("features_to_track", C.c_int), ("device", C.c_int),
                ("use_orb", C.c_int), ("orb_nfeatures", C.c_int), ("orb_scale_factor", C.c_float),
                ("orb_pyr_levels", C.c_int), ("orb_patch_size", C.c_int), ("orb_fast_threshold", C.c_int)]


_SIGS = [
    ("svo_tracking_create", C.c_int, [C.POINTER(TrackingConfig), _f32p, C.POINTER(_vp)]),
    ("svo_tracking_destroy", None, [_vp]),
    ("svo_tracking_last_error", C.c_char_p, [_vp]),
    ("svo_tracking_push_stereo", C.c_int, [_vp, _u8p, _u8p, C.c_int, C.c_int, C.c_int]),
    ("svo_tracking_push_stereo_bgr", C.c_int, [_vp, _u8p, _u8p, C.c_int, C.c_int, C.c_int]),
    ("svo_tracking_step", C.c_int, [_vp]),
    ("svo_tracking_frame_info", C.c_int, [_vp, _i64p, _i32p, _i64p, _i64p, _f64p, _f64p]),
    ("svo_tracking_features", C.c_int, [_vp, _f32p, _f64p, _i64p, C.c_int, _i32p]),
    ("svo_tracking_trace", C.c_int64, [_vp, C.c_char_p, _vp, C.c_int64]),
]
SYMBOLS = [s[0] for s in _SIGS]

# trace field -> (dtype, columns)
TRACE_FIELDS = {
    "lk_prev": (np.float32, 2), "lk_next": (np.float32, 2), "lk_status": (np.uint8, 1),
    "pnp_obj": (np.float64, 3), "pnp_img": (np.float32, 2), "pnp_inliers": (np.int32, 1),
    "pnp_pose": (np.float64, 1), "mask_pts": (np.float32, 2), "kps": (np.float32, 2),
    "stereo_right": (np.float32, 2), "stereo_status": (np.uint8, 1), "kept_left": (np.float32, 2),
    "kept_right": (np.float32, 2), "tri_xyz": (np.float32, 3),
}


def lib_path() -> str:
    return os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libsvo_tracking.so")


def lib():
    global _LIB
    if _LIB is None:
        _gpu_lib()  # libsvo_gpu.so first (dependency, loud failure if missing)
        path = lib_path()
        if not os.path.exists(path):
            raise SvoError(f"host tracking library not built: {path} missing (run __graft_entry__.build())")
        L = C.CDLL(path)
        for name, res, args in _SIGS:
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _LIB = L
    return _LIB


class Tracking:
    """The reference's Tracking (stereo, FAST) on the GPU path, one frame per step()."""

    def __init__(self, calib, fast_threshold=20, fast_nonmax=True, y_threshold=40.0, features_to_track=70,
                 device=0, use_orb=False, orb_nfeatures=150, orb_scale_factor=1.2, orb_pyr_levels=8,
                 orb_patch_size=31, orb_fast_threshold=20):
        """Defaults: R:configs/config.yaml (its ORB block; use_orb=True is what it ships)."""
        calib = np.ascontiguousarray(calib, np.float32).reshape(24)
        cfg = TrackingConfig(int(fast_threshold), int(bool(fast_nonmax)), float(y_threshold),
                             int(features_to_track), int(device), int(bool(use_orb)), int(orb_nfeatures),
                             float(orb_scale_factor), int(orb_pyr_levels), int(orb_patch_size),
                             int(orb_fast_threshold))
        h = _vp()
        rc = lib().svo_tracking_create(C.byref(cfg), calib.ctypes.data_as(_f32p), C.byref(h))
        if rc != 0:
            raise SvoError(f"svo_tracking_create failed ({rc})")
        self.handle = h

    def close(self):
        if getattr(self, "handle", None):
            lib().svo_tracking_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def push(self, left: np.ndarray, right: np.ndarray):
        left = np.ascontiguousarray(left, np.uint8)
        right = np.ascontiguousarray(right, np.uint8)
        h, w = left.shape
        if right.shape != left.shape:
            raise ValueError("left/right sizes differ")
        if lib().svo_tracking_push_stereo(self.handle, left.ctypes.data_as(_u8p), right.ctypes.data_as(_u8p),
                                          w, h, w) != 0:
            raise SvoError("svo_tracking_push_stereo failed")

    def push_bgr(self, left: np.ndarray, right: np.ndarray):
        """Queue a colour (h, w, 3) BGR pair; grey conversion happens on the device."""
        left = np.ascontiguousarray(left, np.uint8)
        right = np.ascontiguousarray(right, np.uint8)
        h, w, c = left.shape
        if right.shape != left.shape or c != 3:
            raise ValueError("need two (h, w, 3) BGR images of one size")
        if lib().svo_tracking_push_stereo_bgr(self.handle, left.ctypes.data_as(_u8p), right.ctypes.data_as(_u8p),
                                              w, h, 3 * w) != 0:
            raise SvoError("svo_tracking_push_stereo_bgr: " + lib().svo_tracking_last_error(self.handle).decode())

    def step(self) -> bool:
        rc = lib().svo_tracking_step(self.handle)
        if rc < 0:
            raise SvoError(lib().svo_tracking_last_error(self.handle).decode())
        return rc == 1

    def frame_info(self) -> dict:
        fid, kf, nf, nmp = C.c_int64(), C.c_int(), C.c_int64(), C.c_int64()
        ir = C.c_double()
        pose = np.zeros(12, np.float64)
        if lib().svo_tracking_frame_info(self.handle, C.byref(fid), C.byref(kf), C.byref(nf), C.byref(nmp),
                                         C.byref(ir), pose.ctypes.data_as(_f64p)) != 0:
            raise SvoError("no frame yet")
        return {"id": fid.value, "keyframe": bool(kf.value), "features": nf.value, "map_points": nmp.value,
                "inlier_ratio": ir.value, "R": pose[:9].reshape(3, 3).copy(), "t": pose[9:].copy()}

    def features(self):
        n = C.c_int()
        lib().svo_tracking_features(self.handle, None, None, None, 0, C.byref(n))
        k = n.value
        xy = np.zeros((k, 2), np.float32)
        world = np.zeros((k, 3), np.float64)
        ids = np.zeros(k, np.int64)
        lib().svo_tracking_features(self.handle, xy.ctypes.data_as(_f32p), world.ctypes.data_as(_f64p),
                                    ids.ctypes.data_as(_i64p), k, C.byref(n))
        return xy, world, ids

    def trace(self, field: str) -> np.ndarray:
        dt, cols = TRACE_FIELDS[field]
        nb = lib().svo_tracking_trace(self.handle, field.encode(), None, 0)
        if nb < 0:
            raise KeyError(field)
        out = np.zeros(nb // np.dtype(dt).itemsize, dt)
        lib().svo_tracking_trace(self.handle, field.encode(), out.ctypes.data_as(_vp), nb)
        return out.reshape(-1, cols) if cols > 1 else out
