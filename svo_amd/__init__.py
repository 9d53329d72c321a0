"""svo_amd -- MI355X-native front end of ikryukov/svo (Python host side).

Thin ctypes layer over the C ABI of ``svo_amd/lib/libsvo_gpu.so``
(``include/svo_gpu.h``). The names mirror the OpenCV calls the reference's
``Tracking`` makes (R: = ikryukov/svo):

=================================  ===========================================
svo_amd                            reference call site
=================================  ===========================================
``Context.image`` (pyramid)         pyramid built inside calcOpticalFlowPyrLK,
                                    R:src/tracking.cpp:101, :160
``FastFeatureDetector.detect``      mDetector->detect(img, kps, mask),
                                    R:src/tracking.cpp:82 (created :54-57)
``Context.mask_boxes``              cv::rectangle(mask, ...), :76-79
``Context.bucket_features``         FeatureSet::bucketingFeatures,
                                    R:src/bucket.cpp:24-68
``Context.calc_optical_flow_pyr_lk``  cv::calcOpticalFlowPyrLK, :101-105, :160-165
``Context.pnp_residuals``           PnPRansacCallback::computeError+findInliers
``Context.solve_pnp_ransac``        cv::solvePnPRansac(..., SQPNP), :191-196
=================================  ===========================================

There is no CPU fallback: every compute call goes through the HIP kernels and
raises ``SvoError`` if the extension or a GPU is missing.
"""
from __future__ import annotations

import atexit
import ctypes as C
import os
import weakref

import numpy as np

__all__ = [
    "SvoError", "lib", "Context", "Image", "FastFeatureDetector",
    "TERM_COUNT", "TERM_EPS", "LK_USE_INITIAL_FLOW", "LK_GET_MIN_EIGENVALS", "LK_OPENCV_ORDER",
    "lib_path", "Frontend", "FrontendConfig", "FrontendStats",
]

TERM_COUNT = 1
TERM_EPS = 2
LK_USE_INITIAL_FLOW = 4
PYR_PAD = 32  # SVO_PYR_PAD: stored border of every pyramid level
LK_GET_MIN_EIGENVALS = 8
# SVO_LK_OPENCV_ORDER (not an OpenCV flag): LK's normal equations summed in OpenCV's
# own float order (its SSE build) instead of exactly -- bit-identical to
# cv::calcOpticalFlowPyrLK's x86 results (oracle ACC_SSE)
LK_OPENCV_ORDER = 0x10000

_HERE = os.path.dirname(os.path.abspath(__file__))


def lib_path() -> str:
    # SVO_GPU_LIB: another build of the same library (A/B measurements)
    return os.environ.get("SVO_GPU_LIB") or os.path.join(_HERE, "lib", "libsvo_gpu.so")


# Live handles, closed at interpreter exit in dependency order (front ends and
# images before the contexts they were made on): left to __del__, a context can
# go first and its dependants then free into a destroyed context.
_LIVE = {"frontend": weakref.WeakSet(), "image": weakref.WeakSet(), "context": weakref.WeakSet()}


def _close_all():
    for kind in ("frontend", "image", "context"):
        for obj in list(_LIVE[kind]):
            try:
                obj.close()
            except Exception:
                pass


atexit.register(_close_all)


class SvoError(RuntimeError):
    pass


_LIB = None

_u8p = C.POINTER(C.c_uint8)
_f32p = C.POINTER(C.c_float)
_f64p = C.POINTER(C.c_double)
_i32p = C.POINTER(C.c_int)
_vp = C.c_void_p

# (name, restype, argtypes) for every symbol include/svo_gpu.h declares
_SIGS = [
    ("svo_ctx_create", C.c_int, [C.c_int, C.POINTER(_vp)]),
    ("svo_ctx_destroy", None, [_vp]),
    ("svo_last_error", C.c_char_p, [_vp]),
    ("svo_ctx_synchronize", C.c_int, [_vp]),
    ("svo_version", C.c_char_p, []),
    ("svo_image_create", C.c_int, [_vp, C.c_int, C.c_int, C.c_int, C.POINTER(_vp)]),
    ("svo_image_destroy", None, [_vp, _vp]),
    ("svo_image_upload", C.c_int, [_vp, _vp, _u8p, C.c_int]),
    ("svo_image_upload_bgr", C.c_int, [_vp, _vp, _u8p, C.c_int]),
    ("svo_image_build_pyramid", C.c_int, [_vp, _vp]),
    ("svo_image_level_size", C.c_int, [_vp, C.c_int, _i32p, _i32p]),
    ("svo_image_download_level", C.c_int, [_vp, _vp, C.c_int, _u8p, C.c_int]),
    ("svo_image_scharr_level", C.c_int, [_vp, _vp, C.c_int, C.POINTER(C.c_int16), C.POINTER(C.c_int16), C.c_int]),
    ("svo_fast_detect", C.c_int, [_vp, _vp, C.c_int, C.c_int, _u8p, _f32p, C.c_int, _i32p]),
    ("svo_orb_detect", C.c_int, [_vp, _vp, _vp, _u8p, _f32p, _i32p, C.c_int, _i32p]),
    ("svo_fast_score_map", C.c_int, [_vp, _vp, C.c_int, _u8p, _u8p]),
    ("svo_mask_boxes", C.c_int, [_vp, C.c_int, C.c_int, _f32p, C.c_int, C.c_float, _u8p]),
    ("svo_bucket_features", C.c_int, [_vp, _f32p, _i32p, C.c_int, C.c_int, C.c_int, C.c_int,
                                      C.c_int, _f32p, _i32p, C.c_int, _i32p]),
    ("svo_calc_optical_flow_pyr_lk", C.c_int, [_vp, _vp, _vp, _f32p, C.c_int, _f32p, _u8p, _f32p,
                                               C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                               C.c_double, C.c_int, C.c_double]),
    ("svo_lk_last_iterations", C.c_int64, [_vp]),
    ("svo_pnp_residuals", C.c_int, [_vp, _f32p, _f32p, C.c_int, _f64p, C.c_int, _f64p, C.c_float,
                                    _f32p, _u8p, _i32p]),
    ("svo_solve_pnp_ransac", C.c_int, [_vp, _f64p, _f32p, C.c_int, _f64p, C.c_int, C.c_float,
                                       C.c_double, _f64p, _f64p, _i32p, _i32p]),
    ("svo_epnp_subsets", C.c_int, [_vp, _f32p, C.c_int, _f64p, C.c_int, _f64p, _i32p]),
    ("svo_solve_pnp_sqpnp", C.c_int, [_f64p, _f32p, C.c_int, _f64p, _f64p, _f64p]),
    ("svo_triangulate_points", C.c_int, [_vp, _f32p, _f32p, _f32p, _f32p, C.c_int, _f32p, _f32p]),
    ("svo_reprojection_jacobians", C.c_int, [_vp, _f64p, _f32p, _i32p, C.c_int, C.c_int, _f64p, _f64p,
                                             C.c_double, _f64p, _f64p, _f64p]),
    ("svo_refine_poses", C.c_int, [_vp, _f64p, _f32p, _i32p, C.c_int, C.c_int, _f64p, C.c_double, C.c_int,
                                   _f64p, _f64p, _i32p]),
    ("svo_frontend_create", C.c_int, [_vp, _vp, C.POINTER(_vp)]),
    ("svo_frontend_destroy", None, [_vp]),
    ("svo_frontend_set_frame", C.c_int, [_vp, C.c_int, C.c_int, _u8p, _u8p, C.c_int]),
    ("svo_frontend_set_frame_bgr", C.c_int, [_vp, C.c_int, C.c_int, _u8p, _u8p, C.c_int]),
    ("svo_frontend_map_points", C.c_int, [_vp, C.c_int, _f64p, C.c_int, _i32p]),
    ("svo_frontend_time_pyramid", C.c_int, [_vp, C.c_int, C.c_int, _f64p]),
    ("svo_frontend_time_fast", C.c_int, [_vp, C.c_int, C.c_int, _f64p]),
    ("svo_frontend_pyramid_level", C.c_int, [_vp, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_uint8), C.c_int]),
    ("svo_frontend_scharr_level", C.c_int, [_vp, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int16),
                                            C.POINTER(C.c_int16), C.c_int]),
    ("svo_frontend_prebuild_pyramids", C.c_int, [_vp]),
    ("svo_frontend_queue_frames", C.c_int, [_vp, C.c_int, C.POINTER(_u8p), C.POINTER(_u8p), C.c_int, C.c_int]),
    ("svo_frontend_upload_wait", C.c_int, [_vp, C.c_int]),
    ("svo_pinned_alloc", C.c_int, [C.c_size_t, C.POINTER(_vp)]),
    ("svo_pinned_free", None, [_vp]),
    ("svo_frontend_init", C.c_int, [_vp, C.c_int]),
    ("svo_frontend_step", C.c_int, [_vp, C.c_int, _vp]),
    ("svo_frontend_synchronize", C.c_int, [_vp]),
    ("svo_frontend_pose", C.c_int, [_vp, C.c_int, _f64p, _f64p]),
    ("svo_frontend_features", C.c_int, [_vp, C.c_int, _f32p, C.c_int, _i32p]),
    ("svo_frontend_phase_times", C.c_int, [_vp, _f64p, C.POINTER(C.c_int64), C.c_int]),
    ("svo_frontend_reset_times", None, [_vp]),
    ("svo_host_cpu_plan", C.c_int, [C.c_int, C.c_int, _i32p, _i32p, C.c_int, _i32p]),
    ("svo_frontend_host_cpus", C.c_int, [_vp, _i32p, C.c_int, _i32p]),
    ("svo_frontend_streams", C.c_int, [_vp, C.POINTER(_vp), C.c_int, _i32p]),
    ("svo_pool_selftest", C.c_int, [C.c_int, C.c_int, C.POINTER(C.c_int64)]),
]

SYMBOLS = [s[0] for s in _SIGS]


def solve_pnp_sqpnp(obj, img_pts, K):
    """cv::solvePnP(..., SOLVEPNP_SQPNP) -> (ok, rvec, tvec): solvePnPRansac's final
    fit (svo_solve_pnp_sqpnp, host code of the library; no GPU context)."""
    obj = _c(obj, np.float64).reshape(-1, 3)
    img_pts = _c(img_pts, np.float32).reshape(-1, 2)
    K = _c(K, np.float64).reshape(9)
    rv = np.zeros(3)
    tv = np.zeros(3)
    rc = lib().svo_solve_pnp_sqpnp(_p(obj, _f64p), _p(img_pts, _f32p), len(obj), _p(K, _f64p), _p(rv, _f64p),
                                   _p(tv, _f64p))
    if rc < 0:
        raise SvoError(f"svo_solve_pnp_sqpnp: error {rc}")
    return rc == 1, rv, tv


class PinnedBuffer:
    """Page-locked host memory (svo_pinned_alloc) viewed as a numpy array: the
    source of svo_frontend_queue_frames' H2D copies at full PCIe rate. Freed by
    close() or when the object goes away (the array view must not outlive it)."""

    def __init__(self, shape, dtype=np.uint8):
        dtype = np.dtype(dtype)
        nbytes = int(np.prod(shape)) * dtype.itemsize
        p = _vp()
        if lib().svo_pinned_alloc(nbytes, C.byref(p)) != 0 or not p.value:
            raise SvoError(f"svo_pinned_alloc({nbytes}) failed")
        self._p = p
        buf = (C.c_uint8 * nbytes).from_address(p.value)
        self.array = np.frombuffer(buf, dtype=dtype, count=int(np.prod(shape))).reshape(shape)

    def close(self):
        if getattr(self, "_p", None) is not None and self._p.value:
            self.array = None
            lib().svo_pinned_free(self._p)
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001  (interpreter shutdown)
            pass


def pool_selftest(threads=8, jobs=2000):
    """svo_pool_selftest: tasks of the front end's host pool run other than exactly
    once over `jobs` jobs of changing sizes (host code, no GPU); 0 = correct."""
    bad = C.c_int64(0)
    rc = lib().svo_pool_selftest(int(threads), int(jobs), C.byref(bad))
    if rc < 0:
        raise SvoError(f"svo_pool_selftest: error {rc}")
    return int(bad.value)


def host_cpu_plan(local_rank, local_world, gpu_node=None, cap=4096):
    """svo_host_cpu_plan: this rank's share of the node's CPUs (host code, no GPU)."""
    cpus = np.zeros(cap, np.int32)
    n = C.c_int(0)
    gn = None if gpu_node is None else np.ascontiguousarray(gpu_node, np.int32)
    rc = lib().svo_host_cpu_plan(int(local_rank), int(local_world), None if gn is None else _p(gn, _i32p),
                                 _p(cpus, _i32p), cap, C.byref(n))
    if rc != 0:
        raise SvoError(f"svo_host_cpu_plan: error {rc}")
    return cpus[:min(n.value, cap)].tolist()


def lib():
    """Load libsvo_gpu.so (built by __graft_entry__.build() / make)."""
    global _LIB
    if _LIB is None:
        path = lib_path()
        if not os.path.exists(path):
            raise SvoError(f"HIP extension not built: {path} missing (run __graft_entry__.build())")
        L = C.CDLL(path)
        ab = bool(os.environ.get("SVO_GPU_LIB"))
        for name, res, args in _SIGS:
            if ab and not hasattr(L, name):  # an older build under A/B: its missing entry points stay unbound
                continue
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _LIB = L
    return _LIB


def _p(a, t):
    return a.ctypes.data_as(t)


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


class Image:
    """A device-resident 8U image with its pyrDown pyramid (levels 0..max_levels)."""

    def __init__(self, ctx: "Context", handle, w: int, h: int, max_levels: int):
        self.ctx, self.handle, self.w, self.h, self.max_levels = ctx, handle, w, h, max_levels
        _LIVE["image"].add(self)

    def level(self, l: int) -> np.ndarray:
        L = lib()
        w, h = C.c_int(), C.c_int()
        if L.svo_image_level_size(self.handle, l, C.byref(w), C.byref(h)) != 0:
            raise SvoError(f"no level {l}")
        out = np.empty((h.value, w.value), np.uint8)
        self.ctx._check(L.svo_image_download_level(self.ctx.handle, self.handle, l, _p(out, _u8p), w.value))
        return out

    def scharr(self, l: int):
        """(ix, iy) of level l as the LK kernels read them: Scharr derivatives x 4
        (int16) -- svo_image_scharr_level."""
        L = lib()
        w, h = C.c_int(), C.c_int()
        if L.svo_image_level_size(self.handle, l, C.byref(w), C.byref(h)) != 0:
            raise SvoError(f"no level {l}")
        ix = np.empty((h.value, w.value), np.int16)
        iy = np.empty_like(ix)
        self.ctx._check(L.svo_image_scharr_level(self.ctx.handle, self.handle, l,
                                                 ix.ctypes.data_as(C.POINTER(C.c_int16)),
                                                 iy.ctypes.data_as(C.POINTER(C.c_int16)), w.value))
        return ix, iy

    def upload(self, gray: np.ndarray):
        gray = _c(gray, np.uint8)
        assert gray.shape == (self.h, self.w)
        self.ctx._check(lib().svo_image_upload(self.ctx.handle, self.handle, _p(gray, _u8p), self.w))

    def upload_bgr(self, bgr: np.ndarray):
        """H2D of an (h, w, 3) BGR image, grey conversion on the device (cvtColor BGR2GRAY)."""
        bgr = _c(bgr, np.uint8)
        assert bgr.shape == (self.h, self.w, 3)
        self.ctx._check(lib().svo_image_upload_bgr(self.ctx.handle, self.handle, _p(bgr, _u8p), 3 * self.w))

    def close(self):
        if self.handle:
            lib().svo_image_destroy(self.ctx.handle, self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class OrbParams(C.Structure):
    """svo_orb_params; defaults = the reference's ORB (R:configs/config.yaml:20-27,
    R:src/tracking.cpp:33-50: edgeThreshold = patch_size, firstLevel 0, WTA_K 4, HARRIS)."""
    _fields_ = [("nfeatures", C.c_int), ("scale_factor", C.c_float), ("nlevels", C.c_int),
                ("edge_threshold", C.c_int), ("first_level", C.c_int), ("wta_k", C.c_int),
                ("score_type", C.c_int), ("patch_size", C.c_int), ("fast_threshold", C.c_int)]

    HARRIS, FAST = 0, 1

    def __init__(self, nfeatures=150, scale_factor=1.2, nlevels=8, patch_size=31, fast_threshold=20,
                 edge_threshold=None, score_type=0):
        super().__init__()
        self.nfeatures, self.scale_factor, self.nlevels = nfeatures, scale_factor, nlevels
        self.edge_threshold = patch_size if edge_threshold is None else edge_threshold
        self.first_level, self.wta_k, self.score_type = 0, 4, score_type
        self.patch_size, self.fast_threshold = patch_size, fast_threshold


class Context:
    """One HIP device + stream (svo_ctx)."""

    def __init__(self, device: int = 0):
        L = lib()
        h = _vp()
        self.device = device
        rc = L.svo_ctx_create(device, C.byref(h))
        if rc != 0:
            raise SvoError(f"svo_ctx_create(device={device}) failed: {rc} (no usable HIP device?)")
        self.handle = h
        _LIVE["context"].add(self)

    def _check(self, rc):
        if rc < 0:
            raise SvoError(lib().svo_last_error(self.handle).decode() or f"error {rc}")
        return rc

    def close(self):
        if getattr(self, "handle", None):
            lib().svo_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------- images
    def image(self, gray: np.ndarray, max_levels: int = 4) -> Image:
        gray = _c(gray, np.uint8)
        h, w = gray.shape
        hd = _vp()
        self._check(lib().svo_image_create(self.handle, w, h, max_levels, C.byref(hd)))
        img = Image(self, hd, w, h, max_levels)
        img.upload(gray)
        return img

    def image_bgr(self, bgr: np.ndarray, max_levels: int = 4) -> Image:
        """Device image from an (h, w, 3) BGR frame (svo_image_upload_bgr)."""
        bgr = _c(bgr, np.uint8)
        h, w, c = bgr.shape
        assert c == 3
        hd = _vp()
        self._check(lib().svo_image_create(self.handle, w, h, max_levels, C.byref(hd)))
        img = Image(self, hd, w, h, max_levels)
        img.upload_bgr(bgr)
        return img

    # ---------------------------------------------------------------- FAST
    def fast_detect(self, img: Image, threshold: int = 20, nonmax: bool = True, mask=None,
                    cap: int = 1 << 20) -> np.ndarray:
        """cv::FastFeatureDetector::detect -> float32 array (n, 3): x, y, response."""
        out = np.empty((cap, 3), np.float32)
        n = C.c_int()
        mp = None
        if mask is not None:
            mask = _c(mask, np.uint8)
            assert mask.shape == (img.h, img.w)
            mp = _p(mask, _u8p)
        self._check(lib().svo_fast_detect(self.handle, img.handle, int(threshold), int(bool(nonmax)), mp,
                                          _p(out, _f32p), cap, C.byref(n)))
        return out[: min(n.value, cap)].copy()

    def orb_detect(self, img: Image, params: "OrbParams" = None, mask=None, cap: int = 1 << 16):
        """cv::ORB::detect -> (float32 (n, 3) x, y, response; int32 (n,) octave)."""
        params = params or OrbParams()
        out = np.empty((cap, 3), np.float32)
        octv = np.empty(cap, np.int32)
        n = C.c_int()
        mp = None
        if mask is not None:
            mask = _c(mask, np.uint8)
            assert mask.shape == (img.h, img.w)
            mp = _p(mask, _u8p)
        self._check(lib().svo_orb_detect(self.handle, img.handle, C.byref(params), mp, _p(out, _f32p),
                                         _p(octv, _i32p), cap, C.byref(n)))
        k = min(n.value, cap)
        return out[:k].copy(), octv[:k].copy()

    def fast_score_map(self, img: Image, threshold: int = 20):
        score = np.empty((img.h, img.w), np.uint8)
        corner = np.empty((img.h, img.w), np.uint8)
        self._check(lib().svo_fast_score_map(self.handle, img.handle, int(threshold), _p(score, _u8p),
                                             _p(corner, _u8p)))
        return score, corner

    def mask_boxes(self, w: int, h: int, pts, half: float = 10.0) -> np.ndarray:
        pts = _c(pts, np.float32).reshape(-1, 2)
        mask = np.empty((h, w), np.uint8)
        self._check(lib().svo_mask_boxes(self.handle, w, h, _p(pts, _f32p), len(pts), float(half),
                                         _p(mask, _u8p)))
        return mask

    # ---------------------------------------------------------------- bucket
    def bucket_features(self, pts, img_w: int, img_h: int, bucket_size: int, per_bucket: int,
                        ages=None):
        pts = _c(pts, np.float32).reshape(-1, 2)
        n = len(pts)
        cap = (img_h // bucket_size + 1) * (img_w // bucket_size + 1) * per_bucket + 1
        xy_out = np.empty((cap, 2), np.float32)
        ages_out = np.empty(cap, np.int32)
        ap = None
        if ages is not None:
            ages = _c(ages, np.int32)
            ap = _p(ages, _i32p)
        nout = C.c_int()
        self._check(lib().svo_bucket_features(self.handle, _p(pts, _f32p), ap, n, img_w, img_h, bucket_size,
                                              per_bucket, _p(xy_out, _f32p), _p(ages_out, _i32p), cap,
                                              C.byref(nout)))
        k = min(nout.value, cap)
        return xy_out[:k].copy(), ages_out[:k].copy()

    # ---------------------------------------------------------------- LK
    def calc_optical_flow_pyr_lk(self, prev: Image, nxt: Image, prev_pts, next_pts=None,
                                 win_size=(21, 21), max_level: int = 3,
                                 criteria=(TERM_COUNT | TERM_EPS, 30, 0.01), flags: int = 0,
                                 min_eig_threshold: float = 1e-4, want_err: bool = True):
        """cv::calcOpticalFlowPyrLK -> (next_pts (n,2) f32, status (n,) u8, err (n,) f32)."""
        prev_pts = _c(prev_pts, np.float32).reshape(-1, 2)
        n = len(prev_pts)
        if next_pts is None:
            nxt_pts = np.zeros((n, 2), np.float32)
        else:
            nxt_pts = _c(next_pts, np.float32).reshape(-1, 2).copy()
        status = np.zeros(n, np.uint8)
        err = np.zeros(n, np.float32) if want_err else None
        ctype, count, eps = criteria
        self._check(lib().svo_calc_optical_flow_pyr_lk(
            self.handle, prev.handle, nxt.handle, _p(prev_pts, _f32p), n, _p(nxt_pts, _f32p),
            _p(status, _u8p), _p(err, _f32p) if err is not None else None, int(win_size[0]),
            int(win_size[1]), int(max_level), int(ctype), int(count), float(eps), int(flags),
            float(min_eig_threshold)))
        return nxt_pts, status, err

    def lk_last_iterations(self) -> int:
        return int(lib().svo_lk_last_iterations(self.handle))

    # ---------------------------------------------------------------- PnP
    def pnp_residuals(self, obj, img_pts, hyps, K, thresh2: float = 64.0, want_err: bool = True):
        """hyps: (m, 12) = R row-major + t. -> (err (m,n) f32, mask (m,n) u8, counts (m,))."""
        obj = _c(obj, np.float32).reshape(-1, 3)
        img_pts = _c(img_pts, np.float32).reshape(-1, 2)
        hyps = _c(hyps, np.float64).reshape(-1, 12)
        K = _c(K, np.float64).reshape(9)
        n, m = len(obj), len(hyps)
        err = np.empty((m, n), np.float32) if want_err else None
        mask = np.empty((m, n), np.uint8)
        counts = np.empty(m, np.int32)
        self._check(lib().svo_pnp_residuals(self.handle, _p(obj, _f32p), _p(img_pts, _f32p), n,
                                            _p(hyps, _f64p), m, _p(K, _f64p), float(thresh2),
                                            _p(err, _f32p) if err is not None else None,
                                            _p(mask, _u8p), _p(counts, _i32p)))
        return err, mask, counts

    def epnp_subsets(self, subsets, K, device=True):
        """RANSAC's EPnP on (m, 25) float subsets (obj xyz x5, img xy x5) -> (Rt (m, 12), ok (m,)):
        device 0 / False: the host solver the RANSAC uses (bit-identical to the
        oracle's EPnP); 1 / True: the QL variant, one wave per subset on the GPU;
        2: that variant's host twin (bit-identical to 1); 3 / 4 / 5: device 0 forced
        to its scalar / AVX2 / AVX-512 form; 6: device 0's solver on the GPU, one
        lane per subset (bit-identical to 0)."""
        subsets = _c(subsets, np.float32).reshape(-1, 25)
        K = _c(K, np.float64).reshape(9)
        m = len(subsets)
        Rt = np.zeros((m, 12), np.float64)
        ok = np.zeros(m, np.int32)
        self._check(lib().svo_epnp_subsets(self.handle, _p(subsets, _f32p), m, _p(K, _f64p), int(device),
                                           _p(Rt, _f64p), _p(ok, _i32p)))
        return Rt, ok

    def triangulate_points(self, P1, P2, pts1, pts2):
        """cv::triangulatePoints + convertPointsFromHomogeneous -> (xyzw (n,4), xyz (n,3)) float32."""
        P1 = _c(P1, np.float32).reshape(12)
        P2 = _c(P2, np.float32).reshape(12)
        pts1 = _c(pts1, np.float32).reshape(-1, 2)
        pts2 = _c(pts2, np.float32).reshape(-1, 2)
        n = len(pts1)
        if len(pts2) != n:
            raise ValueError("pts1 and pts2 differ in length")
        h = np.empty((n, 4), np.float32)
        x = np.empty((n, 3), np.float32)
        self._check(lib().svo_triangulate_points(self.handle, _p(P1, _f32p), _p(P2, _f32p), _p(pts1, _f32p),
                                                 _p(pts2, _f32p), n, _p(h, _f32p), _p(x, _f32p)))
        return h, x

    def reprojection_jacobians(self, obj, img_pts, poses, K, counts=None, huber_delta: float = 0.0):
        """obj (P, n, 3) f64, img (P, n, 2) f32, poses (P, 12) -> (res (P,n,2), jac (P,n,2,6), normal (P,28))."""
        obj = _c(obj, np.float64)
        if obj.ndim == 2:
            obj = obj[None]
        P, n = obj.shape[0], obj.shape[1]
        img_pts = _c(img_pts, np.float32).reshape(P, n, 2)
        poses = _c(poses, np.float64).reshape(P, 12)
        K = _c(K, np.float64).reshape(9)
        cnt = _c(counts, np.int32).reshape(P) if counts is not None else None
        res = np.empty((P, n, 2), np.float64)
        jac = np.empty((P, n, 2, 6), np.float64)
        ne = np.empty((P, 28), np.float64)
        self._check(lib().svo_reprojection_jacobians(self.handle, _p(obj, _f64p), _p(img_pts, _f32p),
                                                     _p(cnt, _i32p) if cnt is not None else None, P, n,
                                                     _p(poses, _f64p), _p(K, _f64p), float(huber_delta),
                                                     _p(res, _f64p), _p(jac, _f64p), _p(ne, _f64p)))
        return res, jac, ne

    def refine_poses(self, obj, img_pts, poses, K, counts=None, huber_delta: float = 0.0, max_iterations: int = 20):
        """Motion-only LM over SE(3) -> (poses (P,12), costs (P,), iterations)."""
        obj = _c(obj, np.float64)
        if obj.ndim == 2:
            obj = obj[None]
        P, n = obj.shape[0], obj.shape[1]
        img_pts = _c(img_pts, np.float32).reshape(P, n, 2)
        poses = np.array(poses, np.float64).reshape(P, 12)
        K = _c(K, np.float64).reshape(9)
        cnt = _c(counts, np.int32).reshape(P) if counts is not None else None
        costs = np.empty(P, np.float64)
        it = C.c_int()
        self._check(lib().svo_refine_poses(self.handle, _p(obj, _f64p), _p(img_pts, _f32p),
                                           _p(cnt, _i32p) if cnt is not None else None, P, n, _p(K, _f64p),
                                           float(huber_delta), int(max_iterations), _p(poses, _f64p),
                                           _p(costs, _f64p), C.byref(it)))
        return poses, costs, it.value

    def solve_pnp_ransac(self, obj, img_pts, K, iterations: int = 100, reproj_err: float = 8.0,
                         confidence: float = 0.999):
        """cv::solvePnPRansac(..., SOLVEPNP_SQPNP) -> (ok, rvec, tvec, inliers)."""
        obj = _c(obj, np.float64).reshape(-1, 3)
        img_pts = _c(img_pts, np.float32).reshape(-1, 2)
        K = _c(K, np.float64).reshape(9)
        n = len(obj)
        rvec = np.zeros(3, np.float64)
        tvec = np.zeros(3, np.float64)
        inl = np.zeros(max(n, 1), np.int32)
        ninl = C.c_int()
        rc = self._check(lib().svo_solve_pnp_ransac(self.handle, _p(obj, _f64p), _p(img_pts, _f32p), n,
                                                    _p(K, _f64p), int(iterations), float(reproj_err),
                                                    float(confidence), _p(rvec, _f64p), _p(tvec, _f64p),
                                                    _p(inl, _i32p), C.byref(ninl)))
        return rc == 1, rvec, tvec, inl[: ninl.value].copy()


KF_EVERY, KF_REFERENCE = 0, 1  # SVO_KF_EVERY / SVO_KF_REFERENCE


class FrontendConfig(C.Structure):
    """svo_frontend_config (include/svo_gpu.h); defaults = the reference's
    temporal-tracking call (R:src/tracking.cpp:157-165), FAST params
    (R:configs/config.yaml:29-32), solvePnPRansac args (:191-196) and
    features_to_track (R:configs/config.yaml:15). keyframe_rule: KF_EVERY (every
    frame a keyframe topping the set up to n_features; the benchmark) or
    KF_REFERENCE (Tracking::nextFrame's rule, R:src/tracking.cpp:68-69).
    use_orb=1 + orb=OrbParams(...): the keyframe detector is ORB (the shipped
    config, R:configs/config.yaml:19-27) instead of FAST."""
    _fields_ = [
        ("width", C.c_int), ("height", C.c_int), ("n_seq", C.c_int), ("n_frames", C.c_int),
        ("n_features", C.c_int), ("max_level", C.c_int), ("win", C.c_int), ("lk_max_count", C.c_int),
        ("lk_epsilon", C.c_double), ("min_eig", C.c_double), ("lk_flags", C.c_int),
        ("fast_threshold", C.c_int), ("fast_nonmax", C.c_int), ("mask_half", C.c_float),
        ("bucket_size", C.c_int), ("per_bucket", C.c_int), ("pnp_iterations", C.c_int),
        ("pnp_reproj", C.c_float), ("pnp_confidence", C.c_double), ("K", C.c_double * 9),
        ("host_threads", C.c_int), ("timing", C.c_int), ("keyframe_rule", C.c_int), ("features_to_track", C.c_int),
        ("P_left", C.c_float * 12), ("P_right", C.c_float * 12), ("y_threshold", C.c_float),
        ("stereo_win", C.c_int), ("stereo_max_level", C.c_int), ("stereo_max_count", C.c_int),
        ("stereo_epsilon", C.c_double), ("use_orb", C.c_int), ("orb", OrbParams),
    ]

    def __init__(self, width, height, K, n_seq=1, n_frames=2, n_features=2000, P_left=None, P_right=None, **kw):
        """P_left / P_right: the stereo rig's 3x4 projection matrices (KITTI calib P2 /
        P3, R:src/main.cpp:25-32); default K[I|0] and K[I|(-bf, 0, 0)] with the
        synthetic scene's fx * baseline (svo_amd.scene.STEREO_BF)."""
        super().__init__()
        d = dict(max_level=3, win=21, lk_max_count=50, lk_epsilon=1e-3, min_eig=1e-4,
                 lk_flags=LK_GET_MIN_EIGENVALS, fast_threshold=20, fast_nonmax=1, mask_half=10.0,
                 bucket_size=0, per_bucket=0, pnp_iterations=100, pnp_reproj=8.0, pnp_confidence=0.999,
                 host_threads=0, timing=0, keyframe_rule=KF_EVERY, features_to_track=70, y_threshold=40.0,
                 stereo_win=11, stereo_max_level=3,
                 stereo_max_count=30, stereo_epsilon=1e-3, use_orb=0)
        orb = kw.pop("orb", None)
        d.update(kw)
        self.width, self.height, self.n_seq, self.n_frames, self.n_features = width, height, n_seq, n_frames, n_features
        for k, v in d.items():
            setattr(self, k, v)
        self.orb = orb if orb is not None else OrbParams()
        self.K[:] = [float(x) for x in np.asarray(K, np.float64).ravel()]
        if P_left is None or P_right is None:
            from .scene import stereo_projections
            P_left, P_right = stereo_projections(K)
        self.P_left[:] = [float(x) for x in np.asarray(P_left, np.float32).ravel()]
        self.P_right[:] = [float(x) for x in np.asarray(P_right, np.float32).ravel()]


class FrontendStats(C.Structure):
    _fields_ = [("lk_iterations", C.c_int64), ("tracked", C.c_int64), ("inliers", C.c_int64),
                ("added", C.c_int64), ("features", C.c_int64), ("hypotheses", C.c_int64),
                ("host_ms_hyp", C.c_double), ("host_ms_fit", C.c_double), ("host_ms_wait", C.c_double),
                ("keyframes", C.c_int64),
                ("host_ms_wait_post", C.c_double), ("host_ms_wait_score", C.c_double),
                ("host_ms_wait_kf", C.c_double), ("host_ms_enqueue", C.c_double), ("host_ms_step", C.c_double),
                ("ransac_rounds", C.c_int64), ("max_hypotheses", C.c_int64), ("serial_keyframe", C.c_int64),
                ("full_copy", C.c_int64), ("kf_overflow", C.c_int64), ("host_ms_orb", C.c_double),
                ("spec_margin", C.c_int64)]

    def as_dict(self):
        return {k: (float(getattr(self, k)) if k.startswith("host_") else int(getattr(self, k)))
                for k, _ in self._fields_}


PHASES = ["pyramid", "lk", "post_lk", "stereo_lk", "pnp_score", "tail", "fast", "bucket", "append", "pyramid_right"]


class Frontend:
    """Batched tracking loop of Tracking::startStereo (R:src/tracking.cpp:232-276) over
    n_seq independent sequences (svo_frontend_*)."""

    def __init__(self, ctx: Context, cfg: FrontendConfig):
        self.ctx, self.cfg = ctx, cfg
        h = _vp()
        ctx._check(lib().svo_frontend_create(ctx.handle, C.byref(cfg), C.byref(h)))
        self.handle = h
        self._queued = {}  # ring slot -> (t, lefts, rights) of queue_frames, until upload_wait(t)
        _LIVE["frontend"].add(self)

    def set_frame(self, seq, t, left, right):
        """Stereo pair t of sequence seq: (h, w) grey, or (h, w, 3) BGR converted on the device."""
        left = _c(left, np.uint8)
        right = _c(right, np.uint8)
        if left.shape != right.shape:
            raise SvoError("set_frame: left / right shapes differ")
        if left.ndim == 3:
            self.ctx._check(lib().svo_frontend_set_frame_bgr(self.handle, seq, t, _p(left, _u8p), _p(right, _u8p),
                                                             3 * left.shape[1]))
            return
        self.ctx._check(lib().svo_frontend_set_frame(self.handle, seq, t, _p(left, _u8p), _p(right, _u8p),
                                                     left.shape[1]))

    def prebuild_pyramids(self):
        self.ctx._check(lib().svo_frontend_prebuild_pyramids(self.handle))

    def queue_frames(self, t, lefts, rights):
        """svo_frontend_queue_frames: frame t of every sequence from host arrays
        (lefts[s], rights[s]: (height, width) grey or (height, width, 3) BGR of the
        config's size, all of one shape), queued as asynchronous H2D copies (see
        include/svo_gpu.h for the ring discipline). The copies read the arrays after
        this call returns: the wrapper keeps them referenced until upload_wait(t) (or
        until ring slot t % n_frames is queued again); their contents must stay
        unchanged until then."""
        S = self.cfg.n_seq
        if len(lefts) != S or len(rights) != S:
            raise SvoError("queue_frames: one left and one right image per sequence")
        a0 = lefts[0]
        hw = (self.cfg.height, self.cfg.width)
        if a0.shape not in (hw, hw + (3,)):
            raise SvoError(f"queue_frames: images must be {hw} grey or {hw + (3,)} BGR, got {a0.shape}")
        bgr = a0.ndim == 3
        for a in list(lefts) + list(rights):
            if a.shape != a0.shape or a.dtype != np.uint8 or not a.flags["C_CONTIGUOUS"]:
                raise SvoError("queue_frames: C-contiguous uint8 images of one shape")
        L = (_u8p * S)(*[a.ctypes.data_as(_u8p) for a in lefts])
        R = (_u8p * S)(*[a.ctypes.data_as(_u8p) for a in rights])
        stride = a0.shape[1] * (3 if bgr else 1)
        self.ctx._check(lib().svo_frontend_queue_frames(self.handle, int(t), L, R, stride, int(bgr)))
        # the asynchronous copies read these buffers: hold them until upload_wait(t)
        self._queued[int(t) % max(self.cfg.n_frames, 1)] = (int(t), list(lefts), list(rights))

    def upload_wait(self, t):
        self.ctx._check(lib().svo_frontend_upload_wait(self.handle, int(t)))
        slot = int(t) % max(self.cfg.n_frames, 1)
        held = self._queued.get(slot)
        if held is not None and held[0] == int(t):
            del self._queued[slot]

    def init(self, t0=0):
        self.ctx._check(lib().svo_frontend_init(self.handle, t0))

    def step(self, t) -> FrontendStats:
        st = FrontendStats()
        self.ctx._check(lib().svo_frontend_step(self.handle, t, C.byref(st)))
        return st

    def synchronize(self):
        """Wait for all of the front end's streams and finish the pose fits."""
        self.ctx._check(lib().svo_frontend_synchronize(self.handle))

    def pose(self, seq):
        r = np.zeros(3)
        t = np.zeros(3)
        self.ctx._check(lib().svo_frontend_pose(self.handle, seq, _p(r, _f64p), _p(t, _f64p)))
        return r, t

    def features(self, seq, cap=1 << 16):
        xy = np.empty((cap, 2), np.float32)
        n = C.c_int()
        self.ctx._check(lib().svo_frontend_features(self.handle, seq, _p(xy, _f32p), cap, C.byref(n)))
        return xy[: min(n.value, cap)].copy()

    def map_points(self, seq, cap=1 << 16):
        """World positions of the current features' map points (float64, (n, 3))."""
        xyz = np.empty((cap, 3), np.float64)
        n = C.c_int()
        self.ctx._check(lib().svo_frontend_map_points(self.handle, seq, _p(xyz, _f64p), cap, C.byref(n)))
        return xyz[: min(n.value, cap)].copy()

    def time_pyramid(self, t, reps=20):
        """ms per pyramid + Scharr launch chain of frame t, timed alone."""
        ms = np.zeros(1)
        self.ctx._check(lib().svo_frontend_time_pyramid(self.handle, int(t), int(reps), _p(ms, _f64p)))
        return float(ms[0])

    def time_fast(self, t, reps=20):
        """ms per FAST detection launch (unmasked, every sequence) of frame t, timed alone."""
        ms = np.zeros(1)
        self.ctx._check(lib().svo_frontend_time_fast(self.handle, int(t), int(reps), _p(ms, _f64p)))
        return float(ms[0])

    def phase_times(self):
        ms = np.zeros(16)
        n = np.zeros(16, np.int64)
        k = lib().svo_frontend_phase_times(self.handle, _p(ms, _f64p), n.ctypes.data_as(C.POINTER(C.c_int64)), 16)
        return {PHASES[i]: (float(ms[i]), int(n[i])) for i in range(k)}

    def reset_times(self):
        lib().svo_frontend_reset_times(self.handle)

    def scharr(self, seq, t, level, w, h):
        """(ix, iy) of frame t's level (w x h) as the fused pyrDown + Scharr pass built
        them (svo_frontend_scharr_level)."""
        ix = np.empty((h, w), np.int16)
        iy = np.empty_like(ix)
        self.ctx._check(lib().svo_frontend_scharr_level(self.handle, int(seq), int(t), int(level),
                                                        ix.ctypes.data_as(C.POINTER(C.c_int16)),
                                                        iy.ctypes.data_as(C.POINTER(C.c_int16)), w))
        return ix, iy

    def pyramid_level(self, seq, t, level, w, h, right=False):
        """Level `level` (w x h) of frame t's left / right pyramid with its stored
        REFLECT_101 border of PYR_PAD pixels (svo_frontend_pyramid_level)."""
        out = np.empty((h + 2 * PYR_PAD, w + 2 * PYR_PAD), np.uint8)
        self.ctx._check(lib().svo_frontend_pyramid_level(self.handle, int(seq), int(t), int(bool(right)), int(level),
                                                         out.ctypes.data_as(C.POINTER(C.c_uint8)), out.shape[1]))
        return out

    def host_cpus(self):
        """CPUs the host pool is pinned to (svo_host_cpu_plan's share of this rank)."""
        cpus = np.zeros(4096, np.int32)
        n = C.c_int(0)
        self.ctx._check(lib().svo_frontend_host_cpus(self.handle, _p(cpus, _i32p), 4096, C.byref(n)))
        return cpus[:n.value].tolist()

    def streams(self):
        """The HIP stream handles (LK, FAST, copies) this front end runs on."""
        arr = (_vp * 3)()
        n = C.c_int(0)
        self.ctx._check(lib().svo_frontend_streams(self.handle, arr, 3, C.byref(n)))
        return [arr[i] for i in range(n.value)]

    def close(self):
        if getattr(self, "handle", None):
            lib().svo_frontend_destroy(self.handle)  # waits for the front end's streams
            self.handle = None
            self._queued = {}

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class FastFeatureDetector:
    """cv::FastFeatureDetector::create(threshold, nonmaxSuppression) (TYPE_9_16),
    as the reference creates it at R:src/tracking.cpp:54-57."""

    def __init__(self, ctx: Context, threshold: int = 20, nonmax_suppression: bool = True):
        self.ctx, self.threshold, self.nonmax = ctx, threshold, nonmax_suppression

    @classmethod
    def create(cls, ctx: Context, threshold: int = 20, nonmax_suppression: bool = True):
        return cls(ctx, threshold, nonmax_suppression)

    def detect(self, img: Image, mask=None) -> np.ndarray:
        return self.ctx.fast_detect(img, self.threshold, self.nonmax, mask)


