"""ctypes binding of the CPU oracle (oracle/build/libsvo_oracle.so).

TEST INFRASTRUCTURE ONLY: the oracle is the checker the HIP path is compared
against (see oracle/svo_oracle.h for what it restates and its pinning status).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PATH = os.path.join(ROOT, "oracle", "build", "libsvo_oracle.so")

ACC_EXACT, ACC_SCALAR, ACC_SSE = 0, 1, 2
LEVEL_ITERS = 0x100  # oracle/svo_oracle.h SVO_ORACLE_LEVEL_ITERS
TERM_COUNT, TERM_EPS = 1, 2
LK_USE_INITIAL_FLOW, LK_GET_MIN_EIGENVALS = 4, 8

_u8p = C.POINTER(C.c_uint8)
_f32p = C.POINTER(C.c_float)
_f64p = C.POINTER(C.c_double)
_i32p = C.POINTER(C.c_int)
_u64p = C.POINTER(C.c_uint64)
_L = None


def load():
    global _L
    if _L is None:
        if not os.path.exists(PATH):
            subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle")])
        L = C.CDLL(PATH)
        sig = {
            "svo_oracle_pyr_down": (None, [_u8p, C.c_int, C.c_int, C.c_int, _u8p, C.c_int]),
            "svo_oracle_pyramid_levels": (C.c_int, [C.c_int] * 5 + [_i32p, _i32p]),
            "svo_oracle_build_pyramid": (C.c_int, [_u8p] + [C.c_int] * 6 + [_u8p]),
            "svo_oracle_scharr": (None, [_u8p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int16)]),
            "svo_oracle_lk": (C.c_int, [_u8p, _u8p, C.c_int, C.c_int, C.c_int, _f32p, _f32p, _u8p, _f32p,
                                        C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double,
                                        C.c_int, C.c_double, C.c_int, _i32p]),
            "svo_oracle_fast": (C.c_int, [_u8p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _u8p, _f32p,
                                          C.c_int]),
            "svo_oracle_fast_score": (None, [_u8p, C.c_int, C.c_int, C.c_int, C.c_int, _u8p, _u8p]),
            "svo_oracle_mask_boxes": (None, [C.c_int, C.c_int, _f32p, C.c_int, C.c_float, _u8p]),
            "svo_oracle_bucket": (C.c_int, [_f32p, _i32p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                            _f32p, _i32p, C.c_int, _i32p]),
            "svo_oracle_rng_next": (C.c_uint32, [_u64p]),
            "svo_oracle_rodrigues": (None, [_f64p, _f64p]),
            "svo_oracle_rodrigues_inv": (None, [_f64p, _f64p]),
            "svo_oracle_pnp_residuals": (None, [_f32p, _f32p, C.c_int, _f64p, C.c_int, _f64p, C.c_float,
                                                _f32p, _u8p, _i32p]),
            "svo_oracle_epnp": (C.c_int, [_f32p, _f32p, C.c_int, _f64p, _f64p, _f64p]),
            "svo_oracle_ransac_update_num_iters": (C.c_int, [C.c_double, C.c_double, C.c_int, C.c_int]),
            "svo_oracle_solve_pnp_ransac": (C.c_int, [_f64p, _f32p, C.c_int, _f64p, C.c_int, C.c_float,
                                                      C.c_double, _f64p, _f64p, _u8p, _i32p, _i32p]),
            "svo_oracle_get_subset": (C.c_int, [_u64p, C.c_int, C.c_int, _i32p]),
            "svo_oracle_sqpnp": (C.c_int, [_f64p, _f64p, C.c_int, _f64p, _f64p]),
            "svo_oracle_triangulate": (None, [_f32p, _f32p, _f32p, _f32p, C.c_int, _f32p, _f32p]),
            "svo_oracle_set_threads": (None, [C.c_int]),
            "svo_oracle_bgr2gray": (None, [_u8p, C.c_int, C.c_int, C.c_int, _u8p]),
            "svo_oracle_resize_linear_exact": (None, [_u8p, C.c_int, C.c_int, C.c_int, _u8p, C.c_int, C.c_int,
                                                       C.c_int]),
            "svo_oracle_orb_level_info": (None, [C.c_int, C.c_int, C.c_float, C.c_int, C.c_int, _i32p, _i32p,
                                                  _f32p, _i32p]),
            "svo_oracle_orb_detect": (C.c_int, [_u8p, C.c_int, C.c_int, C.c_int, _u8p, C.c_int, C.c_float, C.c_int,
                                                C.c_int, C.c_int, C.c_int, C.c_int, _f32p, _i32p, C.c_int]),
        }
        for k, (r, a) in sig.items():
            f = getattr(L, k)
            f.restype, f.argtypes = r, a
        _L = L
    return _L


def _p(a, t):
    return a.ctypes.data_as(t)


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def pyr_levels(w, h, win, max_level):
    lw = np.zeros(32, np.int32)
    lh = np.zeros(32, np.int32)
    ml = load().svo_oracle_pyramid_levels(w, h, win[0], win[1], max_level, _p(lw, _i32p), _p(lh, _i32p))
    return ml, [(int(lw[i]), int(lh[i])) for i in range(ml + 1)]


def pyr_down(img):
    img = _c(img, np.uint8)
    h, w = img.shape
    out = np.empty(((h + 1) // 2, (w + 1) // 2), np.uint8)
    load().svo_oracle_pyr_down(_p(img, _u8p), w, h, w, _p(out, _u8p), out.shape[1])
    return out


def build_pyramid(img, win=(21, 21), max_level=3):
    img = _c(img, np.uint8)
    h, w = img.shape
    ml, sizes = pyr_levels(w, h, win, max_level)
    total = sum(a * b for a, b in sizes)
    buf = np.empty(total, np.uint8)
    load().svo_oracle_build_pyramid(_p(img, _u8p), w, h, w, win[0], win[1], max_level, _p(buf, _u8p))
    out, off = [], 0
    for (a, b) in sizes:
        out.append(buf[off: off + a * b].reshape(b, a).copy())
        off += a * b
    return out


def scharr(img):
    img = _c(img, np.uint8)
    h, w = img.shape
    out = np.empty((h, w, 2), np.int16)
    load().svo_oracle_scharr(_p(img, _u8p), w, h, w, out.ctypes.data_as(C.POINTER(C.c_int16)))
    return out


def lk(prev, nxt, prev_pts, win=(21, 21), max_level=3, criteria=(3, 30, 0.01), flags=0, min_eig=1e-4,
       acc=ACC_EXACT, next_pts=None, want_err=True, level_iters=False):
    """cv::calcOpticalFlowPyrLK (oracle/lk.c). level_iters: iters is (max_level + 1, n), one row
    per pyramid level (GN iterations of each point at that level), instead of the per-point sum."""
    prev = _c(prev, np.uint8)
    nxt = _c(nxt, np.uint8)
    h, w = prev.shape
    pp = _c(prev_pts, np.float32).reshape(-1, 2)
    n = len(pp)
    npts = np.zeros((n, 2), np.float32) if next_pts is None else _c(next_pts, np.float32).reshape(-1, 2).copy()
    st = np.zeros(n, np.uint8)
    err = np.zeros(n, np.float32)
    iters = np.zeros((max_level + 1, n) if level_iters else n, np.int32)
    load().svo_oracle_lk(_p(prev, _u8p), _p(nxt, _u8p), w, h, w, _p(pp, _f32p), _p(npts, _f32p), _p(st, _u8p),
                         _p(err, _f32p) if want_err else None, n, win[0], win[1], max_level, criteria[0],
                         criteria[1], criteria[2], flags, min_eig, acc | (LEVEL_ITERS if level_iters else 0),
                         _p(iters, _i32p))
    return npts, st, err, iters


def fast(img, threshold=20, nonmax=True, mask=None, cap=1 << 20):
    img = _c(img, np.uint8)
    h, w = img.shape
    out = np.empty((cap, 3), np.float32)
    mp = _p(_c(mask, np.uint8), _u8p) if mask is not None else None
    n = load().svo_oracle_fast(_p(img, _u8p), w, h, w, threshold, int(bool(nonmax)), mp, _p(out, _f32p), cap)
    return out[: min(n, cap)].copy()


def fast_score(img, threshold=20):
    img = _c(img, np.uint8)
    h, w = img.shape
    s = np.empty((h, w), np.uint8)
    c = np.empty((h, w), np.uint8)
    load().svo_oracle_fast_score(_p(img, _u8p), w, h, w, threshold, _p(s, _u8p), _p(c, _u8p))
    return s, c


def mask_boxes(w, h, pts, half=10.0):
    pts = _c(pts, np.float32).reshape(-1, 2)
    m = np.empty((h, w), np.uint8)
    load().svo_oracle_mask_boxes(w, h, _p(pts, _f32p), len(pts), half, _p(m, _u8p))
    return m


def bucket(pts, img_w, img_h, bucket_size, per_bucket, ages=None):
    pts = _c(pts, np.float32).reshape(-1, 2)
    n = len(pts)
    cap = (img_h // bucket_size + 1) * (img_w // bucket_size + 1) * per_bucket + 1
    xo = np.empty((cap, 2), np.float32)
    ao = np.empty(cap, np.int32)
    tot = C.c_int()
    ap = _p(_c(ages, np.int32), _i32p) if ages is not None else None
    k = load().svo_oracle_bucket(_p(pts, _f32p), ap, n, img_w, img_h, bucket_size, per_bucket, _p(xo, _f32p),
                                 _p(ao, _i32p), cap, C.byref(tot))
    return xo[:k].copy(), ao[:k].copy()


def rodrigues(rv):
    rv = _c(rv, np.float64)
    R = np.empty(9, np.float64)
    load().svo_oracle_rodrigues(_p(rv, _f64p), _p(R, _f64p))
    return R.reshape(3, 3)


def rodrigues_inv(R):
    R = _c(R, np.float64).reshape(9)
    rv = np.empty(3, np.float64)
    load().svo_oracle_rodrigues_inv(_p(R, _f64p), _p(rv, _f64p))
    return rv


def pnp_residuals(obj, img, hyps, K, thresh2=64.0):
    obj = _c(obj, np.float32).reshape(-1, 3)
    img = _c(img, np.float32).reshape(-1, 2)
    hyps = _c(hyps, np.float64).reshape(-1, 12)
    K = _c(K, np.float64).reshape(9)
    n, m = len(obj), len(hyps)
    err = np.empty((m, n), np.float32)
    mask = np.empty((m, n), np.uint8)
    cnt = np.empty(m, np.int32)
    load().svo_oracle_pnp_residuals(_p(obj, _f32p), _p(img, _f32p), n, _p(hyps, _f64p), m, _p(K, _f64p),
                                    thresh2, _p(err, _f32p), _p(mask, _u8p), _p(cnt, _i32p))
    return err, mask, cnt


def epnp(obj, img, K):
    obj = _c(obj, np.float32).reshape(-1, 3)
    img = _c(img, np.float32).reshape(-1, 2)
    K = _c(K, np.float64).reshape(9)
    R = np.empty(9, np.float64)
    t = np.empty(3, np.float64)
    rc = load().svo_oracle_epnp(_p(obj, _f32p), _p(img, _f32p), len(obj), _p(K, _f64p), _p(R, _f64p), _p(t, _f64p))
    return rc, R.reshape(3, 3), t


def solve_pnp_ransac(obj, img, K, iterations=100, reproj=8.0, confidence=0.999):
    obj = _c(obj, np.float64).reshape(-1, 3)
    img = _c(img, np.float32).reshape(-1, 2)
    K = _c(K, np.float64).reshape(9)
    n = len(obj)
    rv = np.zeros(3)
    tv = np.zeros(3)
    mask = np.zeros(max(n, 1), np.uint8)
    ni = C.c_int()
    nh = C.c_int()
    rc = load().svo_oracle_solve_pnp_ransac(_p(obj, _f64p), _p(img, _f32p), n, _p(K, _f64p), iterations, reproj,
                                            confidence, _p(rv, _f64p), _p(tv, _f64p), _p(mask, _u8p),
                                            C.byref(ni), C.byref(nh))
    return rc, rv, tv, np.nonzero(mask[:n])[0].astype(np.int32), nh.value


def ransac_subsets(n, count):
    """The first `count` 5-point subsets solvePnPRansac draws for n points
    (RANSACPointSetRegistrator::getSubset with RNG(-1), ptsetreg.cpp)."""
    st = C.c_uint64(0xFFFFFFFFFFFFFFFF)
    out = np.empty((count, 5), np.int32)
    for k in range(count):
        load().svo_oracle_get_subset(C.byref(st), n, 5, _p(out[k], _i32p))
    return out


def sqpnp(pw, q):
    """calib3d/src/sqpnp.cpp PoseSolver on object points pw (n, 3) and normalised
    image points q (n, 2): (rc, R, t), rc 0 on success."""
    pw = _c(pw, np.float64).reshape(-1, 3)
    q = _c(q, np.float64).reshape(-1, 2)
    R = np.zeros(9)
    t = np.zeros(3)
    rc = load().svo_oracle_sqpnp(_p(pw, _f64p), _p(q, _f64p), len(pw), _p(R, _f64p), _p(t, _f64p))
    return rc, R.reshape(3, 3), t


def update_num_iters(p, ep, model_points, max_iters):
    return load().svo_oracle_ransac_update_num_iters(p, ep, model_points, max_iters)


def bgr2gray(bgr):
    bgr = _c(bgr, np.uint8)
    h, w, _ = bgr.shape
    out = np.empty((h, w), np.uint8)
    load().svo_oracle_bgr2gray(_p(bgr, _u8p), w, h, 3 * w, _p(out, _u8p))
    return out


def resize_linear_exact(img, dw, dh):
    img = _c(img, np.uint8)
    h, w = img.shape
    out = np.empty((dh, dw), np.uint8)
    load().svo_oracle_resize_linear_exact(_p(img, _u8p), w, h, w, _p(out, _u8p), dw, dh, dw)
    return out


def orb_level_info(w, h, scale_factor=1.2, nlevels=8, nfeatures=150):
    lw, lh, nper = (np.zeros(nlevels, np.int32) for _ in range(3))
    ls = np.zeros(nlevels, np.float32)
    load().svo_oracle_orb_level_info(w, h, scale_factor, nlevels, nfeatures, _p(lw, _i32p), _p(lh, _i32p),
                                     _p(ls, _f32p), _p(nper, _i32p))
    return lw, lh, ls, nper


def orb_detect(img, mask=None, nfeatures=150, scale_factor=1.2, nlevels=8, edge_threshold=31, patch_size=31,
               fast_threshold=20, harris=True, cap=1 << 16):
    img = _c(img, np.uint8)
    h, w = img.shape
    out = np.empty((cap, 3), np.float32)
    octv = np.empty(cap, np.int32)
    mp = None
    if mask is not None:
        mask = _c(mask, np.uint8)
        mp = _p(mask, _u8p)
    n = load().svo_oracle_orb_detect(_p(img, _u8p), w, h, w, mp, nfeatures, scale_factor, nlevels, edge_threshold,
                                     patch_size, fast_threshold, int(bool(harris)), _p(out, _f32p),
                                     _p(octv, _i32p), cap)
    k = min(n, cap)
    return out[:k].copy(), octv[:k].copy()


def set_threads(n: int):
    """Threads of the oracle's LK point loop (OpenMP)."""
    load().svo_oracle_set_threads(int(n))


def triangulate(P1, P2, pts1, pts2):
    """cv::triangulatePoints + convertPointsFromHomogeneous -> (xyzw (n,4), xyz (n,3)) float32."""
    P1 = _c(P1, np.float32).reshape(12)
    P2 = _c(P2, np.float32).reshape(12)
    pts1 = _c(pts1, np.float32).reshape(-1, 2)
    pts2 = _c(pts2, np.float32).reshape(-1, 2)
    n = len(pts1)
    h = np.empty((n, 4), np.float32)
    x = np.empty((n, 3), np.float32)
    load().svo_oracle_triangulate(_p(P1, _f32p), _p(P2, _f32p), _p(pts1, _f32p), _p(pts2, _f32p), n,
                                  _p(h, _f32p), _p(x, _f32p))
    return h, x


def rng_sequence(n, state=0xFFFFFFFFFFFFFFFF):
    s = C.c_uint64(state)
    return [load().svo_oracle_rng_next(C.byref(s)) for _ in range(n)]
