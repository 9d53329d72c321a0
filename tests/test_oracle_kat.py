"""Known-answer tests pinning the CPU oracle, CPU only.

The reference has no tests and OpenCV is absent ("parity unpinned" against
OpenCV itself), so the oracle is pinned by answers derivable by hand:
pyrDown of constant / ramp images, hand-built FAST rings and their scores,
NMS tie rules, LK on exact translations, RANSAC on exact correspondences plus
far outliers, RANSACUpdateNumIters values, cv::RNG's MWC recurrence, and the
reference's own bucket.cpp quirks on hand-listed points. Plus a drift check
against the committed golden fixtures (tests/golden/make_golden.py).
"""
import math
import os

import numpy as np
import pytest

import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))


# ------------------------------------------------------------------ pyrDown
def test_pyrdown_constant():
    for v in (0, 1, 77, 255):
        img = np.full((37, 53), v, np.uint8)
        d = O.pyr_down(img)
        assert d.shape == (19, 27) and (d == v).all()


def test_pyrdown_ramp_interior_and_reflect101_border():
    img = np.tile(np.arange(64, dtype=np.uint8), (10, 1))  # I(x, y) = x
    d = O.pyr_down(img)
    # interior: symmetric kernel summing to 256 -> exactly 2x
    assert (d[:, 1:31] == 2 * np.arange(1, 31)).all()
    # x = 0 with REFLECT_101: row taps (2,1,0,1,2)*(1,4,6,4,1) = 12, *16 rows = 192, (192+128)>>8 = 1
    assert (d[:, 0] == 1).all()
    # last output x = 31 samples 60..64 -> 64 reflects to 62: 60+4*61+6*62+4*63+62 = 990*16/256 -> 62
    assert (d[:, 31] == (990 * 16 + 128) >> 8).all()


def test_pyrdown_size_and_levels():
    assert O.pyr_down(np.zeros((5, 7), np.uint8)).shape == (3, 4)
    ml, sizes = O.pyr_levels(1241, 376, (21, 21), 3)
    assert ml == 3 and sizes == [(1241, 376), (621, 188), (311, 94), (156, 47)]
    # buildOpticalFlowPyramid stops when the next size would be <= the window
    ml, sizes = O.pyr_levels(64, 48, (21, 21), 5)
    assert ml == 1 and sizes == [(64, 48), (32, 24)]


def test_scharr_known_answer():
    img = np.tile(np.arange(16, dtype=np.uint8) * 3, (8, 1))  # I = 3x: Ix = 32*3*2 = 96... check formula
    d = O.scharr(img)
    # t0 = 3(r0+r2)+10r1 = 16*I ; Ix = t0[x+1]-t0[x-1] = 16*3*2 = 96 ; Iy = 0
    assert (d[:, 1:15, 0] == 96).all() and (d[:, :, 1] == 0).all()
    # x = 0 reflects to x = 1: t0[1] - t0[1] = 0
    assert (d[:, 0, 0] == 0).all()


# ------------------------------------------------------------------ FAST
RING = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3),
        (0, -3), (-1, -3), (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def ring_patch(center, ring_vals, size=15):
    img = np.full((size, size), center, np.uint8)
    c = size // 2
    for (dx, dy), v in zip(RING, ring_vals):
        img[c + dy, c + dx] = v
    return img, c


@pytest.mark.parametrize("start", [0, 5, 11, 15])
def test_fast_nine_contiguous_is_corner_eight_is_not(start):
    for run, expect in ((9, True), (8, False), (12, True)):
        vals = [100] * 16
        for k in range(run):
            vals[(start + k) % 16] = 130          # brighter by 30 > t = 20
        img, c = ring_patch(100, vals)
        s, corner = O.fast_score(img, 20)
        assert bool(corner[c, c]) == expect, (run, start)
        if expect:
            # score = max threshold keeping the corner: 130 > 100 + t  <=>  t <= 29
            assert s[c, c] == 29
            kps = O.fast(img, 20, True)
            assert [tuple(k) for k in kps] == [(c, c, 29.0)]


def test_fast_dark_corner_and_threshold_is_strict():
    vals = [100] * 16
    for k in range(9):
        vals[k] = 80                                # darker by exactly 20
    img, c = ring_patch(100, vals)
    assert not O.fast_score(img, 20)[1][c, c]      # x < v - t is strict
    assert O.fast_score(img, 19)[1][c, c]
    assert O.fast_score(img, 19)[0][c, c] == 19    # 80 < 100 - t  <=>  t <= 19


def test_fast_nms_equal_scores_suppress_each_other():
    # two identical corners side by side: strict '>' removes both
    img = np.full((20, 20), 100, np.uint8)
    img[8:12, 8:10] = 200                          # a 2-wide bright bar end
    raw = O.fast(img, 20, False)
    nms = O.fast(img, 20, True)
    s, c = O.fast_score(img, 20)
    for x, y, r in nms:
        x, y = int(x), int(y)
        nb = s[y - 1:y + 2, x - 1:x + 2].copy()
        nb[1, 1] = 0
        assert s[y, x] > nb.max()
    assert len(nms) <= len(raw)
    assert (raw[:, 2] == 0).all()                  # no NMS -> response 0


def test_fast_mask_applied_after_nms():
    img, c = ring_patch(100, [130] * 9 + [100] * 7, size=21)
    mask = np.full(img.shape, 255, np.uint8)
    assert len(O.fast(img, 20, True, mask)) == 1
    mask[c, c] = 0
    assert len(O.fast(img, 20, True, mask)) == 0


def test_mask_boxes_rounding_and_clip():
    m = O.mask_boxes(40, 30, np.array([[10.5, 10.5]], np.float32), 10.0)
    # cvRound(0.5) = 0, cvRound(20.5) = 20 (half to even): inclusive 21 x 21 box
    assert (m[0:21, 0:21] == 0).all() and m[21, 0] == 255 and m[0, 21] == 255
    m = O.mask_boxes(40, 30, np.array([[11.5, 11.5]], np.float32), 10.0)
    assert (m[2:23, 2:23] == 0).all() and m[1, 1] == 255 and m[23, 23] == 255


# ------------------------------------------------------------------ LK
def smooth_image(w, h, shift=(0.0, 0.0)):
    y, x = np.mgrid[0:h, 0:w].astype(np.float64)
    x = x - shift[0]
    y = y - shift[1]
    v = 128 + 60 * np.sin(x / 7.0) * np.cos(y / 9.0) + 40 * np.sin((x + 2 * y) / 13.0)
    return np.clip(np.rint(v), 0, 255).astype(np.uint8)


def test_lk_integer_translation_exact():
    A = smooth_image(200, 160)
    B = np.roll(np.roll(A, 3, axis=1), -2, axis=0)
    pts = np.array([[60 + 7 * i, 50 + 5 * (i % 9)] for i in range(12)], np.float32)
    nx, st, err, _ = O.lk(A, B, pts, (21, 21), 3, (3, 50, 1e-3), 0)
    assert st.all()
    assert np.abs(nx - (pts + [3, -2])).max() < 0.01


def test_lk_subpixel_translation():
    A = smooth_image(200, 160)
    B = smooth_image(200, 160, shift=(1.37, -0.82))
    pts = np.array([[60 + 7 * i, 50 + 5 * (i % 9)] for i in range(12)], np.float32)
    nx, st, _, _ = O.lk(A, B, pts, (21, 21), 3, (3, 50, 1e-3), O.LK_GET_MIN_EIGENVALS)
    assert st.all()
    assert np.abs(nx - (pts + [1.37, -0.82])).max() < 0.05


def test_lk_accumulation_modes_agree_within_tolerance():
    A = smooth_image(200, 160)
    B = smooth_image(200, 160, shift=(0.6, 0.3))
    pts = np.array([[40 + 9 * i, 40 + 6 * (i % 11)] for i in range(14)], np.float32)
    ex = O.lk(A, B, pts, (21, 21), 3, (3, 50, 1e-3), 0, acc=O.ACC_EXACT)
    for acc in (O.ACC_SCALAR, O.ACC_SSE):
        r = O.lk(A, B, pts, (21, 21), 3, (3, 50, 1e-3), 0, acc=acc)
        assert np.array_equal(r[1], ex[1])
        assert np.abs(r[0] - ex[0]).max() < 1e-3


def test_lk_out_of_image_point_fails_and_flat_window_fails():
    A = np.full((100, 100), 128, np.uint8)
    pts = np.array([[50, 50], [-40, 50], [50, 150]], np.float32)
    nx, st, err, _ = O.lk(A, A, pts, (21, 21), 2, (3, 30, 0.01), O.LK_GET_MIN_EIGENVALS)
    assert not st.any()                              # flat: minEig < 1e-4; outside: bounds
    assert err[1] == 0 and err[2] == 0


# ------------------------------------------------------------------ RANSAC / PnP
def test_rng_mwc_recurrence():
    s = 0xFFFFFFFFFFFFFFFF
    ref = []
    for _ in range(5):
        s = ((s & 0xFFFFFFFF) * 4164903690 + (s >> 32)) & 0xFFFFFFFFFFFFFFFF
        ref.append(s & 0xFFFFFFFF)
    assert O.rng_sequence(5) == ref


def test_ransac_update_num_iters():
    assert O.update_num_iters(0.999, 0.5, 5, 100) == 100                  # 217.6 -> capped
    assert O.update_num_iters(0.999, 0.1, 5, 100) == round(math.log(0.001) / math.log(1 - 0.9 ** 5))
    assert O.update_num_iters(0.999, 0.0, 5, 100) == 0                    # all inliers: stop
    assert O.update_num_iters(0.999, 1.0, 5, 100) == 100


def test_rodrigues_roundtrip():
    for rv in ([0.1, -0.2, 0.3], [1e-9, 0, 0], [0, 0, math.pi - 1e-3], [2.0, 1.0, -0.5]):
        R = O.rodrigues(rv)
        assert np.allclose(R @ R.T, np.eye(3), atol=1e-12)
        assert np.allclose(O.rodrigues(O.rodrigues_inv(R)), R, atol=1e-9)


def _pnp_case(n=300, outliers=40, seed=0):
    rng = np.random.default_rng(seed)
    K = np.array([[718.856, 0, 607.1928], [0, 718.856, 185.2157], [0, 0, 1]], np.float32).astype(np.float64)
    X = np.c_[rng.uniform(-8, 8, n), rng.uniform(-3, 3, n), rng.uniform(6, 40, n)]
    rv = np.array([0.02, -0.05, 0.01])
    t = np.array([0.3, -0.1, 0.5])
    R = O.rodrigues(rv)
    uv = (K @ (R @ X.T + t[:, None])).T
    uv = (uv[:, :2] / uv[:, 2:]).astype(np.float32)
    bad = rng.choice(n, outliers, replace=False)
    uv[bad] += rng.uniform(60, 200, (outliers, 2)).astype(np.float32) * rng.choice([-1, 1], (outliers, 2))
    return X, uv, K, R, t, bad


def test_ransac_exact_inliers_known():
    X, uv, K, R, t, bad = _pnp_case()
    rc, rv, tv, inl, nh = O.solve_pnp_ransac(X, uv, K)
    assert rc == 1
    assert np.array_equal(inl, np.setdiff1d(np.arange(len(X)), bad))
    assert np.allclose(O.rodrigues(rv), R, atol=1e-6) and np.allclose(tv, t, atol=1e-5)


def test_epnp_exact_on_clean_points():
    X, uv, K, R, t, bad = _pnp_case(outliers=0)
    rc, Re, te = O.epnp(X[:50], uv[:50], K)
    assert rc == 0 and np.allclose(Re, R, atol=1e-5) and np.allclose(te, t, atol=1e-4)


def test_pnp_residual_formula():
    X, uv, K, R, t, bad = _pnp_case(outliers=0)
    err, mask, cnt = O.pnp_residuals(X, uv, np.r_[R.ravel(), t][None], K, 64.0)
    assert cnt[0] == len(X) and err.max() < 1e-6


def test_ransac_too_few_points():
    assert O.solve_pnp_ransac(np.zeros((3, 3)), np.zeros((3, 2), np.float32), np.eye(3))[0] == -1


# ------------------------------------------------------------------ bucket (R:src/bucket.cpp)
def test_bucket_slot0_overwrite_quirk():
    # 4 points in bucket (0,0) with k = 2: slot 0 ends with the LAST point
    pts = np.array([[1, 1], [2, 2], [3, 3], [4, 4]], np.float32)
    xy, ages = O.bucket(pts, 100, 100, 50, 2)
    assert np.array_equal(xy, np.array([[4, 4], [2, 2]], np.float32))


def test_bucket_stride_aliasing_quirk():
    # W = 120, B = 50: nw = 2 but column index 2 exists (x in [100, 120)):
    # idx = r*2 + 2 == (r+1)*2 + 0, and that bucket is read out twice
    pts = np.array([[110, 10], [5, 60]], np.float32)
    xy, _ = O.bucket(pts, 120, 100, 50, 3)
    assert np.array_equal(xy, np.array([[110, 10], [5, 60], [110, 10], [5, 60]], np.float32))


def test_bucket_order_by_bucket_then_input():
    # readout walks r in [0, nh], c in [0, nw] with idx = r*nw + c: with W = H = 100,
    # B = 50 (nw = nh = 2), cell (0, 2) is bucket 2 == cell (1, 0), so the point
    # of cell (1, 0) comes out twice, right after row 0's buckets
    pts = np.array([[60, 5], [5, 5], [70, 8], [6, 60]], np.float32)
    xy, _ = O.bucket(pts, 100, 100, 50, 4)
    assert np.array_equal(xy, np.array([[5, 5], [60, 5], [70, 8], [6, 60], [6, 60]], np.float32))


# ------------------------------------------------------------------ golden drift guard
def test_oracle_matches_committed_golden():
    g = np.load(os.path.join(HERE, "golden", "small_160x120.npz"))
    A, B = g["A"], g["B"]
    pyr = O.build_pyramid(A, (21, 21), 3)
    for l in range(1, len(pyr)):
        assert np.array_equal(pyr[l], g[f"pyr{l}"])
    assert np.array_equal(O.fast(A, 20, True), g["kp_nms"])
    assert np.array_equal(O.fast(A, 20, False), g["kp_all"])
    assert np.array_equal(O.fast(A, 20, True, g["mask"]), g["kp_mask"])
    pts = g["pts"]
    n, s, e, _ = O.lk(A, B, pts, (21, 21), 3, (3, 50, 1e-3), O.LK_GET_MIN_EIGENVALS)
    assert np.array_equal(n, g["t_next"]) and np.array_equal(s, g["t_status"]) and np.array_equal(e, g["t_err"])
    n, s, e, _ = O.lk(A, B, pts, (11, 11), 3, (3, 30, 1e-3), 0)
    assert np.array_equal(n, g["s_next"]) and np.array_equal(s, g["s_status"]) and np.array_equal(e, g["s_err"])
    bx, _ = O.bucket(g["kp_all"][:, :2], 160, 120, 50, 2)
    assert np.array_equal(bx, g["bucket_xy"])
    rc, rv, tv, inl, _ = O.solve_pnp_ransac(g["X"], g["t_next"], g["K"])
    assert np.array_equal(inl, g["pnp_inliers"])
    assert np.allclose(rv, g["pnp_rvec"], atol=1e-9) and np.allclose(tv, g["pnp_tvec"], atol=1e-9)


# ------------------------------------------------------------------ triangulation (cv::triangulatePoints)
def test_kat_triangulate_exact_projections():
    """Points projected exactly by P0 = K[I|0] and P1 = K[I|(-b,0,0)] triangulate back."""
    K = np.array([[718.856, 0, 607.1928], [0, 718.856, 185.2157], [0, 0, 1]])
    P0 = np.zeros((3, 4)); P0[:, :3] = K
    P1 = P0.copy(); P1[0, 3] = -386.1448
    P0, P1 = P0.astype(np.float32), P1.astype(np.float32)
    rng = np.random.default_rng(0)
    X = np.c_[rng.uniform(-5, 5, 50), rng.uniform(-2, 2, 50), rng.uniform(4, 40, 50)]
    Xh = np.c_[X, np.ones(50)]
    p1 = (P0.astype(np.float64) @ Xh.T); p1 = (p1[:2] / p1[2]).T.astype(np.float32)
    p2 = (P1.astype(np.float64) @ Xh.T); p2 = (p2[:2] / p2[2]).T.astype(np.float32)
    h, x = O.triangulate(P0, P1, p1, p2)
    assert np.all(h[:, 3] >= 0)
    assert np.allclose(np.linalg.norm(h, axis=1), 1, atol=1e-6)
    rel = np.abs(x - X).max(1) / X[:, 2]
    assert rel.max() < 2e-4, rel.max()     # float pixel rounding only
    # behind-camera point keeps z < 0 (the reference filters on z > 0)
    Xb = np.array([[0.5, 0.2, -8.0, 1.0]])
    q1 = P0.astype(np.float64) @ Xb.T; q2 = P1.astype(np.float64) @ Xb.T
    _, xb = O.triangulate(P0, P1, (q1[:2] / q1[2]).T, (q2[:2] / q2[2]).T)
    assert xb[0, 2] < 0 and abs(xb[0, 2] + 8.0) < 1e-3


# ------------------------------------------------------------------ SQPnP (solvePnP SOLVEPNP_SQPNP)
def _sqpnp_case(n, noise, seed):
    from scipy.spatial.transform import Rotation as Rot
    rng = np.random.default_rng(seed)
    X = np.c_[rng.uniform(-15, 15, n), rng.uniform(-4, 4, n), rng.uniform(6, 40, n)]
    R = Rot.from_rotvec([0.02, -0.05, 0.01]).as_matrix()
    t = np.array([0.3, -0.1, 0.8])
    Y = X @ R.T + t
    q = Y[:, :2] / Y[:, 2:] + rng.normal(0, noise, (n, 2))
    return X, q, R, t


def test_kat_sqpnp_exact_correspondences():
    """Noise-free normalised projections: SQPnP returns the generating pose."""
    X, q, R, t = _sqpnp_case(200, 0.0, 1)
    rc, Rs, ts = O.sqpnp(X, q)
    assert rc == 0
    assert np.abs(Rs - R).max() < 1e-9 and np.abs(ts - t).max() < 1e-9


def test_kat_sqpnp_is_the_algebraic_cost_minimiser():
    """With noise, SQPnP's pose is the global minimiser of its cost, the
    algebraic image-space error [1 0 -x; 0 1 -y](R X + t) summed over the points
    (PoseSolver::computeOmega): an independent least-squares solve from the
    generating pose lands on the same pose."""
    from scipy.optimize import least_squares
    from scipy.spatial.transform import Rotation as Rot
    X, q, R, t = _sqpnp_case(500, 6e-4, 2)  # ~0.4 px at KITTI's focal length
    rc, Rs, ts = O.sqpnp(X, q)
    assert rc == 0

    def res(p):
        Y = X @ Rot.from_rotvec(p[:3]).as_matrix().T + p[3:]
        return np.r_[Y[:, 0] - q[:, 0] * Y[:, 2], Y[:, 1] - q[:, 1] * Y[:, 2]]
    p = least_squares(res, np.r_[Rot.from_matrix(R).as_rotvec(), t], xtol=1e-15, ftol=1e-15, gtol=1e-15).x
    assert np.abs(Rot.from_rotvec(p[:3]).as_matrix() - Rs).max() < 1e-8
    assert np.abs(p[3:] - ts).max() < 1e-8
    assert np.abs(Rs @ Rs.T - np.eye(3)).max() < 1e-9          # a rotation
    assert np.abs(Rs - R).max() > 1e-6                          # (and not the noise-free pose)


def test_kat_sqpnp_degenerate_image_points():
    """All image points at one spot: SQPnP's point-variance assert (rc -1)."""
    X, q, _, _ = _sqpnp_case(50, 0.0, 3)
    q[:] = q[0]
    rc, _, _ = O.sqpnp(X, q)
    assert rc == -1
