"""LK in OpenCV's own float summation order (SVO_LK_OPENCV_ORDER, lk_cv_kernel).

cv::calcOpticalFlowPyrLK's x86 build sums the normal equations in float: four
SSE lanes plus a scalar tail, then its lane reduction (LKTrackerInvoker in
lkpyramid.cpp; restated by oracle/lk.c as ACC_SSE). The product's default LK
sums exactly; under SVO_LK_OPENCV_ORDER it reproduces the SSE order, and then
every output -- points, status, err, iteration counts -- is bit-identical to the
oracle's ACC_SSE at the reference's two call sites (R:src/tracking.cpp:101-105
stereo 11x11 flags 0, :160-165 temporal 21x21 MIN_EIGENVALS), at BASELINE.json's
configs, for runtime windows whose SIMD / scalar column split differs, and
through the whole reference loop (the batched front end against the oracle loop
run with ACC_SSE: zero differing positions, no exemption for points that run
into the iteration cap).
"""
import numpy as np
import pytest

import oracle as O
import svo_amd as S
from oracle_loop import OracleLoop
from svo_amd.scene import Scene, SceneForward

pytestmark = pytest.mark.gpu

CV = S.LK_OPENCV_ORDER
TEMPORAL = dict(win=(21, 21), ml=3, crit=(3, 50, 1e-3), flags=S.LK_GET_MIN_EIGENVALS)  # R:src/tracking.cpp:160-165
STEREO = dict(win=(11, 11), ml=3, crit=(3, 30, 1e-3), flags=0)                        # R:src/tracking.cpp:101-105


@pytest.fixture(scope="module")
def ctx():
    return S.Context(0)


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _check(ctx, A, B, pts, win, ml, crit, flags, want_err=True):
    ga, gb = ctx.image(A, ml + 2), ctx.image(B, ml + 2)
    gn, gs, ge = ctx.calc_optical_flow_pyr_lk(ga, gb, pts, win_size=win, max_level=ml, criteria=crit,
                                              flags=flags | CV, want_err=want_err)
    git = ctx.lk_last_iterations()
    rn, rs, re_, it = O.lk(A, B, pts, win, ml, crit, flags, acc=O.ACC_SSE, want_err=want_err)
    assert np.array_equal(gs, rs), f"status differs at {np.nonzero(gs != rs)[0][:10]}"
    bad = np.nonzero((_bits(gn) != _bits(rn)).any(1))[0]
    assert len(bad) == 0, f"{len(bad)} points differ, first {bad[:8]}: {gn[bad[:4]]} vs {rn[bad[:4]]}"
    if want_err:
        assert np.array_equal(_bits(ge), _bits(re_))
    assert git == int(it.sum())
    return gn, gs


@pytest.fixture(params=["four-per-wave", "one-per-wave"])
def cv_kernel(request, monkeypatch):
    """Both OpenCV-order kernels: lk_cvq_kernel (21x21 / 11x11, four features per
    wave; not the SAD error of flags 0 + err) and lk_cv_kernel (one per wave: every
    other window and SVO_LK_QUAD=0)."""
    monkeypatch.setenv("SVO_LK_QUAD", "1" if request.param == "four-per-wave" else "0")
    return request.param


@pytest.mark.parametrize("cfg", [TEMPORAL, STEREO], ids=["temporal21", "stereo11"])
@pytest.mark.parametrize("wh,seed,n", [((1241, 376), 0, 2000), ((160, 120), 1, 300), ((1920, 1080), 2, 4000)])
@pytest.mark.parametrize("want_err", [True, False], ids=["err", "noerr"])
def test_lk_opencv_order_bit_exact(ctx, cv_kernel, cfg, wh, seed, n, want_err):
    sc = Scene(*wh, seed=seed)
    A, B = sc.frame(0), sc.frame(1) if cfg is TEMPORAL else sc.right(0)
    pts = O.fast(A, 20, True)[:n, :2]
    gn, gs = _check(ctx, A, B, pts, cfg["win"], cfg["ml"], cfg["crit"], cfg["flags"], want_err=want_err)
    if wh == (1241, 376):
        # not vacuous: the exact sums (the default) stop elsewhere for some points
        xn, xs, _, _ = O.lk(A, B, pts, cfg["win"], cfg["ml"], cfg["crit"], cfg["flags"], acc=O.ACC_EXACT)
        assert (_bits(xn) != _bits(gn)).any()


@pytest.mark.parametrize("cfg", [TEMPORAL, STEREO], ids=["temporal21", "stereo11"])
@pytest.mark.parametrize("wh,seed,n,ml", [((1920, 1080), 2, 8000, 4), ((3840, 2160), 3, 16000, 3)],
                         ids=["1080p-8000-ml4", "4k-16000-ml3"])
def test_lk_opencv_order_baseline_configs(ctx, cfg, wh, seed, n, ml):
    """BASELINE.json configs[2] / [3] at full size, both windows; the temporal call
    with the config's maxLevel, the stereo call with the reference's 3."""
    sc = Scene(*wh, seed=seed)
    A, B = sc.frame(0), sc.frame(1) if cfg is TEMPORAL else sc.right(0)
    pts = O.fast(A, 20, True)[:n, :2]
    assert len(pts) == n
    _, gs = _check(ctx, A, B, pts, cfg["win"], ml if cfg is TEMPORAL else 3, cfg["crit"], cfg["flags"])
    assert gs.sum() > 0.9 * n


@pytest.mark.parametrize("win", [(3, 3), (4, 4), (5, 7), (7, 5), (8, 8), (9, 9), (12, 12), (13, 9), (15, 15),
                                 (16, 16), (17, 13), (23, 23), (31, 31)])
def test_lk_opencv_order_windows(ctx, win):
    """Windows whose 4- / 8-column SIMD ends and scalar tails differ (se4 = 0..28,
    se8 = 0..24), with points near and beyond the image borders."""
    sc = Scene(320, 240, seed=win[0] * 7 + win[1])
    A, B = sc.frame(0), sc.frame(1)
    rng = np.random.default_rng(win[0])
    pts = np.concatenate([O.fast(A, 20, True)[:300, :2], rng.uniform(-40, 360, (100, 2)),
                          np.array([[0, 0], [319, 239], [-21, 5], [5, -21], [339.9, 120]])]).astype(np.float32)
    for flags in (S.LK_GET_MIN_EIGENVALS, 0):
        _check(ctx, A, B, pts, win, 3, (3, 30, 1e-3), flags)


def test_lk_opencv_order_initial_flow_and_criteria(ctx):
    """USE_INITIAL_FLOW guesses and criteria without EPS / COUNT (OpenCV's
    defaults 30 / 0.01) in the ordered mode."""
    sc = Scene(640, 376, seed=5)
    A, B = sc.frame(0), sc.frame(2)
    pts = O.fast(A, 20, True)[:800, :2]
    guess = (pts + np.float32(1.5)).astype(np.float32)
    ga, gb = ctx.image(A, 5), ctx.image(B, 5)
    for crit in ((3, 50, 1e-3), (1, 7, 0.0), (2, 0, 0.3)):
        gn, gs, ge = ctx.calc_optical_flow_pyr_lk(ga, gb, pts, guess, win_size=(21, 21), max_level=3, criteria=crit,
                                                  flags=S.LK_USE_INITIAL_FLOW | CV)
        rn, rs, re_, _ = O.lk(A, B, pts, (21, 21), 3, crit, O.LK_USE_INITIAL_FLOW, acc=O.ACC_SSE, next_pts=guess)
        assert np.array_equal(gs, rs)
        assert np.array_equal(_bits(gn), _bits(rn))
        assert np.array_equal(_bits(ge), _bits(re_))


def _loop(ctx, scenes, T, N):
    sc0 = scenes[0]
    cfg = S.FrontendConfig(sc0.w, sc0.h, sc0.K, n_seq=len(scenes), n_frames=T, n_features=N,
                           lk_flags=S.LK_GET_MIN_EIGENVALS | CV)
    fe = S.Frontend(ctx, cfg)
    for s, sc in enumerate(scenes):
        for t in range(T):
            fe.set_frame(s, t, sc.frame(t), sc.right(t))
    return fe


def test_frontend_opencv_order_200_frames_kitti(ctx):
    """The reference loop (R:src/tracking.cpp:232-276) at BASELINE configs[1]'s size
    for 200 frames, both LK calls in OpenCV's order, against the oracle loop with
    ACC_SSE every step: counts (including GN iterations), feature lists bit for bit
    (zero differing positions), poses and map points."""
    W, H, N, T = 1241, 376, 2000, 201
    fe = _loop(ctx, [Scene(W, H, seed=0)], T, N)
    fe.init(0)
    ref = OracleLoop(Scene(W, H, seed=0), N, acc=O.ACC_SSE).init(0)
    assert np.array_equal(fe.features(0), ref.pts)
    for t in range(1, T):
        st = fe.step(t).as_dict()
        rs = ref.step(t)
        for k in ("tracked", "lk_iterations", "inliers", "added", "features"):
            assert st[k] == rs[k], f"{k} differs at t={t}: {st[k]} vs {rs[k]}"
        got = fe.features(0)
        assert got.shape == ref.pts.shape and np.array_equal(_bits(got), _bits(ref.pts)), f"features differ at t={t}"
        rv, tv = fe.pose(0)
        np.testing.assert_allclose(rv, ref.pose[0], atol=1e-7)
        np.testing.assert_allclose(tv, ref.pose[1], atol=1e-6)
        if t % 50 == 0:
            np.testing.assert_allclose(fe.map_points(0), ref.X, rtol=2e-5, atol=1e-6)
    fe.close()


def test_frontend_opencv_order_forward_occluder(ctx):
    """The forward / occluder scene (RANSAC drops 9-26 %; features near the occluder
    run to the 50-iteration cap) on two sequences, 30 steps, against the oracle
    loop with ACC_SSE."""
    W, H, N, T = 1241, 376, 2000, 31
    seeds = (1, 4)
    fe = _loop(ctx, [SceneForward(W, H, seed=s) for s in seeds], T, N)
    fe.init(0)
    refs = [OracleLoop(SceneForward(W, H, seed=s), N, acc=O.ACC_SSE).init(0) for s in seeds]
    for t in range(1, T):
        st = fe.step(t).as_dict()
        rss = [r.step(t) for r in refs]
        for k in ("tracked", "lk_iterations", "inliers", "added", "features"):
            assert st[k] == sum(rs[k] for rs in rss), f"{k} differs at t={t}"
        for q, ref in enumerate(refs):
            assert np.array_equal(_bits(fe.features(q)), _bits(ref.pts)), f"seq {q} features differ at t={t}"
            rv, tv = fe.pose(q)
            np.testing.assert_allclose(rv, ref.pose[0], atol=1e-7)
            np.testing.assert_allclose(tv, ref.pose[1], atol=1e-6)
    fe.close()
