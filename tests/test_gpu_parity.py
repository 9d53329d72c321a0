"""GPU-vs-oracle parity of every HIP kernel on the hot path.

All calls go through the C ABI (libsvo_gpu.so via svo_amd's ctypes layer).
Bar: bit-exact for the integer work (pyramid, FAST score map, keypoint lists,
masks, bucket selection) and for the fixed-point LK / double PnP residuals
against the oracle's EXACT accumulation mode; LK additionally within 0.1 px of
the oracle's restatement of OpenCV's own (SSE) float accumulation order.
"""
import numpy as np
import pytest

import oracle as O
import svo_amd as S
from svo_amd.scene import Scene

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    return S.Context(0)


def frames(w, h, seed=0, t0=0, t1=1):
    sc = Scene(w, h, seed=seed)
    return sc, sc.frame(t0), sc.frame(t1)


# ------------------------------------------------------------------ pyramid
@pytest.mark.parametrize("wh", [(1241, 376), (160, 120), (161, 121), (97, 33), (1920, 1080), (7, 5), (1, 1), (2, 3)])
def test_pyramid_bit_exact(ctx, wh):
    w, h = wh
    rng = np.random.default_rng(w * 1000 + h)
    img = rng.integers(0, 256, (h, w), dtype=np.uint8)
    g = ctx.image(img, max_levels=4)
    lvl = img
    for l in range(5):
        got = g.level(l)
        assert got.shape == lvl.shape
        assert np.array_equal(got, lvl), f"level {l} differs"
        lvl = O.pyr_down(lvl)


# ------------------------------------------------------------------ Scharr derivative pyramid
@pytest.mark.parametrize("wh", [(1241, 376), (161, 121), (97, 33), (7, 5), (2, 3)])
def test_scharr_levels_bit_exact(ctx, wh):
    """svo_image_scharr_level: every level's Scharr derivatives (stored x4, as LK
    reads them) against the oracle's calcSharrDeriv restatement on that level."""
    w, h = wh
    rng = np.random.default_rng(w + 7 * h)
    img = rng.integers(0, 256, (h, w), dtype=np.uint8)
    g = ctx.image(img, max_levels=3)
    lvl = img
    for l in range(4):
        ix, iy = g.scharr(l)
        ref = O.scharr(lvl).astype(np.int32)
        assert np.array_equal(ix.astype(np.int32), 4 * ref[..., 0]), f"ix level {l}"
        assert np.array_equal(iy.astype(np.int32), 4 * ref[..., 1]), f"iy level {l}"
        lvl = O.pyr_down(lvl)


@pytest.mark.parametrize("wh", [(1241, 376), (640, 376), (401, 203)])
def test_frontend_scharr_pyramid_bit_exact(ctx, wh):
    """The front end's fused pyrDown + Scharr pass (pyr_scharr_kernel; scharr_kernel
    for the coarsest level) against the oracle on every level of its frames."""
    w, h = wh
    scenes = [Scene(w, h, seed=s) for s in (3, 4)]
    cfg = S.FrontendConfig(w, h, scenes[0].K, n_seq=2, n_frames=3, n_features=300)
    fe = S.Frontend(ctx, cfg)
    for s, sc in enumerate(scenes):
        for t in range(3):
            fe.set_frame(s, t, sc.frame(t), sc.right(t))
    fe.init(0)
    fe.step(1)   # builds frame 2's derivatives ahead (frames 1 and 2 resident)
    for s, sc in enumerate(scenes):
        for t in (1, 2):
            lvl = sc.frame(t)
            for l in range(4):
                ix, iy = fe.scharr(s, t, l, lvl.shape[1], lvl.shape[0])
                ref = O.scharr(lvl).astype(np.int32)
                assert np.array_equal(ix.astype(np.int32), 4 * ref[..., 0]), f"seq {s} t {t} ix level {l}"
                assert np.array_equal(iy.astype(np.int32), 4 * ref[..., 1]), f"seq {s} t {t} iy level {l}"
                lvl = O.pyr_down(lvl)
    fe.close()


def _levels_for_window(w, h, win, max_level):
    """common.hpp lk_levels_for_window (buildOpticalFlowPyramid's level cap)."""
    for level in range(max_level + 1):
        w, h = (w + 1) // 2, (h + 1) // 2
        if w <= win or h <= win:
            return level
    return max_level


@pytest.mark.parametrize("wh,max_level,win", [((1241, 376), 3, 21), ((401, 203), 3, 21), ((97, 61), 4, 5),
                                              ((45, 37), 3, 3), ((1920, 1080), 4, 21), ((130, 70), 1, 21),
                                              ((66, 34), 2, 5), ((257, 129), 5, 3)])
@pytest.mark.parametrize("fused", ["1", "0"])
def test_frontend_pyramids_with_borders(ctx, wh, max_level, win, fused, monkeypatch):
    """The front end's left pyramids (pyrDown + Scharr + the source level's border
    per launch; the last two levels, their derivatives and borders in one fused
    launch) and right pyramids, each
    level with its stored REFLECT_101 border, against the oracle's pyrDown chain
    padded by numpy's reflect (= BORDER_REFLECT_101, repeated for tiny levels); the
    derivatives of every level against the oracle's Scharr. Both forms: the fused
    chain of the last two levels (SVO_PYR_FUSED=1, the default) and one launch per
    level + the border pass (0); the switch is read at every launch."""
    monkeypatch.setenv("SVO_PYR_FUSED", fused)
    w, h = wh
    P = S.PYR_PAD
    scenes = [Scene(w, h, seed=s) for s in (5, 6)]
    cfg = S.FrontendConfig(w, h, scenes[0].K, n_seq=2, n_frames=3, n_features=300, max_level=max_level,
                           stereo_max_level=max_level, win=win, stereo_win=win)
    nlev = _levels_for_window(w, h, win, max_level) + 1
    fe = S.Frontend(ctx, cfg)
    for s, sc in enumerate(scenes):
        for t in range(3):
            fe.set_frame(s, t, sc.frame(t), sc.right(t))
    fe.init(0)
    fe.step(1)   # left pyramids of frames 1 and 2, right pyramid of frame 1
    for s, sc in enumerate(scenes):
        for t, right in ((1, False), (2, False), (1, True)):
            lvl = sc.right(t) if right else sc.frame(t)
            for l in range(nlev):
                got = fe.pyramid_level(s, t, l, lvl.shape[1], lvl.shape[0], right=right)
                ref = np.pad(lvl, P, mode="reflect")
                assert np.array_equal(got, ref), f"seq {s} t {t} right {right} level {l} ({lvl.shape})"
                if not right:
                    ix, iy = fe.scharr(s, t, l, lvl.shape[1], lvl.shape[0])
                    rd = O.scharr(lvl).astype(np.int32)
                    assert np.array_equal(ix.astype(np.int32), 4 * rd[..., 0]), f"seq {s} t {t} ix level {l}"
                    assert np.array_equal(iy.astype(np.int32), 4 * rd[..., 1]), f"seq {s} t {t} iy level {l}"
                lvl = O.pyr_down(lvl)
    fe.close()


# ------------------------------------------------------------------ FAST
@pytest.mark.parametrize("wh,seed", [((1241, 376), 0), ((160, 120), 3), ((64, 48), 5), ((3840, 2160), 1)])
def test_fast_score_map_bit_exact(ctx, wh, seed):
    sc, A, _ = frames(*wh, seed=seed)
    g = ctx.image(A, 0)
    for t in (0, 7, 20, 60):
        s, c = ctx.fast_score_map(g, t)
        so, co = O.fast_score(A, t)
        assert np.array_equal(c, co), f"corner map differs at t={t}"
        assert np.array_equal(s, so), f"score map differs at t={t}"


@pytest.mark.parametrize("nonmax", [True, False])
@pytest.mark.parametrize("wh,seed", [((1241, 376), 0), ((160, 120), 2), ((1920, 1080), 4)])
def test_fast_keypoints_identical(ctx, wh, seed, nonmax):
    sc, A, _ = frames(*wh, seed=seed)
    g = ctx.image(A, 0)
    det = S.FastFeatureDetector.create(ctx, 20, nonmax)
    got = det.detect(g)
    ref = O.fast(A, 20, nonmax)
    assert got.shape == ref.shape
    assert np.array_equal(got, ref)


def test_fast_with_mask_identical(ctx):
    sc, A, _ = frames(1241, 376, seed=0)
    g = ctx.image(A, 0)
    prev = O.fast(A, 20, True)[::3, :2] + np.float32(0.37)
    m_gpu = ctx.mask_boxes(1241, 376, prev, 10.0)
    m_ref = O.mask_boxes(1241, 376, prev, 10.0)
    assert np.array_equal(m_gpu, m_ref)
    got = ctx.fast_detect(g, 20, True, m_gpu)
    ref = O.fast(A, 20, True, m_ref)
    assert np.array_equal(got, ref)
    assert len(ref) < len(O.fast(A, 20, True))


def test_mask_boxes_edges(ctx):
    pts = np.array([[0.5, 0.5], [10.5, 10.5], [-3.0, 5.0], [63.4, 47.6], [30.5, 20.5], [100, 100]], np.float32)
    assert np.array_equal(ctx.mask_boxes(64, 48, pts, 10.0), O.mask_boxes(64, 48, pts, 10.0))


def test_fast_threshold_extremes(ctx):
    sc, A, _ = frames(160, 120, seed=9)
    g = ctx.image(A, 0)
    for t in (0, 1, 254, 255, 300, -5):
        assert np.array_equal(ctx.fast_detect(g, t, True), O.fast(A, max(0, min(255, t)), True))


# ------------------------------------------------------------------ bucket
@pytest.mark.parametrize("B,k", [(50, 4), (37, 1), (64, 7), (100, 2)])
def test_bucket_identical(ctx, B, k):
    sc, A, _ = frames(1241, 376, seed=1)
    kp = O.fast(A, 20, True)[:, :2]
    ages = np.arange(len(kp), dtype=np.int32) % 5
    for a in (None, ages):
        gx, ga = ctx.bucket_features(kp, 1241, 376, B, k, a)
        rx, ra = O.bucket(kp, 1241, 376, B, k, a)
        assert np.array_equal(gx, rx)
        assert np.array_equal(ga, ra)


def test_bucket_empty(ctx):
    gx, ga = ctx.bucket_features(np.zeros((0, 2), np.float32), 640, 480, 50, 4)
    assert len(gx) == 0


# ------------------------------------------------------------------ LK
def _lk_pair(ctx, w, h, seed, npts, win, ml, crit, flags, t1=1):
    sc, A, B = frames(w, h, seed=seed, t1=t1)
    pts = O.fast(A, 20, True)[:npts, :2]
    ga, gb = ctx.image(A, 6), ctx.image(B, 6)
    got = ctx.calc_optical_flow_pyr_lk(ga, gb, pts, win_size=win, max_level=ml, criteria=crit, flags=flags)
    ref = O.lk(A, B, pts, win, ml, crit, flags, acc=O.ACC_EXACT)
    sse = O.lk(A, B, pts, win, ml, crit, flags, acc=O.ACC_SSE)
    return sc, pts, got, ref, sse


TEMPORAL = dict(win=(21, 21), ml=3, crit=(3, 50, 1e-3), flags=S.LK_GET_MIN_EIGENVALS)  # R:src/tracking.cpp:160-165
STEREO = dict(win=(11, 11), ml=3, crit=(3, 30, 1e-3), flags=0)                        # R:src/tracking.cpp:101-105


@pytest.fixture(params=["fixed-window", "generic", "one-per-wave"])
def lk_kernel(request, monkeypatch):
    """Every LK kernel: the compile-time-window ones (21x21 four features per
    wave by default, 11x11, 15x15, 31x31), the 21x21 one-feature-per-wave kernel
    (SVO_LK_QUAD=0) and the runtime-window one every other size uses
    (SVO_LK_GENERIC=1)."""
    monkeypatch.setenv("SVO_LK_GENERIC", "1" if request.param == "generic" else "0")
    monkeypatch.setenv("SVO_LK_QUAD", "0" if request.param == "one-per-wave" else "1")
    return request.param


@pytest.mark.parametrize("cfg", [TEMPORAL, STEREO], ids=["temporal21", "stereo11"])
@pytest.mark.parametrize("wh,seed,n", [((1241, 376), 0, 2000), ((160, 120), 1, 300), ((1920, 1080), 2, 4000)])
def test_lk_bit_exact(ctx, cfg, wh, seed, n, lk_kernel):
    sc, pts, got, ref, sse = _lk_pair(ctx, *wh, seed, n, cfg["win"], cfg["ml"], cfg["crit"], cfg["flags"])
    gn, gs, ge = got
    rn, rs, re_, _ = ref
    assert np.array_equal(gs, rs), f"status differs at {np.nonzero(gs != rs)[0][:10]}"
    assert np.array_equal(gn.view(np.uint32), rn.view(np.uint32)), \
        f"max |d| {np.abs(gn - rn).max()} at {np.argmax(np.abs(gn - rn).max(1))}"
    assert np.array_equal(ge.view(np.uint32), re_.view(np.uint32))
    # OpenCV's own float accumulation order (SSE path) is within 0.1 px
    sn, ss, _, _ = sse
    ok = (gs == 1) & (ss == 1)
    assert np.abs(gn[ok] - sn[ok]).max() <= 0.1
    # observed on every case here: no status differs from the SSE-order accumulation
    assert int((gs != ss).sum()) == 0, f"{int((gs != ss).sum())} status flips vs the SSE order"


@pytest.mark.parametrize("wh,seed,n", [((1241, 376), 0, 2000), ((160, 120), 1, 300), ((1920, 1080), 2, 4000)])
def test_lk_stereo_without_err_bit_exact(ctx, wh, seed, n):
    """The stereo call as the front end makes it (11 x 11, flags 0, no err output:
    findLeftFeaturesInRight reads status and points only) runs the four-features-
    per-wave kernel (lk_multi_kernel<.., 11, 11, 11>, one 11-row strip per lane):
    points and status bit-identical to the oracle's EXACT accumulation, also for
    points outside the image."""
    sc, A, B = frames(*wh, seed=seed)
    pts = O.fast(A, 20, True)[:n, :2]
    rng = np.random.default_rng(seed)
    pts = np.concatenate([pts, rng.uniform(-30, max(wh) + 30, (64, 2))]).astype(np.float32)
    ga, gb = ctx.image(A, 6), ctx.image(B, 6)
    c = STEREO
    gn, gs, ge = ctx.calc_optical_flow_pyr_lk(ga, gb, pts, win_size=c["win"], max_level=c["ml"], criteria=c["crit"],
                                              flags=c["flags"], want_err=False)
    assert ge is None
    rn, rs, _, it = O.lk(A, B, pts, c["win"], c["ml"], c["crit"], c["flags"], acc=O.ACC_EXACT)
    assert np.array_equal(gs, rs), f"status differs at {np.nonzero(gs != rs)[0][:10]}"
    assert np.array_equal(gn.view(np.uint32), rn.view(np.uint32))
    assert ctx.lk_last_iterations() == int(it.sum())


# BASELINE.json configs[2] / [3] at full size: 1080p, 8000 features, maxLevel 4 (five
# levels, not clamped by the window) and 4K, 16000 features, maxLevel 3; the temporal
# call's window / criteria / flags (R:src/tracking.cpp:160-165)
@pytest.mark.parametrize("wh,seed,n,ml", [((1920, 1080), 2, 8000, 4), ((3840, 2160), 3, 16000, 3)],
                         ids=["1080p-8000-ml4", "4k-16000-ml3"])
def test_lk_baseline_configs(ctx, wh, seed, n, ml):
    sc, A, B = frames(*wh, seed=seed)
    pts = O.fast(A, 20, True)[:n, :2]
    assert len(pts) == n
    ga, gb = ctx.image(A, ml + 1), ctx.image(B, ml + 1)
    crit = (3, 50, 1e-3)
    gn, gs, ge = ctx.calc_optical_flow_pyr_lk(ga, gb, pts, win_size=(21, 21), max_level=ml, criteria=crit,
                                              flags=S.LK_GET_MIN_EIGENVALS)
    rn, rs, re_, it = O.lk(A, B, pts, (21, 21), ml, crit, O.LK_GET_MIN_EIGENVALS, acc=O.ACC_EXACT)
    assert ctx.lk_last_iterations() == int(it.sum())
    assert np.array_equal(gs, rs)
    assert np.array_equal(gn.view(np.uint32), rn.view(np.uint32))
    assert np.array_equal(ge.view(np.uint32), re_.view(np.uint32))
    sn, ss, _, _ = O.lk(A, B, pts, (21, 21), ml, crit, O.LK_GET_MIN_EIGENVALS, acc=O.ACC_SSE)
    ok = (gs == 1) & (ss == 1)
    assert np.abs(gn[ok] - sn[ok]).max() <= 0.1
    assert int((gs != ss).sum()) == 0
    assert gs.sum() > 0.99 * n


def test_lk_iteration_count_matches_oracle(ctx, lk_kernel):
    sc, A, B = frames(1241, 376, seed=0)
    pts = O.fast(A, 20, True)[:1000, :2]
    ga, gb = ctx.image(A, 4), ctx.image(B, 4)
    ctx.calc_optical_flow_pyr_lk(ga, gb, pts, win_size=(21, 21), max_level=3, criteria=(3, 50, 1e-3),
                                 flags=S.LK_GET_MIN_EIGENVALS)
    _, _, _, it = O.lk(A, B, pts, (21, 21), 3, (3, 50, 1e-3), O.LK_GET_MIN_EIGENVALS)
    assert ctx.lk_last_iterations() == int(it.sum())


def test_lk_borders_and_out_of_image(ctx, lk_kernel):
    sc, A, B = frames(320, 240, seed=4)
    rng = np.random.default_rng(0)
    pts = np.concatenate([
        rng.uniform(-40, 360, (400, 2)),                       # includes far outside
        np.array([[0, 0], [319, 239], [-21, 5], [5, -21], [-20.5, 3], [339.9, 120], [160, 259.5]]),
    ]).astype(np.float32)
    ga, gb = ctx.image(A, 4), ctx.image(B, 4)
    for cfg in (TEMPORAL, STEREO):
        gn, gs, ge = ctx.calc_optical_flow_pyr_lk(ga, gb, pts, win_size=cfg["win"], max_level=cfg["ml"],
                                                  criteria=cfg["crit"], flags=cfg["flags"])
        rn, rs, re_, _ = O.lk(A, B, pts, cfg["win"], cfg["ml"], cfg["crit"], cfg["flags"])
        assert np.array_equal(gs, rs)
        assert np.array_equal(gn.view(np.uint32), rn.view(np.uint32))
        assert np.array_equal(ge.view(np.uint32), re_.view(np.uint32))


@pytest.mark.parametrize("wh", [(321, 241), (322, 187), (323, 99), (324, 130), (45, 37)])
def test_lk_border_padding_widths(ctx, wh):
    """Levels are stored with REFLECT_101 borders written dword-wise (DESIGN.md
    §4): every width mod 4 and tiny levels, points hugging all four edges."""
    w, h = wh
    sc, A, B = frames(w, h, seed=w)
    rng = np.random.default_rng(w)
    edge = np.concatenate([
        np.c_[rng.uniform(-22, 12, 60), rng.uniform(0, h, 60)],
        np.c_[rng.uniform(w - 12, w + 22, 60), rng.uniform(0, h, 60)],
        np.c_[rng.uniform(0, w, 60), rng.uniform(-22, 12, 60)],
        np.c_[rng.uniform(0, w, 60), rng.uniform(h - 12, h + 22, 60)],
    ]).astype(np.float32)
    ga, gb = ctx.image(A, 4), ctx.image(B, 4)
    gn, gs, ge = ctx.calc_optical_flow_pyr_lk(ga, gb, edge, **{k: v for k, v in zip(
        ("win_size", "max_level", "criteria", "flags"), TEMPORAL.values())})
    rn, rs, re_, _ = O.lk(A, B, edge, *TEMPORAL.values())
    assert np.array_equal(gs, rs)
    assert np.array_equal(gn.view(np.uint32), rn.view(np.uint32))
    assert np.array_equal(ge.view(np.uint32), re_.view(np.uint32))


def test_lk_initial_flow_and_criteria(ctx):
    sc, A, B = frames(640, 376, seed=6)
    pts = O.fast(A, 20, True)[:500, :2]
    guess = pts + np.float32(1.0)
    ga, gb = ctx.image(A, 4), ctx.image(B, 4)
    for crit in [(1, 5, 0.0), (2, 0, 0.5), (3, 200, 1e-6), (3, 10, 20.0)]:
        for flags in (S.LK_USE_INITIAL_FLOW, S.LK_USE_INITIAL_FLOW | S.LK_GET_MIN_EIGENVALS):
            gn, gs, ge = ctx.calc_optical_flow_pyr_lk(ga, gb, pts, next_pts=guess, win_size=(15, 9), max_level=2,
                                                      criteria=crit, flags=flags, min_eig_threshold=1e-3)
            rn, rs, re_, _ = O.lk(A, B, pts, (15, 9), 2, crit, flags, 1e-3, next_pts=guess)
            assert np.array_equal(gs, rs)
            assert np.array_equal(gn.view(np.uint32), rn.view(np.uint32))
            assert np.array_equal(ge.view(np.uint32), re_.view(np.uint32))


def test_lk_small_image_clamps_levels(ctx):
    sc, A, B = frames(64, 48, seed=7)
    pts = O.fast(A, 10, True)[:50, :2]
    ga, gb = ctx.image(A, 5), ctx.image(B, 5)
    gn, gs, ge = ctx.calc_optical_flow_pyr_lk(ga, gb, pts, win_size=(21, 21), max_level=5, criteria=(3, 30, 0.01))
    rn, rs, re_, _ = O.lk(A, B, pts, (21, 21), 5, (3, 30, 0.01), 0)
    assert np.array_equal(gs, rs)
    assert np.array_equal(gn.view(np.uint32), rn.view(np.uint32))


def test_lk_empty_and_bad_args(ctx):
    sc, A, B = frames(64, 48)
    ga, gb = ctx.image(A, 2), ctx.image(B, 2)
    n, s, e = ctx.calc_optical_flow_pyr_lk(ga, gb, np.zeros((0, 2), np.float32))
    assert len(n) == 0
    with pytest.raises(S.SvoError):
        ctx.calc_optical_flow_pyr_lk(ga, gb, np.ones((3, 2), np.float32), win_size=(2, 2))
    with pytest.raises(S.SvoError):
        ctx.calc_optical_flow_pyr_lk(ga, gb, np.ones((3, 2), np.float32), max_level=-1)


# ------------------------------------------------------------------ PnP
def _pnp_problem(n=2000, seed=0, outlier_frac=0.1):
    sc = Scene(1241, 376, seed=seed)
    rng = np.random.default_rng(seed)
    pts0 = np.c_[rng.uniform(20, 1220, n), rng.uniform(20, 356, n)]
    X = sc.map_points(pts0, 0)
    uv = sc.project(X, 3) + rng.normal(0, 0.3, (n, 2))
    out = rng.random(n) < outlier_frac
    uv[out] += rng.uniform(60, 200, (out.sum(), 2)) * rng.choice([-1, 1], (out.sum(), 2))
    return sc, X, uv.astype(np.float32), out


def test_pnp_residuals_bit_exact(ctx):
    sc, X, uv, _ = _pnp_problem()
    rng = np.random.default_rng(1)
    hyps = []
    for _ in range(100):
        rv = rng.normal(0, 0.01, 3)
        R = O.rodrigues(rv)
        t = rng.normal(0, 0.05, 3)
        hyps.append(np.r_[R.ravel(), t])
    hyps = np.array(hyps)
    ge, gm, gc = ctx.pnp_residuals(X, uv, hyps, sc.K, 64.0)
    re_, rm, rc = O.pnp_residuals(X, uv, hyps, sc.K, 64.0)
    assert np.array_equal(ge.view(np.uint32), re_.view(np.uint32))
    assert np.array_equal(gm, rm)
    assert np.array_equal(gc, rc)


def test_pnp_ransac_inliers_identical(ctx):
    for seed in range(3):
        sc, X, uv, out = _pnp_problem(seed=seed)
        ok, rv, tv, inl = ctx.solve_pnp_ransac(X, uv, sc.K)
        rc, rv_o, tv_o, inl_o, _ = O.solve_pnp_ransac(X, uv, sc.K)
        assert ok and rc == 1
        assert np.array_equal(inl, inl_o)
        assert not np.isin(np.nonzero(out)[0], inl).any()
        np.testing.assert_allclose(rv, rv_o, atol=1e-7)
        np.testing.assert_allclose(tv, tv_o, atol=1e-6)
        # the recovered pose is the true one (pure rotation, t = 0)
        Rt = sc.R(3)
        np.testing.assert_allclose(O.rodrigues(rv), Rt, atol=2e-3)


def test_pnp_ransac_near_threshold(ctx):
    """30 % of the points sit at reprojection error within +-0.5 px^2 of the 8 px
    threshold (64 px^2) under the true pose, so every hypothesis splits them near
    the boundary: any last-bit difference between the product's EPnP (OpenCV's
    Jacobi SVDs in SIMD lanes, epnp_lanes.hpp) and the oracle's (oracle/epnp.c +
    cvsvd.c), or between the two residual computations, would show as a flipped
    inlier here. The EPnP models are bit-identical (test_epnp_cpu.py), so 0 flips
    are required, not merely observed."""
    flips = 0
    for seed in range(4):
        sc = Scene(1241, 376, seed=seed)
        rng = np.random.default_rng(100 + seed)
        n = 2000
        pts0 = np.c_[rng.uniform(20, 1220, n), rng.uniform(20, 356, n)]
        X = sc.map_points(pts0, 0)
        uv = sc.project(X, 3)
        near = rng.random(n) < 0.3
        r = np.sqrt(64.0 + rng.uniform(-0.5, 0.5, near.sum()))
        a = rng.uniform(0, 2 * np.pi, near.sum())
        uv[near] += np.c_[r * np.cos(a), r * np.sin(a)]
        uv = uv.astype(np.float32)
        ok, rv, tv, inl = ctx.solve_pnp_ransac(X, uv, sc.K)
        rc, rv_o, tv_o, inl_o, _ = O.solve_pnp_ransac(X, uv, sc.K)
        assert ok and rc == 1
        flips += np.setxor1d(inl, inl_o).size
        # every clean point is an inlier, and the near-threshold ones split
        assert np.isin(np.nonzero(~near)[0], inl_o).all()
        k = np.isin(np.nonzero(near)[0], inl_o).mean()
        assert 0.2 < k < 0.8
        np.testing.assert_allclose(rv, rv_o, atol=1e-7)
        np.testing.assert_allclose(tv, tv_o, atol=1e-6)
    print(f"near-threshold inlier flips product vs oracle: {flips}")
    assert flips == 0


def _reproj(R, t, sub, K):
    X = sub[:15].reshape(5, 3).astype(np.float64)
    Y = X @ R.T + t
    p = (Y[:, :2] / Y[:, 2:]) * [K[0, 0], K[1, 1]] + [K[0, 2], K[1, 2]]
    return float(np.sqrt(((p - sub[15:].reshape(5, 2)) ** 2).sum(1)).mean())


def test_epnp_wave_matches_host(ctx):
    """The QL-based EPnP run one 64-lane wave per subset on the GPU (epnp_wave.hpp,
    off the front end's path) vs its host twin (epnp_ql.hpp, device = 2):
    bit-identical R / t on 5-point subsets of the RANSAC test problems (clean,
    with outliers, and the near-threshold set). The front end's own solver
    (device = 0) is bit-identical to the oracle's (tests/test_epnp_cpu.py)."""
    rng = np.random.default_rng(5)
    subs, clean = [], []
    for seed in range(3):
        sc, X, uv, out = _pnp_problem(seed=seed)
        for _ in range(200):
            idx = rng.choice(len(X), 5, replace=False)
            clean.append(not out[idx].any())
            subs.append(np.r_[X[idx].astype(np.float32).ravel(), uv[idx].astype(np.float32).ravel()])
    subs = np.array(subs, np.float32)
    K = Scene(1241, 376, seed=0).K
    Rd, okd = ctx.epnp_subsets(subs, K, device=True)
    Rh, okh = ctx.epnp_subsets(subs, K, device=2)
    assert okh.sum() == len(subs)
    assert np.array_equal(okd, okh)
    assert np.array_equal(Rd.view(np.uint64), Rh.view(np.uint64))
    # ... and against the oracle's independent EPnP (calib3d/src/epnp.cpp restated
    # with a Jacobi eigen-solver, oracle/pnp.c). With 5 points M^T M has a 2-D null
    # space whose basis is arbitrary (OpenCV's own comes out of its Jacobi SVD), and
    # the beta approximations depend on it: on subsets of inliers (no outlier among
    # the 5) the models agree to noise level except where one basis sends all three
    # approximations astray; subsets with an outlier have no right answer.
    clean_ok = clean_n = worse = 0
    for k in range(len(subs)):
        if not clean[k]:
            continue
        rc, Ro, to = O.epnp(subs[k, :15].reshape(5, 3), subs[k, 15:].reshape(5, 2), K)
        assert rc == 0
        clean_n += 1
        clean_ok += np.abs(Rd[k, :9].reshape(3, 3) - Ro).max() < 1e-2
        worse += _reproj(Rd[k, :9].reshape(3, 3), Rd[k, 9:], subs[k], K) > 8 * max(1.0, _reproj(Ro, to, subs[k], K))
    print(f"device EPnP vs oracle EPnP on {clean_n} inlier-only subsets: {clean_ok} within 1e-2 rad, "
          f"{worse} where the device model reprojects > 8x worse")
    assert clean_ok >= 0.97 * clean_n and worse <= 0.02 * clean_n


def test_pnp_ransac_too_few_points(ctx):
    with pytest.raises(S.SvoError):
        ctx.solve_pnp_ransac(np.zeros((3, 3)), np.zeros((3, 2), np.float32), np.eye(3))


def test_lk_negative_bilinear_weight_case(ctx, lk_kernel):
    """OpenCV's rounded weights can make iw11 = 2^14 - iw00 - iw01 - iw10 = -1
    (fractional offsets (0.00706080, 0.00132304) or (0.0000501, 0.2830146)):
    the fixed-point dot products must be signed."""
    sc, A, B = frames(640, 376, seed=3)
    base = np.floor(O.fast(A, 20, True)[:300, :2])
    fr = np.array([[0.0070608025416731834, 0.0013230398762971163], [5.0094684411305934e-05, 0.28301456570625305]],
                  np.float32)
    pts = np.concatenate([base + fr[0], base + fr[1]]).astype(np.float32)
    guess = (pts + np.float32(1.0)).astype(np.float32)   # same fractions at the first J sample
    ga, gb = ctx.image(A, 4), ctx.image(B, 4)
    for cfg in (TEMPORAL, STEREO):
        for ml, flags, nxt in ((cfg["ml"], cfg["flags"], None), (0, cfg["flags"] | S.LK_USE_INITIAL_FLOW, guess)):
            gn, gs, ge = ctx.calc_optical_flow_pyr_lk(ga, gb, pts, next_pts=nxt, win_size=cfg["win"], max_level=ml,
                                                      criteria=cfg["crit"], flags=flags)
            rn, rs, re_, _ = O.lk(A, B, pts, cfg["win"], ml, cfg["crit"], flags, next_pts=nxt)
            assert np.array_equal(gs, rs)
            assert np.array_equal(gn.view(np.uint32), rn.view(np.uint32))
            assert np.array_equal(ge.view(np.uint32), re_.view(np.uint32))


# ------------------------------------------------------------------ committed golden fixtures
def test_gpu_matches_committed_golden(ctx):
    import os
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "small_160x120.npz"))
    A, B = g["A"], g["B"]
    ga, gb = ctx.image(A, 4), ctx.image(B, 4)
    for l in range(1, 4):
        if f"pyr{l}" in g:
            assert np.array_equal(ga.level(l), g[f"pyr{l}"])
    assert np.array_equal(ctx.fast_detect(ga, 20, True), g["kp_nms"])
    assert np.array_equal(ctx.fast_detect(ga, 20, False), g["kp_all"])
    assert np.array_equal(ctx.fast_detect(ga, 20, True, g["mask"]), g["kp_mask"])
    n, s, e = ctx.calc_optical_flow_pyr_lk(ga, gb, g["pts"], win_size=(21, 21), max_level=3,
                                          criteria=(3, 50, 1e-3), flags=S.LK_GET_MIN_EIGENVALS)
    assert np.array_equal(n, g["t_next"]) and np.array_equal(s, g["t_status"]) and np.array_equal(e, g["t_err"])
    n, s, e = ctx.calc_optical_flow_pyr_lk(ga, gb, g["pts"], win_size=(11, 11), max_level=3,
                                          criteria=(3, 30, 1e-3), flags=0)
    assert np.array_equal(n, g["s_next"]) and np.array_equal(s, g["s_status"]) and np.array_equal(e, g["s_err"])
    bx, _ = ctx.bucket_features(g["kp_all"][:, :2], 160, 120, 50, 2)
    assert np.array_equal(bx, g["bucket_xy"])
    ok, rv, tv, inl = ctx.solve_pnp_ransac(g["X"], g["t_next"], g["K"])
    assert ok and np.array_equal(inl, g["pnp_inliers"])
    assert np.allclose(rv, g["pnp_rvec"], atol=1e-7) and np.allclose(tv, g["pnp_tvec"], atol=1e-6)


@pytest.mark.parametrize("win", [(15, 15), (31, 31)])
def test_lk_other_fixed_windows(ctx, win, lk_kernel):
    sc, A, B = frames(640, 480, seed=9)
    pts = O.fast(A, 20, True)[:800, :2]
    ga, gb = ctx.image(A, 4), ctx.image(B, 4)
    for flags in (0, S.LK_GET_MIN_EIGENVALS):
        gn, gs, ge = ctx.calc_optical_flow_pyr_lk(ga, gb, pts, win_size=win, max_level=3, criteria=(3, 30, 1e-3),
                                                  flags=flags)
        rn, rs, re_, _ = O.lk(A, B, pts, win, 3, (3, 30, 1e-3), flags)
        assert np.array_equal(gs, rs)
        assert np.array_equal(gn.view(np.uint32), rn.view(np.uint32))
        assert np.array_equal(ge.view(np.uint32), re_.view(np.uint32))
