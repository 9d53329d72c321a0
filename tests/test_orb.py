"""ORB detection: the reference's shipped default detector,
cv::ORB(150, 1.2, 8, 31, 0, 4, HARRIS, 31, 20)::detect (R:configs/config.yaml:20-27,
R:src/tracking.cpp:33-50,82).

CPU: known answers for the oracle's pieces -- the INTER_LINEAR_EXACT resize (a 2x
reduction is the rounded 2x2 mean, constants stay constant, a linear ramp stays a
ramp), ORB's level schedule for the KITTI size (sizes, float scales, features per
level), and properties of the oracle's detection (every keypoint is a FAST corner
of its level, inside the edge, outside the mask, at most the level's quota plus
ties). GPU: svo_orb_detect is identical to the oracle -- same keypoints in the
same order with the same response and octave -- with and without masks, for
Harris and FAST scoring, on the KITTI size and ragged sizes.
"""
import numpy as np
import pytest

import oracle as O
from svo_amd.scene import Scene


# ------------------------------------------------------------------ CPU (oracle)
def test_kat_resize_half_is_rounded_box_mean():
    rng = np.random.default_rng(0)
    a = rng.integers(0, 256, (30, 42), dtype=np.uint8)
    got = O.resize_linear_exact(a, 21, 15).astype(int)
    s = a.reshape(15, 2, 21, 2).astype(int).sum(axis=(1, 3))
    assert np.array_equal(got, (s + 2) >> 2)


@pytest.mark.parametrize("dst", [(1034, 313), (346, 105), (17, 9), (1, 1)])
def test_kat_resize_constant_and_ramp(dst):
    c = np.full((376, 1241), 77, np.uint8)
    assert (O.resize_linear_exact(c, *dst) == 77).all()
    # a horizontal ramp in a range where rounding cannot saturate stays monotone and
    # within half a step of the sampled position (analytic bilinear value)
    w, h = 241, 40
    ramp = np.tile(np.arange(w, dtype=np.uint8), (h, 1))
    dw = max(dst[0] // 5, 1)
    r = O.resize_linear_exact(ramp, dw, 10).astype(float)
    pos = np.clip((np.arange(dw) + 0.5) * (w / dw) - 0.5, 0, w - 1)
    assert np.abs(r[0] - pos).max() <= 0.5 + 1 / 256
    assert (np.diff(r[0]) >= 0).all()


def test_kat_orb_level_schedule_kitti():
    lw, lh, ls, nper = O.orb_level_info(1241, 376, 1.2, 8, 150)
    assert lw.tolist() == [1241, 1034, 862, 718, 598, 499, 416, 346]
    assert lh.tolist() == [376, 313, 261, 218, 181, 151, 126, 105]
    assert nper.tolist() == [33, 27, 23, 19, 16, 13, 11, 8] and nper.sum() == 150
    assert np.float32(ls[1]) == np.float32(1.2000000476837158) and ls[0] == 1.0
    # OpenCV's default nfeatures = 500
    assert O.orb_level_info(1241, 376, 1.2, 8, 500)[3].tolist() == [109, 90, 75, 63, 52, 44, 36, 31]


def _boxes_mask(w, h, pts, half=10.0):
    return O.mask_boxes(w, h, np.asarray(pts, np.float32), half)


def test_oracle_orb_properties():
    sc = Scene(640, 360, seed=2)
    img = sc.frame(0)
    rng = np.random.default_rng(1)
    pts = np.stack([rng.uniform(0, 640, 200), rng.uniform(0, 360, 200)], 1).astype(np.float32)
    mask = _boxes_mask(640, 360, pts)
    kp, octv = O.orb_detect(img, mask)
    lw, lh, ls, nper = O.orb_level_info(640, 360, 1.2, 8, 150)
    assert len(kp) >= 100
    # level order, quota (+ ties at the boundary response)
    assert (np.diff(octv) >= 0).all()
    counts = np.bincount(octv, minlength=8)
    resp_by_level = [kp[octv == l, 2] for l in range(8)]
    for l in range(8):
        if counts[l] > nper[l]:
            r = np.sort(resp_by_level[l])[::-1]
            assert (r[nper[l] - 1:] == r[nper[l] - 1]).all()
    # every keypoint: a FAST corner of its level, inside the edge, mask 255 there
    lv = [img]
    mk = [mask]
    for l in range(1, 8):
        lv.append(O.resize_linear_exact(lv[-1], lw[l], lh[l]))
        m = O.resize_linear_exact(mk[-1], lw[l], lh[l])
        mk.append(np.where(m > 254, m, 0).astype(np.uint8))
    for (x, y, r), l in zip(kp, octv):
        lx, ly = np.float32(x) / ls[l], np.float32(y) / ls[l]
        ix, iy = int(round(float(lx))), int(round(float(ly)))
        assert 31 <= ix < lw[l] - 31 and 31 <= iy < lh[l] - 31
        assert mk[l][iy, ix] == 255
    for l in range(8):
        f = O.fast(lv[l], 20, True, mk[l])
        fs = {(int(a), int(b)) for a, b, _ in f}
        sel = kp[octv == l]
        for x, y, _ in sel:
            assert (int(round(float(np.float32(x) / ls[l]))), int(round(float(np.float32(y) / ls[l])))) in fs


def test_oracle_orb_fast_score_mode_uses_fast_responses():
    sc = Scene(400, 300, seed=3)
    img = sc.frame(0)
    kp, octv = O.orb_detect(img, harris=False, nfeatures=200)
    f0 = O.fast(img, 20, True)
    lvl0 = kp[octv == 0]
    d = {(a, b): r for a, b, r in f0}
    assert all(d[(x, y)] == r for x, y, r in lvl0)


# ------------------------------------------------------------------ GPU parity
@pytest.fixture(scope="module")
def ctx():
    import svo_amd as S
    return S.Context(0)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["kitti", "kitti-mask", "ragged", "fast-score", "many", "small"])
def test_gpu_orb_matches_oracle(ctx, case):
    import svo_amd as S
    w, h, seed, nf, harris, use_mask = {
        "kitti": (1241, 376, 0, 150, True, False),
        "kitti-mask": (1241, 376, 1, 150, True, True),
        "ragged": (333, 217, 2, 150, True, True),
        "fast-score": (800, 450, 3, 300, False, True),
        "many": (1241, 376, 4, 2000, True, True),
        "small": (70, 70, 5, 50, True, False),
    }[case]
    img = Scene(w, h, seed=seed).frame(0)
    mask = None
    if use_mask:
        rng = np.random.default_rng(seed)
        n = 300
        pts = np.stack([rng.uniform(0, w, n), rng.uniform(0, h, n)], 1).astype(np.float32)
        mask = _boxes_mask(w, h, pts)
    ek, eo = O.orb_detect(img, mask, nfeatures=nf, harris=harris)
    g = ctx.image(img, max_levels=0)
    prm = S.OrbParams(nfeatures=nf, score_type=S.OrbParams.HARRIS if harris else S.OrbParams.FAST)
    gk, go = ctx.orb_detect(g, prm, mask)
    assert len(gk) == len(ek)
    assert np.array_equal(go, eo)
    assert np.array_equal(gk, ek)  # x, y, response bit for bit, same order


@pytest.mark.gpu
def test_gpu_orb_rejects_unsupported(ctx):
    import svo_amd as S
    g = ctx.image(np.zeros((64, 64), np.uint8), max_levels=0)
    p = S.OrbParams()
    p.first_level = 1
    with pytest.raises(S.SvoError):
        ctx.orb_detect(g, p)
    p = S.OrbParams(nlevels=9)
    with pytest.raises(S.SvoError):
        ctx.orb_detect(g, p)


# ------------------------------------------------------------------ committed fixture
def _fixture():
    import os
    return np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "orb_ingest_320x240.npz"))


def test_oracle_matches_committed_orb_ingest_fixture():
    g = _fixture()
    assert np.array_equal(O.bgr2gray(g["bgr"]), g["gray"])
    k, o = O.orb_detect(g["gray"], None, nfeatures=150)
    assert np.array_equal(k, g["orb150"]) and np.array_equal(o, g["oct150"])
    k, o = O.orb_detect(g["gray"], g["mask"], nfeatures=500)
    assert np.array_equal(k, g["orb500m"]) and np.array_equal(o, g["oct500m"])


@pytest.mark.gpu
def test_gpu_matches_committed_orb_ingest_fixture(ctx):
    import svo_amd as S
    g = _fixture()
    img = ctx.image_bgr(g["bgr"], max_levels=3)
    assert np.array_equal(img.level(0), g["gray"])
    k, o = ctx.orb_detect(img, S.OrbParams(nfeatures=150))
    assert np.array_equal(k, g["orb150"]) and np.array_equal(o, g["oct150"])
    k, o = ctx.orb_detect(img, S.OrbParams(nfeatures=500), g["mask"])
    assert np.array_equal(k, g["orb500m"]) and np.array_equal(o, g["oct500m"])
