"""Colour ingest: cv::cvtColor(COLOR_BGR2GRAY) of the reference's
loader (R:include/async_image_loader.h:63-69) fused into the level-0 upload.

CPU: the oracle against OpenCV's known grey values of pure colours (the fixed-point
weights 1868/9617/4899 >> 14 give blue 29, green 150, red 76, the values OpenCV
documents for its 8U conversion). GPU: svo_image_upload_bgr bit-exact with the
oracle (ragged widths, non-4-multiple rows), its pyramid equal to one built from the
grey image, and the batched front end's BGR frames equal to grey frames.
"""
import numpy as np
import pytest

import oracle as O


def test_kat_pure_colours():
    px = np.array([[[255, 0, 0], [0, 255, 0], [0, 0, 255], [255, 255, 255], [0, 0, 0], [1, 1, 1],
                    [128, 128, 128], [0, 128, 255]]], np.uint8)  # B, G, R
    got = O.bgr2gray(px)[0].tolist()
    exp = [29, 150, 76, 255, 0, 1, 128, (128 * 9617 + 255 * 4899 + 8192) >> 14]
    assert got == exp


def test_oracle_matches_float_weights_within_rounding():
    rng = np.random.default_rng(3)
    bgr = rng.integers(0, 256, (37, 53, 3), dtype=np.uint8)
    g = O.bgr2gray(bgr).astype(np.float64)
    f = bgr[..., 0] * 0.114 + bgr[..., 1] * 0.587 + bgr[..., 2] * 0.299
    assert np.abs(g - f).max() <= 1.0


@pytest.mark.gpu
@pytest.mark.parametrize("wh", [(1241, 376), (1, 1), (5, 3), (97, 33), (1920, 1080)])
def test_gpu_bgr_upload_bit_exact(wh):
    import svo_amd as S
    ctx = S.Context(0)
    w, h = wh
    rng = np.random.default_rng(w + 7 * h)
    bgr = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
    exp = O.bgr2gray(bgr)
    img = ctx.image_bgr(bgr, max_levels=3)
    assert np.array_equal(img.level(0), exp)
    ref = ctx.image(exp, max_levels=3)
    for l in range(1, 4):
        try:
            a = img.level(l)
        except S.SvoError:
            break
        assert np.array_equal(a, ref.level(l)), l
    # double buffering: back-to-back uploads into distinct images stay correct
    imgs = [ctx.image_bgr(np.roll(bgr, k, axis=1), max_levels=0) for k in range(4)]
    for k, im in enumerate(imgs):
        assert np.array_equal(im.level(0), O.bgr2gray(np.roll(bgr, k, axis=1)))


@pytest.mark.gpu
def test_gpu_frontend_bgr_frames_equal_grey_frames():
    import svo_amd as S
    from svo_amd.scene import Scene
    W, H = 320, 240
    sc = Scene(W, H, seed=4)
    ctx = S.Context(0)
    outs = []
    for colour in (False, True):
        cfg = S.FrontendConfig(W, H, sc.K, n_seq=1, n_frames=3, n_features=300, max_level=3)
        fe = S.Frontend(ctx, cfg)
        for t in range(3):
            g, gr = sc.frame(t), sc.right(t)
            if colour:
                # BGR frames whose conversion is exactly g: equal channels
                fe.set_frame(0, t, np.repeat(g[..., None], 3, axis=2), np.repeat(gr[..., None], 3, axis=2))
            else:
                fe.set_frame(0, t, g, gr)
        fe.init(0)
        fe.step(1)
        fe.step(2)
        fe.synchronize()
        outs.append((fe.features(0), fe.pose(0)))
        fe.close()
    assert np.array_equal(outs[0][0], outs[1][0])
    assert np.allclose(outs[0][1][0], outs[1][1][0]) and np.allclose(outs[0][1][1], outs[1][1][1])
