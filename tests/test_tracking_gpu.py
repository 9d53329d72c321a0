"""The host Tracking mirror (include/svo/tracking.hpp, libsvo_tracking.so) on the
GPU, checked stage by stage against the oracle: every frame's trace (what
trackFrames / calculatePose / extractFeatures / findLeftFeaturesInRight /
triangulateNewMapPoints consumed and produced, R:src/tracking.cpp:74-230) is
replayed through the CPU restatement on the same inputs.

Bars: LK points/status, FAST keypoints, stereo LK, PnP inlier sets bit-identical;
the mirror's two LK calls sum in OpenCV's own float order (SVO_LK_OPENCV_ORDER),
so they are held to the oracle's ACC_SSE restatement of that order;
triangulated points within 1e-5 relative (float DLT; OpenCV's SVD is not
restated bit for bit); poses to 1e-7.
"""
import numpy as np
import pytest

import oracle as O
import svo_amd as S
from svo_amd.scene import Scene
from svo_amd.tracking import Tracking

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    return S.Context(0)


def rodrigues(rv):
    return O.rodrigues(np.asarray(rv, np.float64))


def test_triangulate_matches_oracle_and_truth(ctx):
    sc = Scene(1241, 376, seed=21)
    L, R = sc.frame(0), sc.right(0)
    kp = O.fast(L, 20, True)[:, :2]
    nx, st, _, _ = O.lk(L, R, kp, (11, 11), 3, (3, 30, 1e-3), 0)
    ok = (st == 1) & (np.abs(nx[:, 1] - kp[:, 1]) < 40)
    P0, P1 = sc.projections()
    gh, gx = ctx.triangulate_points(P0, P1, kp[ok], nx[ok])
    oh, ox = O.triangulate(P0, P1, kp[ok], nx[ok])
    assert np.allclose(gh, oh, rtol=0, atol=2e-7)
    assert np.allclose(gx, ox, rtol=1e-5, atol=1e-5)
    truth = sc.map_points(kp[ok], 0)
    rel = np.abs(gx - truth).max(1) / truth[:, 2]
    assert np.median(rel) < 0.02
    # empty input and mismatched arguments
    h0, x0 = ctx.triangulate_points(P0, P1, np.zeros((0, 2)), np.zeros((0, 2)))
    assert h0.shape == (0, 4) and x0.shape == (0, 3)


def _colour(g, t):
    """A BGR frame built around a grey frame (the channels differ, so the device
    conversion's weights matter); the test's grey frame is the oracle's conversion."""
    b = g
    gg = np.roll(g, 1, axis=1)  # same for every frame: the scene's motion is unchanged
    r = 255 - g
    return np.ascontiguousarray(np.stack([b, gg, r], axis=2))


@pytest.mark.parametrize("detector,features_to_track,colour", [
    ("fast", 70, False), ("fast", 1 << 30, False), ("orb", 70, False), ("orb", 1 << 30, True)])
def test_tracking_mirror_stagewise_parity(detector, features_to_track, colour):
    """70 = the reference config (keyframe only at frame 0 here for FAST); 2^30 makes
    every other frame a keyframe (R:src/tracking.cpp:68-69), exercising the
    detect/stereo/triangulate path mid-sequence. "orb" is the detector the reference
    ships (use_orb: 1, 150 features: keyframes recur as tracks are lost); colour
    frames go through the device BGR->grey ingest (R:include/async_image_loader.h:68-69)."""
    sc = Scene(1241, 376, seed=33)
    P0, P1 = sc.projections()
    K = sc.K
    tr = Tracking(np.r_[P0.ravel(), P1.ravel()], features_to_track=features_to_track, use_orb=detector == "orb")
    T = 6
    if colour:
        bgr = [(_colour(sc.frame(t), t), _colour(sc.right(t), t)) for t in range(T)]
        frames = [(O.bgr2gray(a), O.bgr2gray(b)) for a, b in bgr]
    else:
        frames = [(sc.frame(t), sc.right(t)) for t in range(T)]
    prev_xy = None
    n_kf = 0
    for t in range(T):
        L, Rimg = frames[t]
        if colour:
            tr.push_bgr(*bgr[t])
        else:
            tr.push(L, Rimg)
        assert tr.step()
        info = tr.frame_info()
        assert info["id"] == t
        xy, world, ids = tr.features()
        assert len(xy) == info["features"]
        keep_tracked = np.zeros((0, 2), np.float32)
        if t > 0:
            lk_prev, lk_next, st = tr.trace("lk_prev"), tr.trace("lk_next"), tr.trace("lk_status")
            assert np.array_equal(lk_prev, prev_xy)
            on, ost, _, _ = O.lk(frames[t - 1][0], L, lk_prev, (21, 21), 3, (3, 50, 1e-3),
                                 O.LK_GET_MIN_EIGENVALS, acc=O.ACC_SSE, want_err=False)
            assert np.array_equal(st, ost)
            assert np.array_equal(lk_next[st == 1].view(np.uint32), on[ost == 1].view(np.uint32))
            obj, img = tr.trace("pnp_obj"), tr.trace("pnp_img")
            assert np.array_equal(img, lk_next[st == 1])
            inl = tr.trace("pnp_inliers")
            pp = tr.trace("pnp_pose")
            rc, rv, tv, oinl, _ = O.solve_pnp_ransac(obj, img, K)
            assert int(pp[6]) == rc == 1
            assert np.array_equal(inl, np.flatnonzero(oinl) if oinl.dtype == bool else oinl)
            assert np.allclose(pp[:3], rv, atol=1e-7) and np.allclose(pp[3:6], tv, atol=1e-6)
            # frame pose = inverse([R|t]) (R:src/tracking.cpp:198-214)
            Rm = rodrigues(pp[:3])
            assert np.allclose(info["R"], Rm.T, atol=1e-12)
            assert np.allclose(info["t"], -Rm.T @ pp[3:6], atol=1e-12)
            # against the synthetic truth: camera->world rotation R(t)^T, no translation
            dR = info["R"] @ sc.R(t)
            ang = np.degrees(np.arccos(np.clip((np.trace(dR) - 1) / 2, -1, 1)))
            assert ang < 0.5 and np.linalg.norm(info["t"]) < 0.2
            keep_tracked = img[inl]
            assert np.array_equal(xy[:len(keep_tracked)], keep_tracked)
        if t == 0 or info["keyframe"]:
            n_kf += 1
            mask_pts, kps = tr.trace("mask_pts"), tr.trace("kps")
            assert np.array_equal(mask_pts, prev_xy if t > 0 else np.zeros((0, 2), np.float32))
            mask = O.mask_boxes(L.shape[1], L.shape[0], mask_pts, 10.0) if t > 0 else None
            if detector == "orb":
                okp = O.orb_detect(L, mask)[0][:, :2]
            else:
                okp = O.fast(L, 20, True, mask)[:, :2]
            assert np.array_equal(kps, okp)
            sr, ss = tr.trace("stereo_right"), tr.trace("stereo_status")
            on, ost, _, _ = O.lk(L, Rimg, kps, (11, 11), 3, (3, 30, 1e-3), 0, acc=O.ACC_SSE)
            assert np.array_equal(ss, ost) and np.array_equal(sr.view(np.uint32), on.view(np.uint32))
            kept = (ss == 1) & (np.abs(sr[:, 1] - kps[:, 1]) < 40)
            kl, kr = tr.trace("kept_left"), tr.trace("kept_right")
            assert np.array_equal(kl, kps[kept]) and np.array_equal(kr, sr[kept])
            tri = tr.trace("tri_xyz")
            _, ox = O.triangulate(P0, P1, kl, kr)
            assert np.allclose(tri, ox, rtol=1e-5, atol=1e-5)
            pos = tri[:, 2] > 0
            new_xy = xy[len(keep_tracked):]
            assert np.array_equal(new_xy, kl[pos])
            # new map points = frame pose * camera point (R:src/tracking.cpp:137)
            Xw = (info["R"] @ tri[pos].astype(np.float64).T).T + info["t"]
            assert np.allclose(world[len(keep_tracked):], Xw, rtol=1e-12, atol=1e-9)
        else:
            assert len(xy) == len(keep_tracked)
        prev_xy = xy
    if detector == "fast":
        assert n_kf == (1 if features_to_track == 70 else 3)
    else:
        assert n_kf >= (1 if features_to_track == 70 else 3)
    tr.close()


def test_tracking_mirror_too_few_points_raises():
    """calculatePose with < 4 points: OpenCV's CV_Assert throws; the mirror raises."""
    sc = Scene(320, 240, seed=2)
    P0, P1 = sc.projections()
    tr = Tracking(np.r_[P0.ravel(), P1.ravel()])
    flat = np.full((240, 320), 128, np.uint8)        # no FAST corners at all
    tr.push(flat, flat)
    assert tr.step()
    assert tr.frame_info()["features"] == 0
    tr.push(flat, flat)
    with pytest.raises(S.SvoError):
        tr.step()
    tr.close()
