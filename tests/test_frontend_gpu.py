"""Batched device-resident frontend vs the oracle-composed reference loop
(tests/oracle_loop.py): identical feature lists (bit-exact positions), identical
inlier counts, pose equal to the oracle's, and per-sequence results independent
of the batch they run in."""
import numpy as np
import pytest

import oracle as O
import svo_amd as S
from oracle_loop import OracleLoop
from svo_amd.scene import Scene

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["streamed", "after-lk"])
def post_lk_mode(request, monkeypatch):
    """Both post-LK schedules (read when a Frontend is created): the default
    streamed hand-off (post_lk waits on the device for each sequence's LK
    records) and SVO_FE_STREAM=0 (post_lk queued after LK)."""
    monkeypatch.setenv("SVO_FE_STREAM", "1" if request.param == "streamed" else "0")
    return request.param


def make_frontend(ctx, scenes, T, n_features, **kw):
    sc0 = scenes[0]
    cfg = S.FrontendConfig(sc0.w, sc0.h, sc0.K, n_seq=len(scenes), n_frames=T, n_features=n_features, **kw)
    fe = S.Frontend(ctx, cfg)
    for s, sc in enumerate(scenes):
        for t in range(T):
            fe.set_frame(s, t, sc.frame(t), sc.R(t), depth_seed=sc.seed)
    return fe


@pytest.mark.parametrize("bucket", [(0, 0), (50, 4)])
def test_frontend_matches_oracle_loop(bucket):
    ctx = S.Context(0)
    W, H, N, T = 640, 376, 800, 6
    sc = Scene(W, H, seed=3)
    fe = make_frontend(ctx, [sc], T, N, bucket_size=bucket[0], per_bucket=bucket[1])
    fe.init(0)
    ref = OracleLoop(Scene(W, H, seed=3), N, bucket=bucket, depth_seed=3).init(0)
    assert np.array_equal(fe.features(0), ref.pts)
    for t in range(1, T):
        st = fe.step(t).as_dict()
        rs = ref.step(t)
        assert st["tracked"] == rs["tracked"], t
        assert st["lk_iterations"] == rs["lk_iterations"], t
        assert st["inliers"] == rs["inliers"], t
        assert st["added"] == rs["added"], t
        got = fe.features(0)
        assert np.array_equal(got, ref.pts), f"features differ at t={t}"
        rv, tv = fe.pose(0)
        np.testing.assert_allclose(rv, ref.pose[0], atol=1e-6)
        np.testing.assert_allclose(tv, ref.pose[1], atol=1e-5)
        np.testing.assert_allclose(O.rodrigues(rv), sc.R(t), atol=3e-3)


@pytest.mark.parametrize("groups", [1, 2, 3])
def test_frontend_batch_independence(groups):
    """A sequence's result does not depend on the batch it runs in, nor on the
    pipeline slicing of the batch (slices overlap LK and host RANSAC)."""
    ctx = S.Context(0)
    W, H, N, T = 1241, 376, 2000, 4
    scenes = [Scene(W, H, seed=s) for s in range(3)]
    feb = make_frontend(ctx, scenes, T, N, groups=groups)
    feb.init(0)
    solo = [make_frontend(ctx, [sc], T, N) for sc in scenes]
    for f in solo:
        f.init(0)
    for t in range(1, T):
        feb.step(t)
        for s, f in enumerate(solo):
            f.step(t)
            assert np.array_equal(feb.features(s), f.features(0))
            assert np.array_equal(np.r_[feb.pose(s)], np.r_[f.pose(0)])


def test_frontend_kitti_sequence_keeps_2000_features():
    ctx = S.Context(0)
    W, H, N, T = 1241, 376, 2000, 12
    sc = Scene(W, H, seed=0)
    fe = make_frontend(ctx, [sc], T, N, timing=1)
    fe.init(0)
    for t in range(1, T):
        st = fe.step(t).as_dict()
        assert st["features"] == N
        assert st["tracked"] > 0.9 * N
        assert st["inliers"] > 0.9 * st["tracked"]
        rv, tv = fe.pose(0)
        np.testing.assert_allclose(O.rodrigues(rv), sc.R(t), atol=3e-3)
        assert np.abs(tv).max() < 0.05
    pt = fe.phase_times()
    assert pt["lk"][1] == T - 1 and pt["lk"][0] > 0
