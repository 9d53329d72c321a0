"""Parity of the batched front end on the exact workloads bench.py reports
(BASELINE.json configs[1..3]): the 128-sequence KITTI batch, 1920x1080 / 8000
features / maxLevel 4 and 3840x2160 / 16000 features / maxLevel 3, each step
against the reference loop composed from oracle calls (tests/oracle_loop.py:
trackFrames R:src/tracking.cpp:154-179, calculatePose :191-196, extractFeatures
:74-92, findLeftFeaturesInRight :94-118, triangulateNewMapPoints :120-152), plus
the derivative pyramid the 1080p launch builds (all 5 levels)."""
import numpy as np
import pytest

import bench
import oracle as O
import svo_amd as S
from oracle_loop import OracleLoop
from svo_amd.scene import Scene

pytestmark = pytest.mark.gpu


def _frontend(ctx, scenes, T, n_features, max_level, timing=2):
    sc0 = scenes[0]
    cfg = S.FrontendConfig(sc0.w, sc0.h, sc0.K, n_seq=len(scenes), n_frames=T, n_features=n_features,
                           max_level=max_level, timing=timing)
    fe = S.Frontend(ctx, cfg)
    for s, sc in enumerate(scenes):
        for t in range(T):
            fe.set_frame(s, t, sc.frame(t), sc.right(t))
    return fe


def test_bench_kitti_128_sequences_match_oracle_and_solo():
    """bench.py's default launch: 128 KITTI-size sequences (its own seeds), 2000
    features, maxLevel 3. Eight sampled sequences against their own oracle loop at
    every step (feature lists bit-exact, poses 1e-7, map points 2e-5); all 128
    against the same sequence run alone (bitwise: a sequence's result does not
    depend on the 127 others it shares every launch with); the batch-wide counts
    equal the sum of the solo runs'."""
    W, H, N, ML, _ = bench.CONFIGS["kitti"]
    ctx = S.Context(0)
    T = 4
    n_seq = 128  # bench.py's default --seq
    seeds = bench.sequence_seeds(0, n_seq)
    scenes = [Scene(W, H, seed=sd) for sd in seeds]
    fe = _frontend(ctx, scenes, T, N, ML)
    fe.init(0)
    sample = [0, 17, 42, 63, 64, 85, 110, 127]
    refs = {s: OracleLoop(Scene(W, H, seed=seeds[s]), N, max_level=ML).init(0) for s in sample}
    for s in sample:
        assert np.array_equal(fe.features(s), refs[s].pts)
    batch_stats = []
    for t in range(1, T):
        st = fe.step(t).as_dict()
        batch_stats.append(st)
        for s in sample:
            rs = refs[s].step(t)
            assert len(fe.features(s)) == rs["features"], f"seq {s} t={t}"
            assert np.array_equal(fe.features(s), refs[s].pts), f"seq {s}: features differ at t={t}"
            rv, tv = fe.pose(s)
            np.testing.assert_allclose(rv, refs[s].pose[0], atol=1e-7)
            np.testing.assert_allclose(tv, refs[s].pose[1], atol=1e-6)
            np.testing.assert_allclose(fe.map_points(s), refs[s].X, rtol=2e-5, atol=1e-6)
    # every sequence of the batch against its solo run (same library, S = 1)
    final = [(fe.features(s), np.r_[fe.pose(s)], fe.map_points(s)) for s in range(n_seq)]
    fe.close()
    tot = {k: [0] * (T - 1) for k in ("tracked", "inliers", "added", "features", "lk_iterations")}
    for s, sc in enumerate(scenes):
        f1 = _frontend(ctx, [sc], T, N, ML, timing=0)
        f1.init(0)
        for t in range(1, T):
            st1 = f1.step(t).as_dict()
            for k in tot:
                tot[k][t - 1] += st1[k]
        assert np.array_equal(final[s][0], f1.features(0)), f"seq {s}: batch vs solo features"
        assert np.array_equal(final[s][1], np.r_[f1.pose(0)]), f"seq {s}: batch vs solo pose"
        assert np.array_equal(final[s][2], f1.map_points(0)), f"seq {s}: batch vs solo map points"
        f1.close()
    for t in range(1, T):
        for k in tot:
            assert batch_stats[t - 1][k] == tot[k][t - 1], f"batch {k} at t={t}"


@pytest.mark.parametrize("cfg,n_seq", [("1080p", 2), ("4k", 1)])
def test_bench_large_configs_match_oracle_loop(cfg, n_seq):
    """BASELINE configs[2] (1920x1080, 8000 features, maxLevel 4: a 5-level
    pyramid + Scharr chain, CAP 8000) and configs[3] (3840x2160, 16000 features,
    maxLevel 3) through the batched front end, every sequence against its oracle
    loop at every step."""
    W, H, N, ML, _ = bench.CONFIGS[cfg]
    ctx = S.Context(0)
    T = 4
    scenes = [Scene(W, H, seed=s + 1) for s in range(n_seq)]
    fe = _frontend(ctx, scenes, T, N, ML)
    fe.init(0)
    refs = [OracleLoop(Scene(W, H, seed=s + 1), N, max_level=ML).init(0) for s in range(n_seq)]
    for s in range(n_seq):
        assert np.array_equal(fe.features(s), refs[s].pts)
    for t in range(1, T):
        st = fe.step(t).as_dict()
        rss = [r.step(t) for r in refs]
        for k in ("tracked", "inliers", "added", "features", "lk_iterations"):
            assert st[k] == sum(rs[k] for rs in rss), f"{k} differs at t={t}"
        for s in range(n_seq):
            assert np.array_equal(fe.features(s), refs[s].pts), f"seq {s}: features differ at t={t}"
            rv, tv = fe.pose(s)
            np.testing.assert_allclose(rv, refs[s].pose[0], atol=1e-7)
            np.testing.assert_allclose(tv, refs[s].pose[1], atol=1e-6)
            np.testing.assert_allclose(fe.map_points(s), refs[s].X, rtol=2e-5, atol=1e-6)
    fe.close()


def test_frontend_scharr_pyramid_1080p_all_levels():
    """The 1080p launch's pyrDown + Scharr chain (maxLevel 4: 5 levels, the last
    one by scharr_kernel alone) bit-exact against the oracle on every level."""
    W, H, N, ML, _ = bench.CONFIGS["1080p"]
    ctx = S.Context(0)
    scenes = [Scene(W, H, seed=s) for s in (5, 6)]
    fe = _frontend(ctx, scenes, 3, 1000, ML)
    fe.init(0)
    fe.step(1)  # builds frame 2's derivatives ahead (frames 1 and 2 resident)
    for s, sc in enumerate(scenes):
        for t in (1, 2):
            lvl = sc.frame(t)
            for level in range(ML + 1):
                ix, iy = fe.scharr(s, t, level, lvl.shape[1], lvl.shape[0])
                ref = O.scharr(lvl).astype(np.int32)
                assert np.array_equal(ix.astype(np.int32), 4 * ref[..., 0]), f"seq {s} t {t} ix level {level}"
                assert np.array_equal(iy.astype(np.int32), 4 * ref[..., 1]), f"seq {s} t {t} iy level {level}"
                lvl = O.pyr_down(lvl)
    fe.close()


def test_bench_forward_128_slots_match_oracle_loop():
    """bench.py's `workloads.forward` at its own size: 1241x376 / 2000 features /
    maxLevel 3, 128 batch slots filled by the 16 distinct SceneForward sequences
    (seeds 1000..1015, each in 8 slots) -- the workload with real RANSAC outliers
    (occluder + parallax, ~10 % dropped per frame, ~8 hypotheses per sequence).
    All 16 distinct sequences against their own oracle loop at every step: inlier
    sets (the feature lists after outlier removal and the keyframe), counts,
    hypotheses, poses and map points; every hypothesis the oracle's RANSAC drew is
    re-solved by the product's minimal solver and counted when its bits differ
    (printed, asserted 0); every other slot bitwise equal to its twin slot."""
    from svo_amd.scene import SceneForward
    W, H, N, ML, _ = bench.CONFIGS["kitti"]
    ctx = S.Context(0)
    T, n_dist, n_seq = 7, 16, 128
    scs = [SceneForward(W, H, seed=1000 + i) for i in range(n_dist)]
    pairs = [[(sc.frame(t), sc.right(t)) for t in range(T)] for sc in scs]
    fe = S.Frontend(ctx, S.FrontendConfig(W, H, scs[0].K, n_seq=n_seq, n_frames=T, n_features=N, max_level=ML,
                                          timing=0))
    for s in range(n_seq):
        for t in range(T):
            fe.set_frame(s, t, *pairs[s % n_dist][t])
    fe.init(0)
    refs = [OracleLoop(SceneForward(W, H, seed=1000 + i), N, max_level=ML).init(0, *pairs[i][0])
            for i in range(n_dist)]
    K = scs[0].K
    hyps = differ = 0
    drops = []
    for t in range(1, T):
        st = fe.step(t).as_dict()
        rss = [r.step(t, *pairs[i][t]) for i, r in enumerate(refs)]
        reps = n_seq // n_dist
        for k in ("tracked", "inliers", "added", "features", "lk_iterations"):
            assert st[k] == reps * sum(rs[k] for rs in rss), f"{k} differs at t={t}"
        # (the product scores whole chunks: a hypothesis drawn past an accept that
        # lowered niters is scored and ignored, so it scores at least as many)
        assert st["hypotheses"] >= reps * sum(rs.get("hypotheses", 0) for rs in rss), f"hypotheses at t={t}"
        for i, ref in enumerate(refs):
            assert np.array_equal(fe.features(i), ref.pts), f"seq {i}: features differ at t={t}"
            rv, tv = fe.pose(i)
            np.testing.assert_allclose(rv, ref.pose[0], atol=1e-7)
            np.testing.assert_allclose(tv, ref.pose[1], atol=1e-6)
            if t % 3 == 0:
                np.testing.assert_allclose(fe.map_points(i), ref.X, rtol=2e-5, atol=1e-6)
            # the hypotheses of this step's RANSAC, product minimal solver vs oracle
            X2, p2, nh = ref.last_pnp
            if nh:
                obj = X2.astype(np.float32)
                img = np.ascontiguousarray(p2, np.float32)
                idx = O.ransac_subsets(len(obj), nh)
                subs = np.concatenate([obj[idx].reshape(nh, 15), img[idx].reshape(nh, 10)], axis=1)
                # device 0: the front end's host solver; 6: the same solver in GPU
                # lanes, one subset per lane (epnp_lane.hip)
                sols = [ctx.epnp_subsets(subs, K, device=dv) for dv in (0, 6)]
                for k in range(nh):
                    rc, Ro, to = O.epnp(obj[idx[k]], img[idx[k]], K)
                    for Rt, ok in sols:
                        same = (rc == 0) == bool(ok[k]) and (rc != 0 or np.array_equal(
                            np.r_[Ro.ravel(), to].view(np.uint64), Rt[k].view(np.uint64)))
                        differ += not same
                hyps += nh
        drops.append(1 - st["inliers"] / st["tracked"])
        for s in range(n_dist, n_seq, 37):  # twin slots
            assert np.array_equal(fe.features(s), fe.features(s % n_dist)), f"slot {s} vs {s % n_dist} at t={t}"
    print(f"forward 128 slots: RANSAC drops {np.round(drops, 3)}; {hyps} oracle hypotheses re-solved by the "
          f"product's EPnP on the host and in GPU lanes, {differ} differ")
    assert differ == 0
    assert np.mean(drops) > 0.05, "the occluder should make RANSAC outliers"
    fe.close()
