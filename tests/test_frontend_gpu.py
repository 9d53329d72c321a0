"""Batched device-resident frontend vs the oracle-composed reference loop
(tests/oracle_loop.py): identical feature lists (bit-exact positions), identical
per-step counts, map points and poses equal to the oracle's, and per-sequence
results independent of the batch they run in."""
import numpy as np
import pytest

import oracle as O
import svo_amd as S
from oracle_loop import OracleLoop
from svo_amd.scene import Scene, SceneForward

pytestmark = pytest.mark.gpu


def make_frontend(ctx, scenes, T, n_features, **kw):
    sc0 = scenes[0]
    cfg = S.FrontendConfig(sc0.w, sc0.h, sc0.K, n_seq=len(scenes), n_frames=T, n_features=n_features, **kw)
    fe = S.Frontend(ctx, cfg)
    for s, sc in enumerate(scenes):
        for t in range(T):
            fe.set_frame(s, t, sc.frame(t), sc.right(t))
    return fe


def _compare_step(fe, ref, st, rs, t, seq=0, check_map=True):
    for k in ("tracked", "lk_iterations", "inliers", "added", "features"):
        assert st[k] == rs[k], f"{k} differs at t={t}: {st[k]} vs {rs[k]}"
    assert np.array_equal(fe.features(seq), ref.pts), f"features differ at t={t}"
    rv, tv = fe.pose(seq)
    np.testing.assert_allclose(rv, ref.pose[0], atol=1e-7)
    np.testing.assert_allclose(tv, ref.pose[1], atol=1e-6)
    if check_map:
        # triangulation: Jacobi SVD (product) vs the oracle's SVD -> last-bit float
        # differences; the pose fits agree to ~1e-9
        np.testing.assert_allclose(fe.map_points(seq), ref.X, rtol=2e-5, atol=1e-6)


@pytest.mark.parametrize("spec", ["-1", "0", "32"])
@pytest.mark.parametrize("bucket", [(0, 0), (50, 4)])
def test_frontend_matches_oracle_loop(bucket, spec, monkeypatch):
    """spec: SVO_FE_SPEC_MARGIN -- the keyframe's stereo LK run speculatively beside
    the RANSAC (32: the default; 0: the fused keyframe only when RANSAC dropped
    nothing, else the serial tail + stereo LK + append; -1: always serial)."""
    monkeypatch.setenv("SVO_FE_SPEC_MARGIN", spec)
    ctx = S.Context(0)
    W, H, N, T = 640, 376, 800, 8
    sc = Scene(W, H, seed=3)
    fe = make_frontend(ctx, [sc], T, N, bucket_size=bucket[0], per_bucket=bucket[1])
    fe.init(0)
    ref = OracleLoop(Scene(W, H, seed=3), N, bucket=bucket).init(0)
    assert np.array_equal(fe.features(0), ref.pts)
    np.testing.assert_allclose(fe.map_points(0), ref.X, rtol=2e-5, atol=1e-6)
    for t in range(1, T):
        st = fe.step(t).as_dict()
        rs = ref.step(t)
        _compare_step(fe, ref, st, rs, t)
        rv, _ = fe.pose(0)
        np.testing.assert_allclose(O.rodrigues(rv), sc.R(t), atol=3e-3)


@pytest.mark.parametrize("early", ["1", "0"])
def test_frontend_forward_occluder_matches_oracle_loop(early, monkeypatch):
    """The harder synthetic sequence (SceneForward: forward translation with
    parallax, a textured occluder sliding 22 px per frame against the static world)
    on two sequences at once, step by step against the oracle loop: RANSAC now
    drops 9-26 % of the tracked points per frame (more than the speculative stereo
    margin covers in some steps, so the serial keyframe path runs too), and the
    keyframes add several times more points than on the rotation-only scene.
    early: SVO_FE_SPEC_EARLY (the speculative stereo LK behind FAST(t) or behind
    the post-LK)."""
    monkeypatch.setenv("SVO_FE_SPEC_EARLY", early)
    ctx = S.Context(0)
    W, H, N, T = 640, 376, 800, 9
    seeds = (3, 8)
    fe = make_frontend(ctx, [SceneForward(W, H, seed=s) for s in seeds], T, N)
    fe.init(0)
    refs = [OracleLoop(SceneForward(W, H, seed=s), N).init(0) for s in seeds]
    drops = []
    for t in range(1, T):
        st = fe.step(t).as_dict()
        rss = [r.step(t) for r in refs]
        for k in ("tracked", "inliers", "added", "features"):
            assert st[k] == sum(rs[k] for rs in rss), f"{k} differs at t={t}"
        for q, (ref, sc) in enumerate(zip(refs, (SceneForward(W, H, seed=s) for s in seeds))):
            assert np.array_equal(fe.features(q), ref.pts), f"seq {q} features differ at t={t}"
            rv, tv = fe.pose(q)
            np.testing.assert_allclose(rv, ref.pose[0], atol=1e-7)
            np.testing.assert_allclose(tv, ref.pose[1], atol=1e-6)
            np.testing.assert_allclose(fe.map_points(q), ref.X, rtol=2e-5, atol=1e-6)
            R = O.rodrigues(rv)
            np.testing.assert_allclose(R, sc.R(t), atol=1e-2)
            np.testing.assert_allclose(-R.T @ tv, sc.C(t), atol=0.1)  # camera centre (m)
        drops.append(1 - st["inliers"] / st["tracked"])
    assert np.mean(drops) > 0.08, f"the occluder should make 10-30 % outliers ({np.round(drops, 3)})"


@pytest.mark.parametrize("bucket", [(0, 0), (50, 4)])
@pytest.mark.parametrize("pre", ["0", "1", "post"])
def test_frontend_fast_schedules(pre, bucket, monkeypatch):
    """Where FAST(t)'s detection runs, each against the oracle loop: behind LK(t) on
    the FAST stream (SVO_FE_FAST_PRE=0), or unmasked during step t-1 on the
    context stream with only the box filter + scan + emit behind LK(t) (1, the
    default; the mask drops corners after NMS), queued behind frame t-1's pyramid
    or behind step t-1's post-LK ("post": SVO_FE_PRE_AFTER_POST=1)."""
    monkeypatch.setenv("SVO_FE_FAST_PRE", "1" if pre == "post" else pre)
    monkeypatch.setenv("SVO_FE_PRE_AFTER_POST", "1" if pre == "post" else "0")
    ctx = S.Context(0)
    W, H, N, T = 640, 376, 800, 8
    fe = make_frontend(ctx, [Scene(W, H, seed=7)], T, N, bucket_size=bucket[0], per_bucket=bucket[1])
    fe.init(0)
    ref = OracleLoop(Scene(W, H, seed=7), N, bucket=bucket).init(0)
    for t in range(1, T):
        st = fe.step(t).as_dict()
        rs = ref.step(t)
        _compare_step(fe, ref, st, rs, t)


@pytest.mark.parametrize("pre", ["0", "1"])
def test_frontend_streaming_ring_and_reinit(pre, monkeypatch):
    """A ring of T = 3 resident frames filled while the sequence runs (frame t
    uploaded into slot t % 3 right before step(t)): a pyramid built ahead and a
    FAST pre-detection of a slot are dropped when its image is replaced. Then a
    second init on the same front end (everything queued ahead is drained first)
    and more steps, each against the oracle loop."""
    monkeypatch.setenv("SVO_FE_FAST_PRE", pre)
    ctx = S.Context(0)
    W, H, N, T = 640, 376, 800, 3
    sc = Scene(W, H, seed=9)
    fe = S.Frontend(ctx, S.FrontendConfig(W, H, sc.K, n_seq=1, n_frames=T, n_features=N))
    fe.set_frame(0, 0, sc.frame(0), sc.right(0))
    fe.init(0)
    ref = OracleLoop(Scene(W, H, seed=9), N).init(0)
    for t in range(1, 9):
        fe.set_frame(0, t % T, sc.frame(t), sc.right(t))
        st = fe.step(t).as_dict()
        _compare_step(fe, ref, st, ref.step(t), t)
    fe.init(8)  # slot 8 % 3 holds frame 8
    ref = OracleLoop(Scene(W, H, seed=9), N).init(8)
    assert np.array_equal(fe.features(0), ref.pts)
    for t in range(9, 13):
        fe.set_frame(0, t % T, sc.frame(t), sc.right(t))
        st = fe.step(t).as_dict()
        _compare_step(fe, ref, st, ref.step(t), t)
    fe.close()


def test_frontend_reference_keyframe_rule():
    """SVO_KF_REFERENCE: Tracking::nextFrame's rule (R:src/tracking.cpp:68-69) -- a
    frame is a keyframe iff its predecessor was not one and kept fewer than
    features_to_track features -- and a keyframe takes every masked corner (up to
    the capacity n_features), against the oracle loop's same rule. The threshold
    is set so that the synthetic sequence alternates between keyframes and
    tracking-only frames."""
    ctx = S.Context(0)
    W, H, N, T, F2T = 640, 376, 3000, 10, 100000
    sc = Scene(W, H, seed=4)
    fe = make_frontend(ctx, [sc], T, N, keyframe_rule=S.KF_REFERENCE, features_to_track=F2T)
    fe.init(0)
    ref = OracleLoop(Scene(W, H, seed=4), N, rule="reference", features_to_track=F2T).init(0)
    assert np.array_equal(fe.features(0), ref.pts)
    kfs = []
    for t in range(1, T):
        st = fe.step(t).as_dict()
        rs = ref.step(t)
        _compare_step(fe, ref, st, rs, t)
        assert st["keyframes"] == rs["keyframe"]
        kfs.append(st["keyframes"])
    assert kfs == [0, 1] * ((T - 1) // 2) + [0] * ((T - 1) % 2)   # prev KF => no KF, else count < F2T => KF
    # a threshold never reached: only frame 0 is a keyframe
    fe2 = make_frontend(ctx, [sc], 5, N, keyframe_rule=S.KF_REFERENCE, features_to_track=70)
    fe2.init(0)
    ref2 = OracleLoop(Scene(W, H, seed=4), N, rule="reference", features_to_track=70).init(0)
    for t in range(1, 5):
        st = fe2.step(t).as_dict()
        rs = ref2.step(t)
        _compare_step(fe2, ref2, st, rs, t)
        assert st["keyframes"] == 0 and st["added"] == 0


def test_frontend_reference_keyframe_rule_takes_every_corner_kitti():
    """SVO_KF_REFERENCE at 1241x376 on frames whose raw FAST count (~3-4k masked
    corners) exceeds the benchmark's 2000: with the capacity (n_features) sized
    above the detector's count, a keyframe takes every masked corner, as
    extractFeatures does (R:src/tracking.cpp:74-92) -- the step reports no
    overflow (kf_overflow 0) -- and every step matches the oracle loop's
    reference rule, keyframes and tracking-only frames alternating."""
    ctx = S.Context(0)
    W, H, N, T, F2T = 1241, 376, 8192, 7, 100000
    sc = Scene(W, H, seed=21)
    raw = len(O.fast(sc.frame(0), 20, True))
    assert raw > 2000, raw
    fe = make_frontend(ctx, [sc], T, N, keyframe_rule=S.KF_REFERENCE, features_to_track=F2T)
    fe.init(0)
    ref = OracleLoop(Scene(W, H, seed=21), N, rule="reference", features_to_track=F2T).init(0)
    assert ref.init_overflow == 0 and len(ref.pts) > 2000
    assert np.array_equal(fe.features(0), ref.pts)
    kfs = []
    for t in range(1, T):
        st = fe.step(t).as_dict()
        rs = ref.step(t)
        _compare_step(fe, ref, st, rs, t)
        assert st["keyframes"] == rs["keyframe"]
        assert st["kf_overflow"] == rs["kf_overflow"] == 0
        kfs.append(st["keyframes"])
    assert kfs == [0, 1, 0, 1, 0, 1]
    assert max(len(fe.features(0)), len(ref.pts)) > 2000


def test_frontend_fast_without_nms_matches_oracle_loop():
    """FAST without non-maximum suppression through the loop -- what the shipped
    YAML actually runs with use_orb: 0 (the key is spelled `nonmaxsuppression`,
    R:configs/config.yaml:31, the reader asks for `nonMaxSuppression`,
    R:include/config_reader.h:80, so it reads false) -- at the benchmark's
    1241x376 / 2000 features: every corner pixel is a candidate (~8x the NMS
    count, response 0 in raster order), every step against the oracle loop with
    the same detector."""
    ctx = S.Context(0)
    W, H, N, T = 1241, 376, 2000, 9
    sc = Scene(W, H, seed=11)
    assert len(O.fast(sc.frame(0), 20, False)) > 4 * len(O.fast(sc.frame(0), 20, True))
    fe = make_frontend(ctx, [sc], T, N, fast_nonmax=0)
    fe.init(0)
    ref = OracleLoop(Scene(W, H, seed=11), N, nonmax=False).init(0)
    assert np.array_equal(fe.features(0), ref.pts)
    added = 0
    for t in range(1, T):
        st = fe.step(t).as_dict()
        rs = ref.step(t)
        _compare_step(fe, ref, st, rs, t)
        added += rs["added"]
    assert added > 0


def test_frontend_fast_without_nms_reference_rule_kitti():
    """The shipped config's loop with use_orb: 0: FAST without suppression and
    Tracking::nextFrame's keyframe rule (features_to_track as the test needs
    keyframes), a keyframe taking every masked corner -- capacity sized above
    the unsuppressed corner count (no overflow) -- against the oracle loop."""
    ctx = S.Context(0)
    W, H, T, F2T = 1241, 376, 6, 100000
    sc = Scene(W, H, seed=21)
    raw = len(O.fast(sc.frame(0), 20, False))
    N = raw + 4096
    fe = make_frontend(ctx, [sc], T, N, keyframe_rule=S.KF_REFERENCE, features_to_track=F2T, fast_nonmax=0)
    fe.init(0)
    ref = OracleLoop(Scene(W, H, seed=21), N, rule="reference", features_to_track=F2T, nonmax=False).init(0)
    assert ref.init_overflow == 0 and len(ref.pts) > 4 * 2000
    assert np.array_equal(fe.features(0), ref.pts)
    kfs = []
    for t in range(1, T):
        st = fe.step(t).as_dict()
        rs = ref.step(t)
        _compare_step(fe, ref, st, rs, t, check_map=(t == T - 1))
        assert st["keyframes"] == rs["keyframe"]
        assert st["kf_overflow"] == rs["kf_overflow"] == 0
        kfs.append(st["keyframes"])
    assert kfs == [0, 1, 0, 1, 0]


@pytest.mark.parametrize("f2t", [70, 140])
def test_frontend_orb_batch_at_bench_size(f2t):
    """The shipped ORB configuration at the size bench.py times it
    (workloads.orb_reference: 1241x376, n_features 2000, use_orb 1,
    Tracking::nextFrame's rule, SceneForward seeds 2000 + i): 64 slots holding 8
    distinct sequences 8 times, 7 steps. Every distinct sequence against its oracle
    loop (cv::ORB restated, oracle/orb.cpp) every step, and every slot bitwise equal
    to the first slot of its sequence. features_to_track 70 is the shipped value
    (the ORB keyframe at init, then tracking-only steps); 140 makes keyframes recur
    within the 7 steps, so the batched ORB detection runs mid-sequence as well."""
    ctx = S.Context(0)
    W, H, N, T, D, SLOTS = 1241, 376, 2000, 8, 8, 64
    seeds = [2000 + i for i in range(D)]
    scenes = [SceneForward(W, H, seed=sd) for sd in seeds]
    cfg = S.FrontendConfig(W, H, scenes[0].K, n_seq=SLOTS, n_frames=T, n_features=N, use_orb=1,
                           keyframe_rule=S.KF_REFERENCE, features_to_track=f2t)
    fe = S.Frontend(ctx, cfg)
    frames = [[(sc.frame(t), sc.right(t)) for t in range(T)] for sc in scenes]
    for s in range(SLOTS):
        for t in range(T):
            fe.set_frame(s, t, *frames[s % D][t])
    fe.init(0)
    refs = [OracleLoop(SceneForward(W, H, seed=sd), N, rule="reference", features_to_track=f2t,
                       detector="orb").init(0) for sd in seeds]
    for q, ref in enumerate(refs):
        assert np.array_equal(fe.features(q), ref.pts), f"seq {q} features at init"
    kfs = 0
    for t in range(1, T):
        st = fe.step(t).as_dict()
        rss = [r.step(t) for r in refs]
        for k in ("tracked", "inliers", "added", "features"):
            assert st[k] == (SLOTS // D) * sum(rs[k] for rs in rss), f"{k} at t={t}"
        assert st["keyframes"] == (SLOTS // D) * sum(rs["keyframe"] for rs in rss), f"keyframes at t={t}"
        assert st["kf_overflow"] == 0
        kfs += st["keyframes"]
        for q, ref in enumerate(refs):
            assert np.array_equal(fe.features(q), ref.pts), f"seq {q} features at t={t}"
            rv, tv = fe.pose(q)
            np.testing.assert_allclose(rv, ref.pose[0], atol=1e-7)
            np.testing.assert_allclose(tv, ref.pose[1], atol=1e-6)
        for s in range(D, SLOTS):
            assert np.array_equal(fe.features(s), fe.features(s % D)), f"slot {s} at t={t}"
            assert np.array_equal(np.r_[fe.pose(s)], np.r_[fe.pose(s % D)]), f"slot {s} pose at t={t}"
    if f2t == 140:
        assert kfs > 0
    fe.close()


@pytest.mark.parametrize("spec", ["32", "-1"])
def test_frontend_reference_rule_mixed_batch(spec, monkeypatch):
    """SVO_KF_REFERENCE with sequences that are keyframes at different steps in the
    same batch (features_to_track set between their counts), the per-sequence
    targets running through the speculative stereo prep, the keyframe choice of
    fused / serial path (SVO_FE_SPEC_MARGIN 32 and -1): each sequence against its
    own oracle loop."""
    monkeypatch.setenv("SVO_FE_SPEC_MARGIN", spec)
    ctx = S.Context(0)
    W, H, T = 640, 376, 8
    Ns = (900, 1400, 3000)  # capacities; the batch shares the largest
    seeds = (4, 6, 12)
    scenes = [Scene(W, H, seed=sd) for sd in seeds]
    F2T = 1500  # between the sequences' counts: some keyframe, some not
    fe = make_frontend(ctx, scenes, T, max(Ns), keyframe_rule=S.KF_REFERENCE, features_to_track=F2T)
    fe.init(0)
    refs = [OracleLoop(Scene(W, H, seed=sd), max(Ns), rule="reference", features_to_track=F2T).init(0)
            for sd in seeds]
    mixed = False
    for t in range(1, T):
        st = fe.step(t).as_dict()
        rss = [r.step(t) for r in refs]
        for k in ("tracked", "inliers", "added", "features", "keyframe"):
            key = "keyframes" if k == "keyframe" else k
            assert st[key] == sum(rs[k] for rs in rss), f"{k} at t={t}"
        mixed |= 0 < st["keyframes"] < len(seeds)
        for q, ref in enumerate(refs):
            assert np.array_equal(fe.features(q), ref.pts), f"seq {q} features at t={t}"
            rv, tv = fe.pose(q)
            np.testing.assert_allclose(rv, ref.pose[0], atol=1e-7)
            np.testing.assert_allclose(tv, ref.pose[1], atol=1e-6)
    assert mixed, "some step should have keyframe and tracking-only sequences together"


@pytest.mark.parametrize("rule", ["reference", "every"])
def test_frontend_orb_matches_oracle_loop(rule):
    """use_orb = 1, the reference's shipped detector (R:configs/config.yaml:19-27:
    ORB, 150 features, scale 1.2, 8 levels, patch / edge 31, FAST 20, HARRIS;
    R:src/tracking.cpp:35-52): the batched front end detects each keyframe with
    ORB under the box mask (orb_batch_detect: scale + mask pyramids, per-level
    FAST and Harris for every sequence at once, retainBest on the host) -- every
    step against the oracle loop with cv::ORB restated (oracle/orb.cpp): counts,
    bit-identical feature lists (ORB's level-scaled positions), poses. "reference":
    Tracking::nextFrame's rule with features_to_track 140, so keyframes recur as
    the forward scene's tracks are lost; "every": every frame tops up to 400."""
    ctx = S.Context(0)
    W, H, T = 640, 376, 10
    seeds = (3, 8)
    kw = dict(keyframe_rule=S.KF_REFERENCE, features_to_track=140) if rule == "reference" else {}
    N = 2000 if rule == "reference" else 400
    fe = make_frontend(ctx, [SceneForward(W, H, seed=sd) for sd in seeds], T, N, use_orb=1, **kw)
    fe.init(0)
    refs = [OracleLoop(SceneForward(W, H, seed=sd), N, rule=rule, features_to_track=140, detector="orb").init(0)
            for sd in seeds]
    for q, ref in enumerate(refs):
        assert np.array_equal(fe.features(q), ref.pts), f"seq {q} features at init"
    kfs = 0
    for t in range(1, T):
        st = fe.step(t).as_dict()
        rss = [r.step(t) for r in refs]
        for k in ("tracked", "inliers", "added", "features"):
            assert st[k] == sum(rs[k] for rs in rss), f"{k} at t={t}"
        if rule == "reference":
            assert st["keyframes"] == sum(rs["keyframe"] for rs in rss), f"keyframes at t={t}"
            assert st["kf_overflow"] == 0
        kfs += st["keyframes"]
        for q, ref in enumerate(refs):
            assert np.array_equal(fe.features(q), ref.pts), f"seq {q} features at t={t}"
            rv, tv = fe.pose(q)
            np.testing.assert_allclose(rv, ref.pose[0], atol=1e-7)
            np.testing.assert_allclose(tv, ref.pose[1], atol=1e-6)
    assert kfs > 0 and st["added"] >= 0


def test_frontend_trace_mode_matches_oracle_loop(monkeypatch):
    """SVO_FE_TRACE=1 (per-task pool attribution, host trace printing) leaves the
    results unchanged: the same step-by-step match against the oracle loop."""
    monkeypatch.setenv("SVO_FE_TRACE", "1")
    ctx = S.Context(0)
    W, H, N, T = 640, 376, 800, 5
    fe = make_frontend(ctx, [SceneForward(W, H, seed=3), SceneForward(W, H, seed=8)], T, N)
    fe.init(0)
    refs = [OracleLoop(SceneForward(W, H, seed=sd), N).init(0) for sd in (3, 8)]
    for t in range(1, T):
        st = fe.step(t).as_dict()
        rss = [r.step(t) for r in refs]
        for k in ("tracked", "inliers", "added", "features"):
            assert st[k] == sum(rs[k] for rs in rss), f"{k} at t={t}"
        for q, ref in enumerate(refs):
            assert np.array_equal(fe.features(q), ref.pts), f"seq {q} features at t={t}"


def test_frontend_device_fits_match_host_fits(monkeypatch):
    """SVO_FE_DEVICE_FITS=1: the final SQPnP fits run on the device (launch_sqpnp_fit: the
    shared sqpnp.hpp code on the device) instead of the host pool -- the same
    poses bit for bit, hence the same map points and features, and the oracle's
    poses step by step."""
    ctx = S.Context(0)
    W, H, N, T = 640, 376, 800, 6
    seeds = (3, 8, 5)

    def run(device):
        monkeypatch.setenv("SVO_FE_DEVICE_FITS", "1" if device else "0")
        fe = make_frontend(ctx, [SceneForward(W, H, seed=sd) for sd in seeds], T, N)
        fe.init(0)
        out = []
        for t in range(1, T):
            fe.step(t)
            out.append([(np.r_[fe.pose(q)], fe.map_points(q).copy(), fe.features(q).copy())
                        for q in range(len(seeds))])
        return out

    host, dev = run(False), run(True)
    refs = [OracleLoop(SceneForward(W, H, seed=sd), N).init(0) for sd in seeds]
    for t in range(1, T):
        for q, ref in enumerate(refs):
            ref.step(t)
            ph, mh, fh = host[t - 1][q]
            pd, md, fd = dev[t - 1][q]
            assert np.array_equal(ph, pd), f"seq {q} pose at t={t}"
            assert np.array_equal(mh, md) and np.array_equal(fh, fd), f"seq {q} map at t={t}"
            np.testing.assert_allclose(pd[:3], ref.pose[0], atol=1e-7)
            np.testing.assert_allclose(pd[3:], ref.pose[1], atol=1e-6)


def test_frontend_200_frames_kitti_matches_oracle_loop():
    """BASELINE.json configs[0]: 200 frames of a 1241x376 sequence with 2000
    features, every step against the oracle loop (R:src/tracking.cpp:232-276)."""
    ctx = S.Context(0)
    W, H, N, T = 1241, 376, 2000, 201
    sc = Scene(W, H, seed=11)
    fe = make_frontend(ctx, [sc], T, N)
    fe.init(0)
    ref = OracleLoop(Scene(W, H, seed=11), N).init(0)
    assert np.array_equal(fe.features(0), ref.pts)
    for t in range(1, T):
        st = fe.step(t).as_dict()
        rs = ref.step(t)
        _compare_step(fe, ref, st, rs, t, check_map=(t % 25 == 0 or t == T - 1))
    rv, _ = fe.pose(0)
    np.testing.assert_allclose(O.rodrigues(rv), sc.R(T - 1), atol=5e-3)


def test_frontend_batch_independence():
    """A sequence's result does not depend on the batch it runs in."""
    ctx = S.Context(0)
    W, H, N, T = 1241, 376, 2000, 4
    scenes = [Scene(W, H, seed=s) for s in range(3)]
    feb = make_frontend(ctx, scenes, T, N)
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
            assert np.array_equal(feb.map_points(s), f.map_points(0))


def test_frontend_kitti_sequence_keeps_features():
    ctx = S.Context(0)
    W, H, N, T = 1241, 376, 2000, 12
    sc = Scene(W, H, seed=0)
    fe = make_frontend(ctx, [sc], T, N, timing=1)
    fe.init(0)
    for t in range(1, T):
        st = fe.step(t).as_dict()
        assert 0.97 * N <= st["features"] <= N
        assert st["tracked"] > 0.9 * N
        assert st["inliers"] > 0.9 * st["tracked"]
        rv, tv = fe.pose(0)
        np.testing.assert_allclose(O.rodrigues(rv), sc.R(t), atol=3e-3)
        assert np.abs(tv).max() < 0.05
    # the map points sit on the scene's depth field (stereo LK + triangulation)
    X = fe.map_points(0)
    Xt = sc.map_points(fe.features(0), T - 1)
    assert np.median(np.abs(X[:, 2] - Xt[:, 2]) / Xt[:, 2]) < 0.02
    pt = fe.phase_times()
    assert pt["lk"][1] == T - 1 and pt["lk"][0] > 0
    # init's keyframe + one per step (speculative), + a serial one for a step whose
    # RANSAC dropped more than the speculation covered
    assert T <= pt["stereo_lk"][1] <= 2 * T - 1


def test_frontend_kernel_timers_leave_the_sequence_intact():
    """svo_frontend_time_fast / svo_frontend_time_pyramid (bench.py's roofline legs)
    between steps: they overwrite the FAST row words / a pyramid built ahead, and
    the following steps still match the oracle loop (the pre-detection and the
    pyramid are redone)."""
    ctx = S.Context(0)
    W, H, N, T = 640, 376, 800, 8
    sc = Scene(W, H, seed=5)
    fe = make_frontend(ctx, [sc], T, N)
    fe.init(0)
    ref = OracleLoop(Scene(W, H, seed=5), N).init(0)
    for t in range(1, T):
        st = fe.step(t).as_dict()
        _compare_step(fe, ref, st, ref.step(t), t)
        if t in (2, 4):
            assert fe.time_fast(t + 1, 3) > 0
            assert fe.time_pyramid(t + 1, 2) > 0
