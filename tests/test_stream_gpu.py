"""Streamed frames (svo_frontend_queue_frames): each step's stereo pairs travel
over PCIe from page-locked host memory on the front end's upload stream into a
4-slot ring, as the reference's loader hands frames over one at a time
(R:include/async_image_loader.h:36-69; BGR converted as :63-69). The loop must
be the one the resident frames give: identical feature lists, counts and poses
every step, grey and BGR, and the oracle loop's for the first sequence."""
import numpy as np
import pytest

import oracle as O
import svo_amd as S
from oracle_loop import OracleLoop
from svo_amd.scene import Scene

pytestmark = pytest.mark.gpu


def _bgr(gray, seed):
    """A BGR frame whose channels differ (the conversion's weights matter)."""
    rng = np.random.default_rng(seed)
    d = rng.integers(-40, 41, gray.shape + (2,))
    b = np.clip(gray.astype(np.int32) + d[..., 0], 0, 255)
    r = np.clip(gray.astype(np.int32) - d[..., 1], 0, 255)
    return np.ascontiguousarray(np.stack([b, gray, r], axis=-1).astype(np.uint8))


@pytest.mark.parametrize("bgr", [False, True])
def test_streamed_frames_match_resident_frames(bgr):
    ctx = S.Context(0)
    W, H, N, T, NS = 640, 376, 800, 10, 3
    scenes = [Scene(W, H, seed=30 + s) for s in range(NS)]
    # host frames in one page-locked block, [t][s] (consecutive sequences follow each
    # other in memory: one H2D copy per side per step)
    shape = (T, NS, H, W, 3) if bgr else (T, NS, H, W)
    pl, pr = S.PinnedBuffer(shape), S.PinnedBuffer(shape)
    for t in range(T):
        for s, sc in enumerate(scenes):
            if bgr:
                pl.array[t, s] = _bgr(sc.frame(t), 100 * t + s)
                pr.array[t, s] = _bgr(sc.right(t), 100 * t + s + 50)
            else:
                pl.array[t, s] = sc.frame(t)
                pr.array[t, s] = sc.right(t)
    # resident: every frame uploaded before init (the bench's headline path)
    res = S.Frontend(ctx, S.FrontendConfig(W, H, scenes[0].K, n_seq=NS, n_frames=T, n_features=N))
    for t in range(T):
        for s in range(NS):
            res.set_frame(s, t, pl.array[t, s], pr.array[t, s])
    res.init(0)
    # streamed: a ring of 4 slots, frame t + 2 queued before step t
    stm = S.Frontend(ctx, S.FrontendConfig(W, H, scenes[0].K, n_seq=NS, n_frames=4, n_features=N))
    for t in range(3):
        stm.queue_frames(t, list(pl.array[t]), list(pr.array[t]))
    stm.init(0)
    grey = [O.bgr2gray(pl.array[t, 0]) if bgr else pl.array[t, 0] for t in range(T)]
    grey_r = [O.bgr2gray(pr.array[t, 0]) if bgr else pr.array[t, 0] for t in range(T)]
    ref = OracleLoop(scenes[0], N).init(0, grey[0], grey_r[0])
    for s in range(NS):
        assert np.array_equal(stm.features(s), res.features(s))
    assert np.array_equal(stm.features(0), ref.pts)
    for t in range(1, T - 2):
        stm.queue_frames(t + 2, list(pl.array[t + 2]), list(pr.array[t + 2]))
        a = stm.step(t).as_dict()
        b = res.step(t).as_dict()
        rs = ref.step(t, grey[t], grey_r[t])
        for k in ("tracked", "inliers", "added", "features", "lk_iterations"):
            assert a[k] == b[k], f"{k} at t={t}"
        for s in range(NS):
            assert np.array_equal(stm.features(s), res.features(s)), f"seq {s} at t={t}"
            assert np.array_equal(np.r_[stm.pose(s)], np.r_[res.pose(s)]), f"seq {s} pose at t={t}"
        assert np.array_equal(stm.features(0), ref.pts), f"oracle at t={t}"
        assert rs["tracked"] > 0.9 * len(ref.pts) or t == 1
    stm.upload_wait(T - 1)
    stm.close()
    res.close()
    pl.close()
    pr.close()


def test_queue_frames_ring_discipline():
    """Frames outside the ring window are refused (SVO_ERR_ARG), not overwritten."""
    ctx = S.Context(0)
    W, H, N = 320, 240, 300
    sc = Scene(W, H, seed=2)
    fe = S.Frontend(ctx, S.FrontendConfig(W, H, sc.K, n_seq=1, n_frames=4, n_features=N))
    frames = [(np.ascontiguousarray(sc.frame(t)), np.ascontiguousarray(sc.right(t))) for t in range(8)]
    for t in range(3):
        fe.queue_frames(t, [frames[t][0]], [frames[t][1]])
    fe.init(0)
    with pytest.raises(S.SvoError):  # step 1 consumes frame 3's slot ahead: frame 4 would reuse frame 0's
        fe.queue_frames(4, [frames[4][0]], [frames[4][1]])
    with pytest.raises(S.SvoError):  # frame 2 was consumed (its pyramid is built at init + step 1's front)
        fe.queue_frames(2, [frames[2][0]], [frames[2][1]])
    fe.queue_frames(3, [frames[3][0]], [frames[3][1]])
    fe.step(1)
    fe.queue_frames(4, [frames[4][0]], [frames[4][1]])
    fe.step(2)
    fe.upload_wait(4)
    fe.close()


def test_queue_frames_shape_restart_and_set_frame():
    """The wrapper refuses images of another size (the asynchronous copy would read
    past them); a frame at or before the last step restarts the loop, which then
    reproduces the first run; set_frame after streaming keeps the slot in the ring."""
    ctx = S.Context(0)
    W, H, N = 320, 240, 300
    sc = Scene(W, H, seed=4)
    fe = S.Frontend(ctx, S.FrontendConfig(W, H, sc.K, n_seq=1, n_frames=4, n_features=N))
    frames = [(np.ascontiguousarray(sc.frame(t)), np.ascontiguousarray(sc.right(t))) for t in range(7)]
    short = np.ascontiguousarray(frames[0][0][:-1])
    with pytest.raises(S.SvoError):
        fe.queue_frames(0, [short], [short])
    rgba = np.zeros((H, W, 4), np.uint8)
    with pytest.raises(S.SvoError):
        fe.queue_frames(0, [rgba], [rgba])

    def run(first_step_by_set_frame=False):
        for t in range(3):
            fe.queue_frames(t, [frames[t][0].copy()], [frames[t][1].copy()])  # temporaries: held by the wrapper
        fe.init(0)
        out = [fe.features(0)]
        for t in range(1, 5):
            if t + 2 <= 4:
                if first_step_by_set_frame and t + 2 == 3:
                    fe.set_frame(0, 3, frames[3][0], frames[3][1])  # slot 3 = frame 3, resident
                else:
                    fe.queue_frames(t + 2, [frames[t + 2][0]], [frames[t + 2][1]])
            fe.step(t)
            out.append(fe.features(0))
        return out

    a = run()
    b = run()  # frame 0 <= the last step (4): a restart
    c = run(first_step_by_set_frame=True)
    for t in range(len(a)):
        assert np.array_equal(a[t], b[t]) and np.array_equal(a[t], c[t]), f"t={t}"
    fe.close()
