"""Front ends created and destroyed in one long-lived process (the reference's
loop re-creates frames every keyframe, R:src/tracking.cpp:232-276; the bench's
side workloads create and close front ends beside the headline's).

Every front end on a context runs on the context's streams: a second front end
made while the first lives, and a third made after both are closed, bind no new
hardware queues. Their results are those of a front end alone on a fresh
context, step for step. (The bench's side workloads run before the headline in
`--legs first`; the 12 % that order once cost is DESIGN.md section 6.)"""
import numpy as np
import pytest

import svo_amd as S
from svo_amd.scene import Scene

pytestmark = pytest.mark.gpu

W, H, N, T, NS = 640, 376, 600, 7, 2


def _run(ctx, seed0, close=True):
    scenes = [Scene(W, H, seed=seed0 + s) for s in range(NS)]
    fe = S.Frontend(ctx, S.FrontendConfig(W, H, scenes[0].K, n_seq=NS, n_frames=T, n_features=N))
    for s, sc in enumerate(scenes):
        for t in range(T):
            fe.set_frame(s, t, sc.frame(t), sc.right(t))
    fe.init(0)
    out = []
    for t in range(1, T):
        st = fe.step(t).as_dict()
        out.append((st["tracked"], st["inliers"], st["added"], [fe.features(s).copy() for s in range(NS)],
                    [np.r_[fe.pose(s)] for s in range(NS)]))
    streams = fe.streams()
    if close:
        fe.close()
        return out, streams, None
    return out, streams, fe


def _same(a, b):
    assert len(a) == len(b)
    for x, y in zip(a, b):
        assert x[:3] == y[:3]
        for s in range(NS):
            assert np.array_equal(x[3][s], y[3][s])
            assert np.array_equal(x[4][s], y[4][s])


def test_front_ends_share_the_context_streams_and_results_hold():
    ref, _, _ = _run(S.Context(0), 50)           # alone on its own context
    ctx = S.Context(0)
    a, st_a, fe_a = _run(ctx, 50, close=False)   # the first front end, kept alive
    b, st_b, _ = _run(ctx, 50)                   # a second one beside it, then closed
    fe_a.close()
    c, st_c, _ = _run(ctx, 50)                   # a third after both are gone
    assert len(set(st_a)) == 3 and st_a == st_b == st_c
    _same(ref, a)
    _same(ref, b)
    _same(ref, c)
