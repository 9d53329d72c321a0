"""solvePnPRansac's final solvePnP(SQPNP) fit: the product's host solver
(svo_solve_pnp_sqpnp, pose.cpp: SQPnP's cost and solution search, Gauss-Newton
on SO(3) for the SQP runs) against the oracle's independent restatement of
OpenCV's sqpnp.cpp (oracle/sqpnp.c: SQP iterations, nearestRotationMatrix).
Host code only (no GPU context), so it runs in the CPU suite."""
import numpy as np
import pytest

import oracle as O
import svo_amd as S


def _problem(n, noise_px, seed, depth=(6, 40)):
    from scipy.spatial.transform import Rotation as Rot
    rng = np.random.default_rng(seed)
    K = np.array([[718.856, 0, 607.1928], [0, 718.856, 185.2157], [0, 0, 1]])
    X = np.c_[rng.uniform(-15, 15, n), rng.uniform(-4, 4, n), rng.uniform(*depth, n)]
    R = Rot.from_rotvec(rng.normal(0, 0.05, 3)).as_matrix()
    t = rng.normal(0, 0.3, 3)
    Y = X @ R.T + t
    uv = (Y[:, :2] / Y[:, 2:]) * [K[0, 0], K[1, 1]] + [K[0, 2], K[1, 2]] + rng.normal(0, noise_px, (n, 2))
    return X, uv.astype(np.float32), K


def _oracle_pose(X, uv, K):
    q = (uv.astype(np.float64) - [K[0, 2], K[1, 2]]) * [1 / K[0, 0], 1 / K[1, 1]]
    rc, R, t = O.sqpnp(X, q)
    rv = np.zeros(3)
    if rc == 0:
        O.load().svo_oracle_rodrigues_inv(np.ascontiguousarray(R.ravel()).ctypes.data_as(O._f64p),
                                          rv.ctypes.data_as(O._f64p))
    return rc, rv, t


@pytest.mark.parametrize("n,noise,seed", [(2000, 0.0, 0), (2000, 0.3, 1), (500, 1.0, 2), (60, 2.0, 3),
                                          (2000, 0.5, 4), (300, 0.1, 5)])
def test_sqpnp_fit_matches_oracle(n, noise, seed):
    X, uv, K = _problem(n, noise, seed)
    ok, rv, tv = S.solve_pnp_sqpnp(X, uv, K)
    rc, rvo, tvo = _oracle_pose(X, uv, K)
    assert ok and rc == 0
    print(f"n={n} noise={noise}: |drv| {np.abs(rv - rvo).max():.3g} |dtv| {np.abs(tv - tvo).max():.3g}")
    np.testing.assert_allclose(rv, rvo, atol=1e-7)
    np.testing.assert_allclose(tv, tvo, atol=1e-7)


def test_sqpnp_fit_degenerate_points():
    """Every image point at one pixel: SQPnP's variance assert -> no pose, both."""
    X, uv, K = _problem(50, 0.0, 6)
    uv[:] = uv[0]
    ok, _, _ = S.solve_pnp_sqpnp(X, uv, K)
    rc, _, _ = _oracle_pose(X, uv, K)
    assert not ok and rc == -1
