"""Reprojection residual / SE(3) Jacobian / normal-equation kernel (§8 a11) and
the host LM pose solver it feeds. The reference has no implementation (Ceres is
linked but never called), so the kernel is pinned by an
independent float64 numpy restatement and by central finite differences."""
import numpy as np
import pytest

import svo_amd as S

pytestmark = pytest.mark.gpu

K = np.array([[718.856, 0, 607.1928], [0, 718.856, 185.2157], [0, 0, 1]])


@pytest.fixture(scope="module")
def ctx():
    return S.Context(0)


def hat(w):
    return np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])


def se3_exp(xi):
    rho, ph = xi[:3], xi[3:]
    th = np.linalg.norm(ph)
    W = hat(ph)
    if th < 1e-10:
        return np.eye(3) + W, rho
    A, B, C = np.sin(th) / th, (1 - np.cos(th)) / th ** 2, (th - np.sin(th)) / th ** 3
    R = np.eye(3) + A * W + B * W @ W
    V = np.eye(3) + B * W + C * W @ W
    return R, V @ rho


def left_update(T, xi):
    R, t = T[:9].reshape(3, 3), T[9:]
    dR, dt = se3_exp(xi)
    return np.r_[(dR @ R).ravel(), dR @ t + dt]


def project(T, X):
    P = X @ T[:9].reshape(3, 3).T + T[9:]
    return np.c_[K[0, 0] * P[:, 0] / P[:, 2] + K[0, 2], K[1, 1] * P[:, 1] / P[:, 2] + K[1, 2]], P


def ref_normal(T, X, u, delta=0.0):
    """numpy restatement: r, J (analytic), H/g/cost."""
    uv, P = project(T, X)
    r = uv - u.astype(np.float64)
    x, y, z = P[:, 0] / P[:, 2], P[:, 1] / P[:, 2], P[:, 2]
    fx, fy = K[0, 0], K[1, 1]
    J = np.zeros((len(X), 2, 6))
    J[:, 0] = np.c_[fx / z, 0 * z, -fx * x / z, -fx * x * y, fx * (1 + x * x), -fx * y]
    J[:, 1] = np.c_[0 * z, fy / z, -fy * y / z, -fy * (1 + y * y), fy * x * y, fy * x]
    nr = np.linalg.norm(r, axis=1)
    w = np.where((delta > 0) & (nr > delta), delta / np.maximum(nr, 1e-300), 1.0)
    H = np.einsum("n,nai,naj->ij", w, J, J)
    g = np.einsum("n,nai,na->i", w, J, r)
    cost = np.where((delta > 0) & (nr > delta), delta * (nr - 0.5 * delta), 0.5 * nr ** 2).sum()
    iu = np.triu_indices(6)
    return r, J, np.r_[H[iu], g, cost]


def scene(n, seed, noise=0.0, outliers=0.0):
    rng = np.random.default_rng(seed)
    X = np.c_[rng.uniform(-8, 8, n), rng.uniform(-3, 3, n), rng.uniform(5, 40, n)]
    th = rng.normal(0, 0.05, 3)
    R, _ = se3_exp(np.r_[0, 0, 0, th])
    T = np.r_[R.ravel(), rng.normal(0, 0.3, 3)]
    u, _ = project(T, X)
    u = u + rng.normal(0, noise, u.shape) if noise else u
    if outliers:
        m = rng.random(n) < outliers
        u[m] += rng.uniform(-60, 60, (m.sum(), 2))
    return X, u.astype(np.float32), T


def test_residuals_jacobians_normals_match_numpy(ctx):
    X, u, T = scene(3000, 1, noise=1.0)
    T0 = left_update(T, np.r_[0.05, -0.02, 0.1, 0.003, -0.002, 0.001])
    res, jac, ne = ctx.reprojection_jacobians(X, u, T0[None], K)
    r, J, ne_ref = ref_normal(T0, X, u)
    assert np.allclose(res[0], r, rtol=1e-12, atol=1e-9)
    assert np.allclose(jac[0], J, rtol=1e-12, atol=1e-9)
    assert np.allclose(ne[0], ne_ref, rtol=1e-10, atol=1e-6)
    # deterministic reduction order: identical bits on a repeat
    _, _, ne2 = ctx.reprojection_jacobians(X, u, T0[None], K)
    assert np.array_equal(ne.view(np.uint64), ne2.view(np.uint64))


def test_jacobian_matches_finite_differences(ctx):
    X, u, T = scene(200, 2)
    _, jac, _ = ctx.reprojection_jacobians(X, u, T[None], K)
    h = 1e-6
    for k in range(6):
        e = np.zeros(6)
        e[k] = h
        up, _ = project(left_update(T, e), X)
        um, _ = project(left_update(T, -e), X)
        fd = (up - um) / (2 * h)
        assert np.allclose(jac[0, :, :, k], fd, rtol=1e-5, atol=1e-4), k


def test_huber_ragged_batch_and_behind_camera(ctx):
    P, n = 5, 700
    Xs, us, Ts, counts = [], [], [], []
    for b in range(P):
        X, u, T = scene(n, 10 + b, noise=0.5, outliers=0.2)
        Xs.append(X); us.append(u); Ts.append(T); counts.append(n - 97 * b)
    Xs, us, Ts = np.stack(Xs), np.stack(us), np.stack(Ts)
    Xs[0, 5] = [0, 0, -Ts[0][11] - 3.0]        # behind the camera after the pose (roughly): z <= 0 adds 0
    _, _, ne = ctx.reprojection_jacobians(Xs, us, Ts, K, counts=counts, huber_delta=2.0)
    for b in range(P):
        c = counts[b]
        X, u = Xs[b, :c], us[b, :c]
        _, P3 = project(Ts[b], X)
        keep = P3[:, 2] > 0
        _, _, ref = ref_normal(Ts[b], X[keep], u[keep], 2.0)
        assert np.allclose(ne[b], ref, rtol=1e-10, atol=1e-6), b


def test_refine_converges_and_is_robust(ctx):
    P = 16
    Xs, us, Ts, T0s = [], [], [], []
    for b in range(P):
        X, u, T = scene(1500, 100 + b)
        Xs.append(X); us.append(u); Ts.append(T)
        T0s.append(left_update(T, np.r_[0.2, -0.1, 0.3, 0.02, -0.01, 0.015]))
    poses, costs, it = ctx.refine_poses(np.stack(Xs), np.stack(us), np.stack(T0s), K, max_iterations=50)
    for b in range(P):
        assert np.abs(poses[b] - Ts[b]).max() < 1e-5, b        # float observations -> ~1e-6 pose noise
    assert np.all(costs < 1e-6 * 1500) and it > 0
    # with outliers: Huber recovers the pose, plain least squares is pulled away
    X, u, T = scene(2000, 7, noise=0.5, outliers=0.25)
    T0 = left_update(T, np.r_[0.1, 0.1, -0.2, 0.01, 0.0, -0.01])
    ph, _, _ = ctx.refine_poses(X, u, T0[None], K, huber_delta=1.0, max_iterations=100)
    pl, _, _ = ctx.refine_poses(X, u, T0[None], K, huber_delta=0.0, max_iterations=100)
    eh, el = np.abs(ph[0, 9:] - T[9:]).max(), np.abs(pl[0, 9:] - T[9:]).max()
    assert eh < 0.02 and eh < el


def test_bad_arguments_and_empty(ctx):
    X, u, T = scene(10, 3)
    with pytest.raises(S.SvoError):
        ctx.reprojection_jacobians(X, u, T[None], K, counts=[11])
    res, jac, ne = ctx.reprojection_jacobians(X, u, T[None], K, counts=[0])
    assert np.all(ne == 0)
