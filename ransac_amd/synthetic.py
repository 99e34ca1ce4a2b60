"""Synthetic correspondence sets of the BASELINE configurations.

numpy PCG64 streams (``np.random.default_rng(seed)``), so the same seed gives the same
fp32 points on every host.  These are workload generators for the bench and the tests,
not part of the hot path.
"""
import numpy as np


def _h_gt():
    """H_gt = perspective(1e-4, -5e-5) * translate(30, -20) * scale(1.1) * rot(10 deg)."""
    a = np.deg2rad(10.0)
    R = np.array([[np.cos(a), -np.sin(a), 0.0], [np.sin(a), np.cos(a), 0.0], [0.0, 0.0, 1.0]])
    S = np.diag([1.1, 1.1, 1.0])
    T = np.array([[1.0, 0.0, 30.0], [0.0, 1.0, -20.0], [0.0, 0.0, 1.0]])
    P = np.array([[1.0, 0.0, 0.0], [0.0, 1.0, 0.0], [1e-4, -5e-5, 1.0]])
    H = P @ T @ S @ R
    return H / H[2, 2]


def homography_points(n=10000, inlier_ratio=0.3, seed=1, noise=1.0, size=1000.0, cluster=None):
    """cfg2 (and cfg5 with cluster=(cx, cy, half_width)): N x 4 fp32 [x1 y1 x2 y2].

    Inliers: x2 = H_gt x1 + N(0, noise^2); outliers: x2 ~ U[0, size)^2.  Inliers and
    outliers are interleaved by a random permutation.  Returns (points, H_gt, is_inlier).
    """
    rng = np.random.default_rng(seed)
    H = _h_gt()
    n_in = int(round(n * inlier_ratio))
    x1 = rng.uniform(0.0, size, size=(n, 2))
    if cluster is not None:
        cx, cy, hw = cluster
        x1[:n_in, 0] = rng.uniform(cx - hw, cx + hw, size=n_in)
        x1[:n_in, 1] = rng.uniform(cy - hw, cy + hw, size=n_in)
    x1h = np.concatenate([x1, np.ones((n, 1))], axis=1)
    p = x1h @ H.T
    x2 = p[:, :2] / p[:, 2:3]
    x2[:n_in] += rng.normal(0.0, noise, size=(n_in, 2))
    x2[n_in:] = rng.uniform(0.0, size, size=(n - n_in, 2))
    pts = np.concatenate([x1, x2], axis=1)
    perm = rng.permutation(n)
    inl = np.zeros(n, dtype=bool)
    inl[:n_in] = True
    return np.ascontiguousarray(pts[perm], dtype=np.float32), H.astype(np.float32), inl[perm]


def line_points(n=1000, inlier_ratio=0.1, seed=1, noise=3.0, size=1000.0):
    """Line set: inliers near a random line through the image centre, uniform outliers."""
    rng = np.random.default_rng(seed)
    n_in = int(round(n * inlier_ratio))
    alpha = rng.uniform(0, np.pi)
    nx, ny = np.sin(alpha), np.cos(alpha)
    c = -(nx * size / 2 + ny * size / 2)
    t = rng.uniform(-0.5, 0.5, size=n_in) * size
    xs = size / 2 + t * (-ny) + rng.normal(0, noise, n_in) * nx
    ys = size / 2 + t * nx + rng.normal(0, noise, n_in) * ny
    out = rng.uniform(0, size, size=(n - n_in, 2))
    pts = np.concatenate([np.stack([xs, ys], 1), out], 0)
    perm = rng.permutation(n)
    return np.ascontiguousarray(pts[perm], dtype=np.float32), np.array([nx, ny, c], dtype=np.float32)


def _rot_y(deg):
    a = np.deg2rad(deg)
    return np.array([[np.cos(a), 0.0, np.sin(a)], [0.0, 1.0, 0.0], [-np.sin(a), 0.0, np.cos(a)]])


def _skew(t):
    return np.array([[0.0, -t[2], t[1]], [t[2], 0.0, -t[0]], [-t[1], t[0], 0.0]])


def two_view_geometry():
    """cfg3/cfg4 cameras: K = [[1000,0,500],[0,1000,500],[0,0,1]], cam1 = K[I|0],
    cam2 = K[R|t] with R = rotY(10 deg), t = (200, 0, 20).  Returns (K, R, t, E, F) with
    F = K^-T [t]x R K^-1 scaled so F33 = 1 and E = [t]x R / |t|."""
    K = np.array([[1000.0, 0.0, 500.0], [0.0, 1000.0, 500.0], [0.0, 0.0, 1.0]])
    R = _rot_y(10.0)
    t = np.array([200.0, 0.0, 20.0])
    E = _skew(t) @ R
    Ki = np.linalg.inv(K)
    F = Ki.T @ E @ Ki
    return K, R, t, E / np.linalg.norm(t), F / F[2, 2]


def fundamental_points(n=10000, inlier_ratio=0.3, seed=1, noise=0.5, size=1000.0, prosac_order=True,
                       normalized=False):
    """cfg3 (and cfg4 with normalized=True): N x 4 fp32 [x1 y1 x2 y2].

    X ~ U([-500,500]^2 x [1000,3000]) projected through both cameras + N(0, noise^2) px;
    outliers uniform in both images.  With prosac_order the rows are sorted by the PROSAC
    quality q = U(0,1) + 0.5 [inlier], descending; otherwise a random
    permutation.  normalized=True returns K^-1 x (calibrated coordinates, cfg4).
    Returns (points, F_gt (or E_gt when normalized), is_inlier)."""
    rng = np.random.default_rng(seed)
    K, R, t, E, F = two_view_geometry()
    n_in = int(round(n * inlier_ratio))
    X = np.stack([rng.uniform(-500, 500, n_in), rng.uniform(-500, 500, n_in), rng.uniform(1000, 3000, n_in)], 1)
    p1 = X @ K.T
    x1 = p1[:, :2] / p1[:, 2:3]
    p2 = (X @ R.T + t) @ K.T
    x2 = p2[:, :2] / p2[:, 2:3]
    x1 = x1 + rng.normal(0.0, noise, size=x1.shape)
    x2 = x2 + rng.normal(0.0, noise, size=x2.shape)
    o1 = rng.uniform(0.0, size, size=(n - n_in, 2))
    o2 = rng.uniform(0.0, size, size=(n - n_in, 2))
    pts = np.concatenate([np.concatenate([x1, x2], 1), np.concatenate([o1, o2], 1)], 0)
    inl = np.zeros(n, dtype=bool)
    inl[:n_in] = True
    if prosac_order:
        q = rng.uniform(0.0, 1.0, n) + 0.5 * inl
        order = np.argsort(-q, kind="stable")
    else:
        order = rng.permutation(n)
    pts, inl = pts[order], inl[order]
    model = F
    if normalized:
        Ki = np.linalg.inv(K)
        h1 = np.c_[pts[:, :2], np.ones(n)] @ Ki.T
        h2 = np.c_[pts[:, 2:], np.ones(n)] @ Ki.T
        pts = np.concatenate([h1[:, :2], h2[:, :2]], 1)
        model = E
    return np.ascontiguousarray(pts, dtype=np.float32), model.astype(np.float32), inl
