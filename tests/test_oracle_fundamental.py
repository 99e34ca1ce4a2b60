"""CPU oracle, fundamental path, no GPU.

Parity of the 7-point solver against the reference is UNPINNED: the reference's numbers come
from OpenCV's SVDecomp / solveCubic (not in this image) and its only F fixture column
("GT Inl" of results/kusvod2/*.csv) is not reproducible from its data files (see
tests/golden/make_golden.py).  The oracle is pinned instead by identities the reference
algorithm satisfies: exact data recovers the generating F, every returned F is rank-2 and
passes the oriented constraint on its sample, the Sampson error equals the textbook
closed form, and the cubic solver finds the roots of known polynomials.
"""
import numpy as np
import pytest

from ransac_amd import synthetic


def _dist(m, F):
    a = m.reshape(-1) / np.linalg.norm(m)
    b = F.reshape(-1) / np.linalg.norm(F)
    return min(np.linalg.norm(a - b), np.linalg.norm(a + b))


def test_cubic_known_roots(oracle):
    assert oracle.cubic_roots(1, -6, 11, -6) == pytest.approx([1, 2, 3], abs=1e-12)
    assert oracle.cubic_roots(1, 0, 0, -8) == pytest.approx([2], abs=1e-12)
    assert oracle.cubic_roots(2, 0, -2, 0) == pytest.approx([-1, 0, 1], abs=1e-12)
    assert oracle.cubic_roots(0, 1, -3, 2) == pytest.approx([1, 2], abs=1e-12)
    assert oracle.cubic_roots(0, 0, 2, -4) == pytest.approx([2], abs=1e-12)
    assert oracle.cubic_roots(0, 0, 0, 1) == []
    assert oracle.cubic_roots(1, 0, 1, 0) == pytest.approx([0], abs=1e-12)


def test_cubic_matches_numpy_roots(oracle):
    rng = np.random.default_rng(0)
    for _ in range(300):
        c = rng.normal(size=4) * 10.0 ** rng.integers(-3, 4, size=4)
        got = oracle.cubic_roots(*c.tolist())
        ref = np.roots(c)
        real = np.sort(ref[np.abs(ref.imag) < 1e-7 * np.maximum(1, np.abs(ref))].real)
        assert len(got) >= 1
        # every returned value is a root (relative residual) and every clear real root is found
        a, b, cc = c[1] / c[0], c[2] / c[0], c[3] / c[0]
        for r in got:
            scale = 1 + abs(r) ** 3 + abs(a) * r * r + abs(b * r) + abs(cc)
            assert abs(((r + a) * r + b) * r + cc) <= 1e-12 * scale
        if len(real) == len(got):
            np.testing.assert_allclose(got, real, rtol=1e-6, atol=1e-9)


def test_sampson_error_closed_form(oracle, kusvod2_scenes):
    for scene, (pts, F) in kusvod2_scenes.items():
        est = oracle.Estimator(oracle.FUNDAMENTAL, pts)
        e = est.errors(F).astype(np.float64)
        Fd = F.astype(np.float64).reshape(3, 3)
        x1 = np.c_[pts[:, :2], np.ones(len(pts))].astype(np.float64)
        x2 = np.c_[pts[:, 2:], np.ones(len(pts))].astype(np.float64)
        Fx1 = x1 @ Fd.T
        Ftx2 = x2 @ Fd
        num = np.einsum("ij,ij->i", x2, Fx1) ** 2
        den = Fx1[:, 0] ** 2 + Fx1[:, 1] ** 2 + Ftx2[:, 0] ** 2 + Ftx2[:, 1] ** 2
        ref = num / den
        # fp32 cancellation in x2^T F x1: compare the distances sqrt(err) (px), 1e-3 px abs
        np.testing.assert_allclose(np.sqrt(e), np.sqrt(ref), rtol=1e-4, atol=1e-3, err_msg=scene)


def test_seven_point_recovers_exact_F(oracle):
    pts, F, inl = synthetic.fundamental_points(n=2000, inlier_ratio=0.3, seed=1, noise=0.0)
    est = oracle.Estimator(oracle.FUNDAMENTAL, pts)
    idx = np.where(inl)[0]
    rng = np.random.default_rng(0)
    hit = 0
    for _ in range(100):
        s = rng.choice(idx, 7, replace=False).astype(np.int32)
        ms = est.estimate(s)
        assert len(ms) <= 3
        for m in ms:
            M = m.reshape(3, 3).astype(np.float64)
            sv = np.linalg.svd(M, compute_uv=False)
            assert sv[2] <= 1e-3 * sv[0]  # rank 2 up to fp32 rounding
        if len(ms) and min(_dist(m, F) for m in ms) < 1e-3:
            hit += 1
    # fp32, unnormalised pixel coordinates (as the reference): most exact samples recover F
    assert hit >= 75


def test_seven_point_models_pass_oriented_constraint(oracle):
    pts, F, inl = synthetic.fundamental_points(n=500, inlier_ratio=0.3, seed=2)
    est = oracle.Estimator(oracle.FUNDAMENTAL, pts)
    samples = oracle.uniform_samples(4, len(pts), 7, 300)
    models, nm = est.estimate_batch(samples)
    assert models.shape == (300, 3, 9)
    assert nm.min() >= 0 and nm.max() <= 3
    for b in range(300):
        for j in range(nm[b]):
            M = models[b, j].reshape(3, 3)
            e = np.cross(M[0], M[2])
            if np.all(np.abs(e) <= 1.9984e-15):
                e = np.cross(M[1], M[2])
            P = pts[samples[b]]
            sig = (M[0, 0] * P[:, 2] + M[1, 0] * P[:, 3] + M[2, 0]) * (e[1] - e[2] * P[:, 1])
            assert np.all(sig * sig[0] >= -1e-3 * np.abs(sig).max() * abs(sig[0]))
        assert not models[b, nm[b]:].any()


def test_eight_point_recovers_exact_F(oracle):
    pts, F, inl = synthetic.fundamental_points(n=2000, inlier_ratio=0.3, seed=3, noise=0.0)
    est = oracle.Estimator(oracle.FUNDAMENTAL, pts)
    idx = np.where(inl)[0].astype(np.int32)
    assert _dist(est.nonminimal(idx), F) < 1e-5
    assert _dist(est.nonminimal(idx[:9]), F) < 1e-3


def test_ransac_fundamental_finds_inliers(oracle):
    pts, F, inl = synthetic.fundamental_points(n=2000, inlier_ratio=0.3, seed=4, prosac_order=False)
    r = oracle.ransac_run(oracle.FUNDAMENTAL, pts, 2.0, 0.95, 1)
    assert r["ret"] == 0
    found = set(r["inlier_idx"].tolist())
    truth = set(np.where(inl)[0].tolist())
    assert len(found & truth) >= 0.9 * len(truth)
    assert r["iters"] <= 10000 and r["polish_passes"] <= 4
