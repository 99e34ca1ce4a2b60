"""The CPU oracle against the reference's own golden data (runs without a GPU).

Pins (see oracle/usac_oracle.h):
  * glibc random() KAT (the reference sampler's RNG);
  * the homography residual + cv::Mat::inv restatement reproduces the reference's
    published GT inlier counts on all 12 scenes (results/homography/*.csv, GT Inl);
  * the line2d loop (Uniform sampler, 2-pt estimator, standard termination, PCA polish)
    reproduces the published 50-run statistics (results/line2d/uniform_000.csv).
"""
import numpy as np
import pytest

from ransac_amd import synthetic


def test_glibc_random_kat(oracle):
    # glibc srandom(1) TYPE_3 stream (what the reference's random() yields with no srand)
    assert list(oracle.glibc_stream(1, 5)) == [1804289383, 846930886, 1681692777, 1714636915, 1957747793]


def test_uniform_sampler_pool_semantics(oracle):
    n, m = 7, 4
    s = oracle.uniform_samples(3, n, m, 50)
    assert s.min() >= 0 and s.max() < n
    # every n consecutive draws of the persistent pool are a permutation (uniform_sampler.hpp:42-54)
    flat = s.reshape(-1)
    for k in range(0, (flat.size // n) * n, n):
        assert sorted(flat[k:k + n].tolist()) == list(range(n))


def test_homography_gt_inliers_match_reference(oracle, homography_scenes):
    for scene, (pts, model, gt) in homography_scenes.items():
        assert oracle.gt_inliers_homography(pts, model, 2.0) == gt, scene


def test_inverse_matches_numpy(oracle, homography_scenes):
    for scene, (pts, model, gt) in homography_scenes.items():
        inv, ok = oracle.inv3x3(model)
        assert ok
        ref = np.linalg.inv(model.astype(np.float64).reshape(3, 3)).reshape(9)
        np.testing.assert_allclose(inv, ref, rtol=1e-5, atol=1e-9)
    z, ok = oracle.inv3x3(np.zeros(9, np.float32))
    assert not ok and not z.any()


def test_termination_kat(oracle):
    # SURVEY §8 a13 table (N=10k, m=4, p=.95) and the epsilon floor
    assert oracle.std_termination(2000, 10000, 4, 0.95) == 1870
    assert oracle.std_termination(3000, 10000, 4, 0.95) == 368
    assert oracle.std_termination(5000, 10000, 4, 0.95) == 46
    assert oracle.std_termination(1000, 10000, 4, 0.95) == 10000
    assert oracle.std_termination(10000, 10000, 4, 0.95) == 0


def test_dlt_nullspace_fits_exact_samples(oracle):
    pts, H, inl = synthetic.homography_points(n=200, inlier_ratio=1.0, noise=0.0, seed=5)
    est = oracle.Estimator(oracle.HOMOGRAPHY, pts, oracle.DLT_NULLSPACE)
    for k in range(20):
        sample = np.arange(4 * k, 4 * k + 4)
        m = est.estimate(sample)[0].reshape(3, 3)
        np.testing.assert_allclose(m / m[2, 2], H / H[2, 2], rtol=2e-3, atol=2e-5)
    # the reference's thin-SVD row is NOT the null vector
    thin = oracle.Estimator(oracle.HOMOGRAPHY, pts, oracle.DLT_THIN).estimate(np.arange(4))[0]
    assert not np.allclose(thin.reshape(3, 3), H / H[2, 2], rtol=1e-2)


def test_line2d_statistics_match_reference(oracle, line2d_scenes):
    """50 seeded runs per scene vs the reference's published 50-run averages."""
    for name, (pts, gt, st) in sorted(line2d_scenes.items())[:4]:
        inl, its = [], []
        for seed in range(1, 51):
            r = oracle.ransac_run(oracle.LINE2D, pts, 10.0, 0.99, seed)
            assert r["ret"] == 0
            inl.append(r["inliers"])
            its.append(r["iters"])
        se_inl = max(st["std_inliers"], 1.0) / np.sqrt(50)
        se_it = st["std_iters"] / np.sqrt(50)
        assert abs(np.mean(inl) - st["avg_inliers"]) < 4 * se_inl + 1.5, (name, np.mean(inl), st)
        assert abs(np.mean(its) - st["avg_iters"]) < 4 * se_it + 0.02 * st["avg_iters"], (name, np.mean(its), st)


def test_homography_run_real_scene(oracle, homography_scenes):
    pts, model, gt = homography_scenes["adam"]
    for mode in (oracle.DLT_THIN, oracle.DLT_NULLSPACE):
        r = oracle.ransac_run(oracle.HOMOGRAPHY, pts, 2.0, 0.95, 7, dlt_mode=mode)
        assert r["ret"] == 0
        # the reference reports 123-134 inliers after the polish on adam
        assert 115 <= r["inliers"] <= 140, r["inliers"]
        assert len(r["inlier_idx"]) == r["inliers"]


def test_line2d_generator(oracle):
    pts, gt = oracle.generate_line2d(11, 3.0, 100, 900, 1000, 1000)
    assert pts.shape == (1000, 2)
    assert abs(float(np.hypot(gt[0], gt[1])) - 1.0) < 1e-6
    d = np.abs(pts[900:] @ gt[:2] + gt[2])
    assert d.max() < 3.0 * 1.5


def test_line2d_generator_reproduces_reference_dataset(oracle, line2d_scenes):
    """The restated Generate2DLinePoints, run as generate_syntectic_dataset runs it
    (eight scenes on one rand() stream from the default seed), rewrites the reference's own
    dataset/line2d/*.txt: every coordinate and GT line equal at the digits the reference
    printed (ostream default precision 6)."""
    fmt = np.vectorize(lambda v: "%.6g" % v)
    gen = oracle.generate_line2d_dataset()
    assert sorted(n for n, _, _ in gen) == sorted(line2d_scenes)
    for name, pts, gt in gen:
        ref_pts, ref_model, _ = line2d_scenes[name]
        assert pts.shape == ref_pts.shape, name
        assert (fmt(pts.astype(np.float64)) == fmt(ref_pts.astype(np.float64))).all(), name
        assert (fmt(gt.astype(np.float64)) == fmt(ref_model.astype(np.float64))).all(), name


def _weighted_T(pts, idx, w):
    """normalizing_transformation.cpp:117-146 in numpy, fp32 sequential chains as written."""
    m = np.zeros(4, np.float32)
    d = np.zeros(2, np.float32)
    for i in idx:
        q = (w[i] * pts[i]).astype(np.float32)
        m = (m + q).astype(np.float32)
        d[0] = np.float32(np.float64(d[0]) + np.sqrt(np.float64(np.float32(q[0] * q[0] + q[1] * q[1]))))
        d[1] = np.float32(np.float64(d[1]) + np.sqrt(np.float64(np.float32(q[2] * q[2] + q[3] * q[3]))))
    m = (m / np.float32(len(idx))).astype(np.float32)
    s = [np.float32(np.sqrt(2.0) / np.float64(np.float32(d[k] / np.float32(len(idx))))) for k in range(2)]
    T = [np.array([[s[k], 0, -m[2 * k] * s[k]], [0, s[k], -m[2 * k + 1] * s[k]], [0, 0, 1]], np.float64)
         for k in range(2)]
    return T


@pytest.mark.parametrize("kind", ["H", "F"])
def test_weighted_nonminimal_matches_numpy(oracle, kind):
    """The weighted overload (normalized_dlt.cpp:25-36, eight_points.cpp:176-228): the oracle's
    model equals an fp64 numpy least-squares fit under the weighted normalisation (rel 1e-3), and the
    unweighted fit does not (the data hold outliers, so the normalisation moves the algebraic fit)."""
    rng = np.random.default_rng(3)
    if kind == "H":
        pts, _, _ = synthetic.homography_points(n=600, inlier_ratio=0.7, seed=5, noise=2.0)
    else:
        pts, _, _ = synthetic.fundamental_points(n=600, inlier_ratio=0.7, seed=5, noise=1.0, prosac_order=False)
    idx = np.sort(rng.choice(600, 300, replace=False)).astype(np.int32)
    w = (1.0 / (1.0 + rng.exponential(1.0, 600))).astype(np.float32)
    est = oracle.Estimator(oracle.HOMOGRAPHY if kind == "H" else oracle.FUNDAMENTAL, pts)
    got = est.nonminimal_weighted(idx, w)
    T1, T2 = _weighted_T(pts, idx, w)
    p = pts[idx].astype(np.float64)
    a = np.c_[p[:, :2], np.ones(len(idx))] @ T1.T
    b = np.c_[p[:, 2:], np.ones(len(idx))] @ T2.T
    x1, y1, x2, y2 = a[:, 0], a[:, 1], b[:, 0], b[:, 1]
    o, z = np.ones_like(x1), np.zeros_like(x1)
    if kind == "H":
        A = np.r_[np.c_[-x1, -y1, -o, z, z, z, x2 * x1, x2 * y1, x2],
                  np.c_[z, z, z, -x1, -y1, -o, y2 * x1, y2 * y1, y2]]
    else:
        A = np.c_[x2 * x1, x2 * y1, x2, y2 * x1, y2 * y1, y2, x1, y1, o]
    v = np.linalg.svd(A)[2][-1].reshape(3, 3)
    M = np.linalg.inv(T2) @ v @ T1 if kind == "H" else T2.T @ v @ T1
    M = M / M[2, 2]
    tol = dict(rtol=1e-3, atol=1e-5 * np.abs(M).max())
    assert np.allclose(got.reshape(3, 3), M, **tol)
    assert not np.allclose(est.nonminimal(idx).reshape(3, 3), M, **tol)
    with pytest.raises(NotImplementedError):
        oracle.Estimator(oracle.LINE2D, synthetic.line_points(200)[0]).nonminimal_weighted(idx[:10], w[:200])


def test_sym_eig_min_spec(oracle):
    """The 9x9 eigen spec of the LSQ fits (inverse iteration on A + 1e-12 tr(A) I, Jacobi
    fall-back) against numpy's eigh: the smallest eigenvalue's vector to 1e-10 on well-separated
    normal matrices (inverse iteration), on clustered spectra (fall-back) and rank-deficient ones."""
    rng = np.random.default_rng(7)
    n_inv = 0
    for case in range(300):
        Q, _ = np.linalg.qr(rng.normal(size=(9, 9)))
        kind = case % 3
        if kind == 0:    # LSQ-like: one small eigenvalue, ratio 1e-6 .. 1e-2
            w = np.r_[10 ** rng.uniform(-6, -2), rng.uniform(0.5, 5, 8)]
        elif kind == 1:  # the two smallest close together
            a = rng.uniform(0.1, 1)
            w = np.r_[a, a * rng.uniform(1.0, 1.5), rng.uniform(2, 5, 7)]
        else:            # exactly singular (a perfect fit)
            w = np.r_[0.0, rng.uniform(0.5, 5, 8)]
        A = (Q * w) @ Q.T
        A = (A + A.T) / 2
        v, ok = oracle.sym_eig_min(A)
        n_inv += ok
        ev, V = np.linalg.eigh(A)
        ref = V[:, 0]
        if kind == 1 and ev[1] - ev[0] < 1e-3:
            continue  # no well-defined smallest vector
        tol = 1e-10 if kind != 1 else 1e-6
        assert min(np.abs(v - ref).max(), np.abs(v + ref).max()) < tol, (case, ok)
    assert n_inv >= 150  # inverse iteration is the common path; the fall-back covers the rest
