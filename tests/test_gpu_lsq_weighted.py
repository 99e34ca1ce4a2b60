"""usac_lsq_fit with weights: Estimator::EstimateModelNonMinimalSample(sample, n, weights, model)
(estimator.hpp:26) -- the weighted NormalizedDLT (normalized_dlt.cpp:25-36) and the weighted
8-point algorithm (eight_points.cpp:176-228), through the weighted GetNormalizingTransformation
(normalizing_transformation.cpp:117-166).  The device equals the oracle bit for bit.

Parity unpinned against the reference itself: its only caller is the IRLS local optimisation
(irls.hpp:108, out of scope), and no reference test or results file covers a weighted fit."""
import numpy as np
import pytest

from ransac_amd import synthetic

pytestmark = pytest.mark.gpu


def _data(kind, n, seed):
    if kind == "H":
        pts, _, _ = synthetic.homography_points(n=n, inlier_ratio=0.6, seed=seed)
    else:
        pts, _, _ = synthetic.fundamental_points(n=n, inlier_ratio=0.6, seed=seed, prosac_order=False)
    return pts


@pytest.mark.parametrize("kind", ["H", "F"])
@pytest.mark.parametrize("k", [4, 8, 9, 37, 1000, 20000, 70000])
def test_weighted_fit_bit_exact(usac, oracle, kind, k):
    n = max(k, 2000)
    pts = _data(kind, n, seed=k)
    rng = np.random.default_rng(k)
    idx = np.sort(rng.choice(n, size=k, replace=False)).astype(np.int32)
    # IRLS-like weights 1 / (1 + err) in (0, 1], plus exact 0 and 1 entries
    w = (1.0 / (1.0 + rng.exponential(2.0, size=n))).astype(np.float32)
    w[idx[: max(1, k // 10)]] = 1.0
    w[idx[-1]] = 0.0
    est_k = usac.ESTIMATOR.Homography if kind == "H" else usac.ESTIMATOR.Fundamental
    with usac.Context(est_k, pts) as ctx:
        got = ctx.lsq_fit(idx, w)
        plain = ctx.lsq_fit(idx)
        assert (plain.view(np.int32) == ctx.nonminimal(idx).view(np.int32)).all()
    est = oracle.Estimator(oracle.HOMOGRAPHY if kind == "H" else oracle.FUNDAMENTAL, pts)
    ref = est.nonminimal_weighted(idx, w)
    assert ref is not None
    assert (got.view(np.int32) == ref.view(np.int32)).all(), (got, ref)
    # the weights do change the fit (the transformation's centre and scale)
    assert not (got.view(np.int32) == plain.view(np.int32)).all()


def test_weighted_fit_unsupported_estimators(usac):
    pts, _ = synthetic.line_points(n=500, seed=2)
    with usac.Context(usac.ESTIMATOR.Line2d, pts) as ctx:
        with pytest.raises(usac.UsacError):
            ctx.lsq_fit(np.arange(50), np.ones(500, np.float32))
        ctx.lsq_fit(np.arange(50))  # unweighted still works
    pts, _, _ = synthetic.fundamental_points(n=500, seed=2, normalized=True, prosac_order=False)
    with usac.Context(usac.ESTIMATOR.Essential, pts) as ctx:
        with pytest.raises(usac.UsacError):
            ctx.lsq_fit(np.arange(50), np.ones(500, np.float32))
