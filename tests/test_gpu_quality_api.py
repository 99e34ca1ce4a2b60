"""Quality::getNumberInliers through usac_score_models is never an SPRT test
(quality.hpp:60-101): a context whose throughput batches run the SPRT (usac_set_sprt) still
returns exact counts and sequential sums for every model, for every estimator."""
import numpy as np
import pytest

from ransac_amd import synthetic

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind", ["H", "L", "F"])
def test_score_models_ignores_batch_sprt(usac, oracle, kind):
    if kind == "H":
        pts, _, _ = synthetic.homography_points(n=3000, inlier_ratio=0.3, seed=4)
        okind, est, m, thr = oracle.HOMOGRAPHY, usac.ESTIMATOR.Homography, 4, 2.0
    elif kind == "L":
        pts, _ = synthetic.line_points(n=2000, inlier_ratio=0.3, seed=4)
        okind, est, m, thr = oracle.LINE2D, usac.ESTIMATOR.Line2d, 2, 8.0
    else:
        pts, _, _ = synthetic.fundamental_points(n=2000, inlier_ratio=0.4, seed=4, prosac_order=False)
        okind, est, m, thr = oracle.FUNDAMENTAL, usac.ESTIMATOR.Fundamental, 7, 2.0
    o = oracle.Estimator(okind, pts)
    samples = oracle.uniform_samples(3, len(pts), m, 512)
    models, nm = o.estimate_batch(samples)
    models = (models[:, 0] if models.ndim == 3 else models)[nm > 0]
    assert len(models) > 50
    oc, osum = o.score_models(models, thr)
    with usac.Context(est, pts, device=0) as ctx:
        ctx.set_sprt(True, seed=1)
        c, s = ctx.score_models(models, thr)
        # the batch SPRT is still on for hypothesize_* afterwards
        _, _, best = ctx.hypothesize_score(samples=samples[:64], thr=thr)
    assert (c == oc).all() and (c >= 0).all()
    assert (np.asarray(s, np.float32).view(np.int32) == osum.view(np.int32)).all()
