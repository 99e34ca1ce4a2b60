"""Contexts draw device memory, streams and events from process-wide pools (usac_api.cpp
DevPool / StreamPool): blocks are reused across contexts of different sizes, and a block
replaced by a larger one goes back only after the device drained.  Churn many contexts of
varying sizes, two alive at a time, and check every result against the oracle -- a block
handed out while still in use, or a stale size, would show up as a wrong count, sum or model."""
import numpy as np
import pytest

from ransac_amd import synthetic

pytestmark = pytest.mark.gpu


def test_context_churn_matches_oracle(usac, oracle):
    rng = np.random.default_rng(11)
    prev = None
    for it in range(24):
        n = int(rng.integers(40, 30000))
        pts, model, _ = synthetic.homography_points(n=n, inlier_ratio=0.4, seed=100 + it)
        est = oracle.Estimator(oracle.HOMOGRAPHY, pts)
        oc, os_, oidx = est.quality(model, 2.0, with_inliers=True)
        ctx = usac.Context(usac.ESTIMATOR.Homography, pts)
        try:
            c, s, idx = ctx.get_inliers(model, 2.0)
            assert c == oc and np.float32(s) == np.float32(os_)
            np.testing.assert_array_equal(idx, oidx)
            if len(oidx) >= 8:  # grows the context's fit buffers (reserve replaces smaller blocks)
                g = ctx.nonminimal(oidx)
                np.testing.assert_array_equal(g.view(np.int32), est.nonminimal(oidx).view(np.int32))
            samples = oracle.uniform_samples(it + 1, n, 4, 512)
            om, _ = est.estimate_batch(samples)
            ocnt, _ = est.score_models(om, 2.0)
            cnt, _, _ = ctx.hypothesize_score(samples=samples, thr=2.0)
            np.testing.assert_array_equal(cnt, ocnt)
        finally:
            if prev is not None:
                prev.close()
            prev = ctx
    prev.close()
