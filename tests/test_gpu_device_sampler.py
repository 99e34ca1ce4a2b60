"""Device sampler of the throughput batches: uniform draws are distinct and in range; the
PROSAC schedule matches the reference's ProsacSampler (oracle restatement, mt19937) subset
by subset -- the last point of every sample is the subset's last point, the others lie
before it -- and turns uniform after T_N = 200000 hypotheses (prosac_sampler.hpp:117-172)."""
import numpy as np
import pytest

from ransac_amd import synthetic

pytestmark = pytest.mark.gpu


def _check_distinct(s, n):
    assert (s >= 0).all() and (s < n).all()
    srt = np.sort(s, axis=1)
    assert (np.diff(srt, axis=1) > 0).all()


@pytest.mark.parametrize("kind", ["H", "F", "E", "L"])
def test_uniform_device_samples(usac, kind):
    if kind == "L":
        pts, _ = synthetic.line_points(n=1000, seed=3)
        est = usac.ESTIMATOR.Line2d
    else:
        pts, _, _ = synthetic.fundamental_points(n=3000, seed=3) if kind != "H" else \
            synthetic.homography_points(n=3000, seed=3)
        est = {"H": usac.ESTIMATOR.Homography, "F": usac.ESTIMATOR.Fundamental, "E": usac.ESTIMATOR.Essential}[kind]
    with usac.Context(est, pts) as ctx:
        s = ctx.draw_samples(65536, seed=11, first_hyp=123)
        _check_distinct(s, len(pts))
        again = ctx.draw_samples(100, seed=11, first_hyp=123 + 5)
        np.testing.assert_array_equal(again, s[5:105])  # keyed by (seed, global hypothesis index)


def test_prosac_device_schedule(usac, oracle):
    pts, _, _ = synthetic.fundamental_points(n=10000, inlier_ratio=0.3, seed=2)  # quality-sorted
    m, n = 7, len(pts)
    ref, _, _ = oracle.prosac_samples(5, n, m, 20000)
    with usac.Context(usac.ESTIMATOR.Fundamental, pts) as ctx:
        ctx.set_device_sampler(usac.SAMPLER.Prosac)
        s = ctx.draw_samples(20000, seed=9, first_hyp=0)
        np.testing.assert_array_equal(s[:, m - 1], ref[:, m - 1])  # the subset schedule
        assert (s[:, : m - 1] < s[:, m - 1:]).all()
        _check_distinct(s, n)
        late = ctx.draw_samples(4096, seed=9, first_hyp=200000)  # past T_N: uniform
        _check_distinct(late, n)
        assert late.max() > n // 2
        # the throughput path uses the same stream: batch of 65536 with PROSAC still scores
        c, _, best = ctx.hypothesize_score(B=65536, seed=9, first_hyp=0, thr=2.0)
        assert best["inliers"] > 0 and (c >= -1).all()
