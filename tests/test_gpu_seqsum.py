"""The reference's sequential fp32 sums evaluated in parallel (kernels_seqsum.hip): bit-equal
to the left-to-right sum whatever the data -- long chains (segments of up to 31 k elements),
values whose running sum drifts far outside the candidate window (the sequential fall-back),
constant addends (systematic rounding drift), denormals, huge dynamic range.

Σerr: Quality::getNumberInliers (quality.hpp:85) through usac_get_inliers on a line context
with the model (0, 1, 0), whose residual |0 x + 1 y + 0| is |y| -- so the residual sequence is
any list of non-negative floats we choose; the expected sum is numpy's float32
add.accumulate (sequential).  The means / average distances of NormalizedDLT
(normalizing_transformation.cpp:7-113) through usac_nonminimal against the oracle's
sequential C loop, at sizes where the chains span many segments."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _seq_sum(v):
    v = np.ascontiguousarray(v, dtype=np.float32)
    return np.float32(0) if v.size == 0 else np.add.accumulate(v, dtype=np.float32)[-1]


def _residual_sum(usac, errs, seed=0):
    rng = np.random.default_rng(seed)
    pts = np.stack([rng.uniform(-500, 500, errs.size).astype(np.float32), errs.astype(np.float32)], 1)
    with usac.Context(usac.ESTIMATOR.Line2d, np.ascontiguousarray(pts)) as ctx:
        c, s, idx = ctx.get_inliers(np.array([0, 1, 0], np.float32), 3.0e38)
    assert c == errs.size
    return np.float32(s)


@pytest.mark.parametrize("n", [1, 255, 256, 257, 8191, 17000, 100003, 1000003])
def test_residual_sum_uniform(usac, n):
    rng = np.random.default_rng(n)
    errs = rng.uniform(0, 2, n).astype(np.float32)
    assert _residual_sum(usac, errs).view(np.int32) == _seq_sum(errs).view(np.int32)


@pytest.mark.parametrize("kind", ["constant", "lognormal", "denormal", "mixed_scale", "zeros", "sorted_desc"])
def test_residual_sum_adversarial(usac, kind):
    rng = np.random.default_rng(7)
    n = 60000
    if kind == "constant":  # every add rounds the same way: the drift grows linearly
        errs = np.full(n, 0.1, np.float32)
    elif kind == "lognormal":  # values over ~30 decades: most segments miss the window
        errs = np.exp(rng.normal(0, 16, n)).astype(np.float32)
        errs = errs[np.isfinite(errs)]
    elif kind == "denormal":
        errs = (rng.uniform(0, 1, n) * 1e-40).astype(np.float32)
    elif kind == "mixed_scale":  # long runs absorbed by a huge running sum, then tiny ones
        errs = np.concatenate([np.full(5000, 1e20, np.float32), rng.uniform(0, 1, n - 5000).astype(np.float32)])
    elif kind == "zeros":
        errs = np.zeros(n, np.float32)
    else:
        errs = np.sort(rng.uniform(0, 1000, n).astype(np.float32))[::-1].copy()
    assert _residual_sum(usac, errs).view(np.int32) == _seq_sum(errs).view(np.int32)


@pytest.mark.parametrize("n", [5000, 40000, 65536, 65537, 200000])
def test_normalization_long_chains(usac, oracle, n):
    """NormalizedDLT on n correspondences: its four coordinate means and two distance sums are
    sequential chains of n elements (up to 32 segments of 6 k); model bits = the oracle's.
    65536 / 65537: either side of the fused gather + segment-sum kernel's limit
    (kernels_nonmin.hip kFusedGatherMax)."""
    rng = np.random.default_rng(n)
    x1 = rng.uniform(0, 4000, (n, 2))
    H = np.array([[1.1, 0.05, 30.0], [-0.04, 0.95, -12.0], [1e-5, -2e-5, 1.0]])
    p = np.c_[x1, np.ones(n)] @ H.T
    x2 = p[:, :2] / p[:, 2:] + rng.normal(0, 0.5, (n, 2))
    pts = np.ascontiguousarray(np.c_[x1, x2], dtype=np.float32)
    idx = rng.permutation(n).astype(np.int32) if n % 2 else np.arange(n, dtype=np.int32)
    est = oracle.Estimator(oracle.HOMOGRAPHY, pts)
    o = est.nonminimal(idx)
    with usac.Context(usac.ESTIMATOR.Homography, pts) as ctx:
        g = ctx.nonminimal(idx)
        g2 = ctx.nonminimal(idx[::-1].copy())  # another order: another chain
    np.testing.assert_array_equal(g.view(np.int32), o.view(np.int32))
    np.testing.assert_array_equal(g2.view(np.int32), est.nonminimal(idx[::-1].copy()).view(np.int32))


@pytest.mark.parametrize("kind", ["signed", "integer", "half_integer", "around_zero", "binade_edges"])
def test_normalization_chains_adversarial(usac, oracle, kind):
    """The mean / distance chains of NormalizedDLT on data that defeats the binade-piece
    speculation (kernels_seqsum.hip): mixed-sign coordinates whose running sums wander across
    zero, integer and half-integer coordinates (ties at every ulp the running sum reaches),
    sums parked at powers of two.  The device must still equal the oracle's sequential loops."""
    rng = np.random.default_rng(11)
    n = 40000
    if kind == "signed":
        x1 = rng.uniform(-2000, 2000, (n, 2))
    elif kind == "integer":
        x1 = rng.integers(0, 4000, (n, 2)).astype(np.float64)
    elif kind == "half_integer":
        x1 = rng.integers(0, 8000, (n, 2)) / 2.0
    elif kind == "around_zero":  # +-v pairs: the running sum keeps returning to ~0
        a = rng.uniform(0, 1000, (n // 2, 2))
        x1 = np.empty((n, 2))
        x1[0::2], x1[1::2] = a, -a + rng.normal(0, 1e-3, a.shape)
    else:  # 2^k-valued coordinates: the sums sit on binade edges
        x1 = 2.0 ** rng.integers(0, 12, (n, 2)).astype(np.float64)
    H = np.array([[1.1, 0.05, 30.0], [-0.04, 0.95, -12.0], [1e-5, -2e-5, 1.0]])
    p = np.c_[x1, np.ones(n)] @ H.T
    x2 = p[:, :2] / p[:, 2:] + rng.normal(0, 0.5, (n, 2))
    pts = np.ascontiguousarray(np.c_[x1, x2], dtype=np.float32)
    idx = np.arange(n, dtype=np.int32)
    est = oracle.Estimator(oracle.HOMOGRAPHY, pts)
    with usac.Context(usac.ESTIMATOR.Homography, pts) as ctx:
        for sub in (idx, idx[: n // 3], idx[::-1].copy()):
            g = ctx.nonminimal(sub)
            np.testing.assert_array_equal(g.view(np.int32), est.nonminimal(sub).view(np.int32), err_msg=kind)


@pytest.mark.parametrize("kind", ["integer", "half_ulp", "powers_of_two"])
def test_residual_sum_ties(usac, kind):
    """Σerr chains whose addends are exact ties at the running sum's ulp (integers, 0.5s, powers
    of two): rounding then depends on the parity of the running value -- the walk's job."""
    rng = np.random.default_rng(3)
    n = 50000
    if kind == "integer":
        errs = rng.integers(0, 4, n).astype(np.float32)
    elif kind == "half_ulp":
        errs = (rng.integers(0, 8, n) * 0.5 + 2 ** -6).astype(np.float32)
    else:
        errs = (2.0 ** rng.integers(-8, 3, n)).astype(np.float32)
    assert _residual_sum(usac, errs).view(np.int32) == _seq_sum(errs).view(np.int32)
