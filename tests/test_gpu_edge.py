"""Edge cases of the whole loop against the oracle (ransac.cpp:14-238 semantics): NaN rows,
duplicated points, a point count that is not a multiple of the 4-point record groups, the
smallest sets, one iteration, a threshold nobody meets (USAC_ERR_NO_MODEL = the reference's
exit(111)), and many exactly tied scores (the record-candidate exact sums run in several
64-model launches)."""
import numpy as np
import pytest

from ransac_amd import synthetic

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.int32)


def _run(usac, oracle, kind, pts, thr, seed=5, max_iters=10000, lo=0, sampler="uniform"):
    okind, est, m = {"H": (oracle.HOMOGRAPHY, usac.ESTIMATOR.Homography, 4),
                     "F": (oracle.FUNDAMENTAL, usac.ESTIMATOR.Fundamental, 7),
                     "E": (oracle.ESSENTIAL, usac.ESTIMATOR.Essential, 5),
                     "L": (oracle.LINE2D, usac.ESTIMATOR.Line2d, 2)}[kind]
    ref = oracle.ransac_run(okind, pts, thr, 0.95, seed, max_iters=max_iters, lo=lo)
    mdl = usac.Model(thr, m, 0.95, 7, est, usac.SAMPLER.Uniform)
    mdl.ResetRandomGenerator(False)
    mdl.setSeed(seed)
    mdl.lo = usac.LocOpt(lo)
    mdl.max_iterations = max_iters
    mdl.batch = 512
    r = usac.Ransac(mdl, pts)
    err = None
    try:
        r.run()
    except usac.UsacError as e:
        err = e
    return ref, r, err


def _same(ref, r, err):
    if ref["ret"] != 0:
        assert err is not None and err.code == -111
        return
    assert err is None
    out = r.getRansacOutput()
    assert out.getNumberOfMainIterations() == ref["iters"]
    assert [(i, c) for i, c, _ in r.records] == [(i, c) for i, c, _ in ref["records"]]
    assert [np.float32(s) for _, _, s in r.records] == [np.float32(s) for _, _, s in ref["records"]]
    assert (_bits(out.getModel()) == _bits(ref["model"])).all()
    assert (out.getInliers() == ref["inlier_idx"]).all()


def _points(kind, n, ratio, seed):
    if kind == "H":
        return synthetic.homography_points(n=n, inlier_ratio=ratio, seed=seed)[0], 2.0
    if kind == "F":
        return synthetic.fundamental_points(n=n, inlier_ratio=ratio, seed=seed, prosac_order=False)[0], 2.0
    return synthetic.fundamental_points(n=n, inlier_ratio=ratio, seed=seed, normalized=True,
                                        prosac_order=False)[0], 0.002


@pytest.mark.parametrize("kind", ["H", "F", "E"])
def test_nan_rows(usac, oracle, kind):
    pts, thr = _points(kind, 2001, 0.4, 3)
    pts = pts.copy()
    rng = np.random.default_rng(1)
    pts[rng.choice(len(pts), 100, replace=False), rng.integers(0, 4, 100)] = np.nan
    _same(*_run(usac, oracle, kind, pts, thr, lo=1, max_iters=3000))


def test_duplicated_points_and_odd_count(usac, oracle):
    pts, _, _ = synthetic.homography_points(n=1203, inlier_ratio=0.4, seed=4)
    pts = np.concatenate([pts, pts[:400], pts[:7]])  # exact duplicates, n = 1610 (not % 4)
    _same(*_run(usac, oracle, "H", pts, 2.0))


@pytest.mark.parametrize("n", [4, 5, 9])
def test_smallest_sets(usac, oracle, n):
    pts, _, _ = synthetic.homography_points(n=n, inlier_ratio=1.0, seed=n)
    _same(*_run(usac, oracle, "H", pts, 2.0, max_iters=50))


@pytest.mark.parametrize("kind,n", [("F", 7), ("F", 8), ("E", 5), ("E", 6)])
def test_smallest_sets_two_view(usac, oracle, kind, n):
    pts, thr = _points(kind, n, 1.0, n)
    _same(*_run(usac, oracle, kind, pts, thr, max_iters=50))


def test_one_iteration(usac, oracle):
    pts, _, _ = synthetic.homography_points(n=1000, inlier_ratio=0.5, seed=6)
    _same(*_run(usac, oracle, "H", pts, 2.0, max_iters=1))


def test_no_inliers_is_exit_111(usac, oracle):
    pts, _ = synthetic.line_points(n=500, inlier_ratio=0.3, seed=2)
    pts = pts.copy()
    pts[::2, 1] += 0.5  # nobody within 1e-30 of any line through two points... except the pair
    ref, r, err = _run(usac, oracle, "L", pts, 1e-30, max_iters=200)
    _same(ref, r, err)


def test_many_tied_scores(usac, oracle):
    """random points, a tiny threshold: almost every line hypothesis counts exactly its own two
    points, so nearly every slot ties the running best and the record-candidate exact sums run
    in many 64-model launches (Score::bigger then decides on the larger sum)"""
    rng = np.random.default_rng(9)
    pts = rng.uniform(0, 1000, (300, 2)).astype(np.float32)
    ref, r, err = _run(usac, oracle, "L", pts, 0.002, max_iters=2000)
    _same(ref, r, err)
    assert r.getRansacOutput().raw["sum_models"] > 64
