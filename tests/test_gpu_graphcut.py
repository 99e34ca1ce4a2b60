"""GPU parity of the loop with the graph-cut LO (graphcut.hpp:99-153, graphcut.cpp:7-101):
device residuals -> host energies and BK min cut -> batched device least-squares fits and
scores, against the oracle: iterations, records, GC counters (gc_iterations, labellings),
model bits and inlier list identical."""
import numpy as np
import pytest

from ransac_amd import synthetic

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.int32)


CASES = [("H", "knn", False, 3000), ("H", "grid", False, 3000), ("H", "knn", True, 3000), ("F", "knn", False, 2000),
         ("L", "knn", False, 1000), ("E", "knn", False, 1500), ("H", "knn", False, 20000)]


@pytest.mark.parametrize("kind,neigh,sprt,n", CASES)
def test_loop_gc_identical(usac, oracle, kind, neigh, sprt, n):
    if kind == "H":
        pts, _, _ = synthetic.homography_points(n=n, inlier_ratio=0.3, seed=7, cluster=(500, 500, 200))
        thr, okind, est, m = 2.0, oracle.HOMOGRAPHY, usac.ESTIMATOR.Homography, 4
    elif kind == "F":
        pts, _, _ = synthetic.fundamental_points(n=n, inlier_ratio=0.4, seed=7, prosac_order=False)
        thr, okind, est, m = 2.0, oracle.FUNDAMENTAL, usac.ESTIMATOR.Fundamental, 7
    elif kind == "E":
        pts, _, _ = synthetic.fundamental_points(n=n, inlier_ratio=0.5, seed=7, normalized=True, prosac_order=False)
        thr, okind, est, m = 0.002, oracle.ESSENTIAL, usac.ESTIMATOR.Essential, 5
    else:
        pts, _ = synthetic.line_points(n=n, inlier_ratio=0.3, seed=7)
        thr, okind, est, m = 8.0, oracle.LINE2D, usac.ESTIMATOR.Line2d, 2
    onb = oracle.NEIGHBORS_NANOFLANN if neigh == "knn" else oracle.NEIGHBORS_GRID
    ref = oracle.ransac_run(okind, pts, thr, 0.95, 5, sprt=sprt, lo=oracle.LO_GC, max_iters=3000, neighbors=onb, knn=7)
    mdl = usac.Model(thr, m, 0.95, 7, est, usac.SAMPLER.Uniform)
    mdl.ResetRandomGenerator(False)
    mdl.setSeed(5)
    mdl.setSprt(sprt)
    mdl.lo = usac.LocOpt.GC
    mdl.max_iterations = 3000
    mdl.batch = 512
    mdl.setNeighborsType(usac.NeighborsSearch.Nanoflann if neigh == "knn" else usac.NeighborsSearch.Grid)
    r = usac.Ransac(mdl, pts)
    r.run()
    out = r.getRansacOutput()
    assert out.getNumberOfMainIterations() == ref["iters"]
    assert [(i, c) for i, c, _ in r.records] == [(i, c) for i, c, _ in ref["records"]]
    assert [np.float32(s) for _, _, s in r.records] == [np.float32(s) for _, _, s in ref["records"]]
    assert out.getLOIters() == ref["lo_inner_iters"]
    assert out.raw["lo_iterative_iters"] == ref["lo_iterative_iters"]
    assert (_bits(out.raw["minimal_model"]) == _bits(ref["minimal_model"])).all()
    assert (_bits(out.getModel()) == _bits(ref["model"])).all()
    assert (out.getInliers() == ref["inlier_idx"]).all()
