"""The reference's published statistics through the device library (usac_ransac_run): the
homography graph-cut runs of results/homography/uniform_gc*_Grid_c_sz_50.csv and the line2d
LO-RANSAC runs of results/line2d/uniform_100.csv, each run identical to the oracle's (the
CPU pins of tests/test_reference_statistics.py therefore carry over) and the averages within
the same statistical tolerance of the published ones."""
import numpy as np
import pytest

from test_reference_statistics import ERR, INL, SD_ERR, SD_INL, check, gt_error, gt_inliers, inl_floor

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.int32)


def _run(usac, pts, est, m, thr, p, seed, **kw):
    mdl = usac.Model(thr, m, p, kw.pop("knn", 7), est, kw.pop("sampler", usac.SAMPLER.Uniform))
    mdl.ResetRandomGenerator(False)
    mdl.setSeed(seed)
    mdl.setSprt(kw.pop("sprt", False))
    mdl.lo = kw.pop("lo", usac.LocOpt.NullLO)
    if "cell_size" in kw:
        mdl.setCellSize(kw.pop("cell_size"))
    if "neighbors" in kw:
        mdl.setNeighborsType(kw.pop("neighbors"))
    if "max_iterations" in kw:
        mdl.max_iterations = kw.pop("max_iterations")
    r = usac.Ransac(mdl, pts)
    r.run()
    return r.getRansacOutput()


@pytest.mark.parametrize("rel", ["homography/uniform_gc_Grid_c_sz_50.csv",
                                 "homography/uniform_gc_sprt_Grid_c_sz_50.csv"])
def test_homography_gc_statistics_device(usac, oracle, homography_scenes, rel):
    runs = 20
    sprt = "sprt" in rel
    results = {}
    for scene, (pts, model, _) in homography_scenes.items():
        est = oracle.Estimator(oracle.HOMOGRAPHY, pts)
        gt = gt_inliers(oracle, est, pts, model, 2.0)
        inl, err = [], []
        for seed in range(1, runs + 1):
            out = _run(usac, pts, usac.ESTIMATOR.Homography, 4, 2.0, 0.95, seed, lo=usac.LocOpt.GC,
                       neighbors=usac.NeighborsSearch.Grid, cell_size=50, sprt=sprt)
            ref = oracle.ransac_run(oracle.HOMOGRAPHY, pts, 2.0, 0.95, seed, lo=oracle.LO_GC,
                                    neighbors=oracle.NEIGHBORS_GRID, cell_size=50, sprt=sprt)
            assert out.getNumberOfMainIterations() == ref["iters"], (scene, seed)
            assert (_bits(out.getModel()) == _bits(ref["model"])).all(), (scene, seed)
            assert (out.getInliers() == ref["inlier_idx"]).all(), (scene, seed)
            inl.append(out.getNumberOfInliers())
            err.append(gt_error(est, out.getModel(), gt))
        results[scene] = {INL: inl, ERR: err}
    pinned = check(rel, results, [(INL, SD_INL), (ERR, SD_ERR)],
                   {INL: inl_floor, ERR: lambda m: max(0.002, 0.005 * m)})
    assert len(pinned) >= 21


def test_line2d_lo_statistics_device(usac, oracle, line2d_scenes):
    rel = "line2d/uniform_100.csv"
    results = {}
    for name, (pts, _, _) in sorted(line2d_scenes.items()):
        inl = []
        for seed in range(1, 11):
            out = _run(usac, pts, usac.ESTIMATOR.Line2d, 2, 10.0, 0.99, seed, lo=usac.LocOpt.InItLORsc)
            ref = oracle.ransac_run(oracle.LINE2D, pts, 10.0, 0.99, seed, lo=oracle.LO_INITLORSC)
            assert out.getNumberOfMainIterations() == ref["iters"], (name, seed)
            assert (_bits(out.getModel()) == _bits(ref["model"])).all(), (name, seed)
            inl.append(out.getNumberOfInliers())
        results[name] = {INL: inl}
    assert len(check(rel, results, [(INL, SD_INL)], {INL: inl_floor})) == 8


@pytest.mark.parametrize("rel,sprt", [("EVD/uniform_gc_Nanoflann_c_sz_50.csv", False),
                                      ("EVD/uniform_gc_sprt_Nanoflann_c_sz_50.csv", True)])
def test_evd_gc_knn_statistics_device(usac, oracle, rel, sprt):
    """results/EVD uniform graph-cut runs with KNN neighbours (device usac_knn, k = 7) through
    usac_ransac_run: every run identical to the oracle's, the averages within the pin tolerance."""
    import os
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "evd_scenes.npz"))
    results = {}
    for key in sorted(z.files):
        scene, pts = key[:-4], z[key]
        inl = []
        for seed in range(1, 11):
            ref = oracle.ransac_run(oracle.HOMOGRAPHY, pts, 2.0, 0.95, seed, max_iters=15000, sprt=sprt,
                                    lo=oracle.LO_GC, neighbors=oracle.NEIGHBORS_NANOFLANN, knn=7)
            if ref["ret"] != 0:  # no model (the reference's exit(111)): the device says so too
                with pytest.raises(usac.UsacError) as e:
                    _run(usac, pts, usac.ESTIMATOR.Homography, 4, 2.0, 0.95, seed, lo=usac.LocOpt.GC,
                         neighbors=usac.NeighborsSearch.Nanoflann, sprt=sprt, max_iterations=15000)
                assert e.value.code == -111
                inl.append(0)
                continue
            out = _run(usac, pts, usac.ESTIMATOR.Homography, 4, 2.0, 0.95, seed, lo=usac.LocOpt.GC,
                       neighbors=usac.NeighborsSearch.Nanoflann, sprt=sprt, max_iterations=15000)
            assert out.getNumberOfMainIterations() == ref["iters"], (scene, seed)
            assert (_bits(out.getModel()) == _bits(ref["model"])).all(), (scene, seed)
            assert (out.getInliers() == ref["inlier_idx"]).all(), (scene, seed)
            inl.append(out.getNumberOfInliers())
        results[scene] = {INL: inl}
    assert len(check(rel, results, [(INL, SD_INL)], {INL: inl_floor})) >= 14


def test_line2d_sprt_statistics_device(usac, oracle, line2d_scenes):
    """results/line2d/uniform_001.csv through usac_ransac_run: SPRT as sprt.hpp is written
    (shuffled, rolling pool), every run identical to the oracle's (iterations, model bits,
    inlier list), and the four I=200 scenes' averages inside the harness lens
    (test_line2d_sprt_statistics_current_pool; the file-order revision that reproduces all
    eight rows is an oracle switch only)."""
    from test_reference_statistics import ITS, STATS, lens_p
    rel = "line2d/uniform_001.csv"
    runs = int(STATS[rel]["settings"]["Runs for each image"])
    for name, (pts, _, _) in sorted(line2d_scenes.items()):
        if "I=200" not in name:
            continue
        inl, its = [], []
        for seed in range(1, 41):
            out = _run(usac, pts, usac.ESTIMATOR.Line2d, 2, 10.0, 0.99, seed, sprt=True)
            ref = oracle.ransac_run(oracle.LINE2D, pts, 10.0, 0.99, seed, sprt=True)
            assert out.getNumberOfMainIterations() == ref["iters"], (name, seed)
            assert (_bits(out.getModel()) == _bits(ref["model"])).all(), (name, seed)
            assert (out.getInliers() == ref["inlier_idx"]).all(), (name, seed)
            inl.append(out.getNumberOfInliers())
            its.append(out.getNumberOfMainIterations())
        row = STATS[rel]["scenes"][name]
        assert lens_p(inl, row, INL, runs) >= 0.005, name
        assert lens_p(its, row, ITS, runs) >= 0.005, name
