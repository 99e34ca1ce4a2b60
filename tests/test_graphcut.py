"""Graph-cut LO -- CPU oracle checks.

Pins: the oracle's Boykov-Kolmogorov restatement (orc_bk_*) equals the reference's own
vendored gco-v3.0 max-flow (include/gco-v3.0/energy.h + maxflow.inl, compiled from
/root/reference into oracle/_ref/libgco_ref.so by oracle/Makefile) on random graphs and on the
GraphCut::labeling energies of real scenes: identical SINK labels and flow bits.  Without
oracle/_ref (no reference checkout) those comparisons are skipped.  The GC-LO loop
(graphcut.hpp:99-153) never lowers the best score and reports its counters."""
import numpy as np
import pytest

from ransac_amd import synthetic


def _random_problem(rng, n, m, quant):
    unary = rng.uniform(0, 1, n).astype(np.float32)
    if quant:
        unary = (np.round(unary * quant) / quant).astype(np.float32)  # many equal capacities
    ei = rng.integers(0, n, m).astype(np.int32)
    ej = rng.integers(0, n, m).astype(np.int32)
    keep = ei != ej
    ei, ej = ei[keep], ej[keep]
    lam = np.float32(0.1)
    e1, e2 = unary[ei], unary[ej]
    e00 = ((e1 + e2) / np.float32(2)).astype(np.float32)
    e11 = (np.float32(1) - e00).astype(np.float32)
    one = np.ones_like(e00)
    return unary, ei, ej, e00 * lam, one * lam, one * lam, e11 * lam


def _gc_energies(pts, model, thr, nbrs):
    """GraphCut::labeling's terms (graphcut.cpp:17-75) in numpy float32, exp in double."""
    from oracle import oracle as O
    est = O.Estimator(O.HOMOGRAPHY, pts, O.DLT_THIN)
    err = est.errors(model)
    sqr = np.float32(2) * np.float32(thr) * np.float32(thr)
    en = np.exp((-(err * err) / sqr).astype(np.float64)).astype(np.float32)
    ei, ej = [], []
    for i, row in enumerate(nbrs):
        for j in row:
            if j != i and j >= 0:
                ei.append(i)
                ej.append(j)
    ei, ej = np.array(ei, np.int32), np.array(ej, np.int32)
    e00 = ((en[ei] + en[ej]) / np.float32(2)).astype(np.float32)
    e11 = (np.float32(1) - e00).astype(np.float32)
    ok = ~((e00 + e11 > np.float32(2)) | np.isnan(e00))
    ei, ej, e00, e11 = ei[ok], ej[ok], e00[ok], e11[ok]
    lam = np.float32(0.1)
    one = np.ones_like(e00)
    return en, ei, ej, e00 * lam, one * lam, one * lam, e11 * lam


@pytest.mark.parametrize("seed,n,m,quant", [(1, 50, 200, 0), (2, 300, 2000, 0), (3, 300, 2000, 8), (4, 2000, 14000, 0),
                                            (5, 2000, 14000, 16), (6, 10, 0, 0)])
def test_bk_matches_gco_reference_random(oracle, seed, n, m, quant):
    if not oracle.gco_ref_available():
        pytest.skip("oracle/_ref/libgco_ref.so not built (no /root/reference)")
    prob = _random_problem(np.random.default_rng(seed), n, m, quant)
    lab, flow = oracle.bk_label(*prob)
    rlab, rflow = oracle.gco_ref_label(*prob)
    assert (lab == rlab).all()
    assert np.float32(flow).view(np.int32) == np.float32(rflow).view(np.int32)


@pytest.mark.parametrize("neigh", ["knn", "grid"])
def test_bk_matches_gco_reference_gc_energies(oracle, homography_scenes, neigh):
    if not oracle.gco_ref_available():
        pytest.skip("oracle/_ref/libgco_ref.so not built (no /root/reference)")
    for scene in ("adam", "boat", "graf"):
        pts, model, _ = homography_scenes[scene]
        est = oracle.Estimator(oracle.HOMOGRAPHY, pts)
        inv = np.linalg.inv(model.reshape(3, 3).astype(np.float64)).astype(np.float32).reshape(-1)
        if est.quality(inv, 2.0)[0] > est.quality(model, 2.0)[0]:  # GetImage.h:209-231 direction
            model = inv
        if neigh == "knn":
            nbrs, _ = oracle.knn(pts, 7)
        else:
            nbrs = oracle.grid_neighbors(pts, 50)
        prob = _gc_energies(pts, model, 2.0, nbrs)
        lab, flow = oracle.bk_label(*prob)
        rlab, rflow = oracle.gco_ref_label(*prob)
        assert (lab == rlab).all(), scene
        assert lab.sum() > 10
        assert np.float32(flow).view(np.int32) == np.float32(rflow).view(np.int32)


@pytest.mark.parametrize("neigh", ["knn", "grid"])
def test_gc_lo_loop(oracle, neigh):
    pts, _, _ = synthetic.homography_points(n=3000, inlier_ratio=0.3, seed=7, cluster=(500, 500, 200))
    nb = oracle.NEIGHBORS_NANOFLANN if neigh == "knn" else oracle.NEIGHBORS_GRID
    base = oracle.ransac_run(oracle.HOMOGRAPHY, pts, 2.0, 0.95, 5, max_iters=2000)
    r = oracle.ransac_run(oracle.HOMOGRAPHY, pts, 2.0, 0.95, 5, max_iters=2000, lo=oracle.LO_GC, neighbors=nb, knn=7)
    assert r["ret"] == 0
    assert r["lo_iterative_iters"] >= 1          # labelings
    assert r["minimal_inliers"] >= max(c for _, c, _ in r["records"])
    assert r["iters"] <= base["iters"]


def test_gc_rejects_napsac(oracle):
    pts, _, _ = synthetic.homography_points(n=500, inlier_ratio=0.3, seed=7)
    r = oracle.ransac_run(oracle.HOMOGRAPHY, pts, 2.0, 0.95, 5, sampler=oracle.SAMPLER_NAPSAC, lo=oracle.LO_GC)
    assert r["ret"] != 0


@pytest.mark.parametrize("seed,n,m,quant", [(1, 50, 200, 0), (3, 300, 2000, 8), (4, 2000, 14000, 0),
                                            (5, 2000, 14000, 16)])
def test_product_bk_matches_gco_reference(oracle, usac, seed, n, m, quant):
    """the product's host min cut (usac_maxflow.hpp via usac_bk_label) == the gco sources"""
    prob = _random_problem(np.random.default_rng(seed), n, m, quant)
    lab, flow = usac.bk_label(*prob)
    if oracle.gco_ref_available():
        rlab, rflow = oracle.gco_ref_label(*prob)
    else:
        rlab, rflow = oracle.bk_label(*prob)
    assert (lab == rlab).all()
    assert np.float32(flow).view(np.int32) == np.float32(rflow).view(np.int32)


def test_product_bk_gc_energies(oracle, usac, homography_scenes):
    for scene in ("adam", "boat", "graf", "city"):
        pts, model, _ = homography_scenes[scene]
        est = oracle.Estimator(oracle.HOMOGRAPHY, pts)
        inv = np.linalg.inv(model.reshape(3, 3).astype(np.float64)).astype(np.float32).reshape(-1)
        if est.quality(inv, 2.0)[0] > est.quality(model, 2.0)[0]:
            model = inv
        nbrs, _ = oracle.knn(pts, 7)
        prob = _gc_energies(pts, model, 2.0, nbrs)
        lab, _ = usac.bk_label(*prob)
        rlab, _ = (oracle.gco_ref_label if oracle.gco_ref_available() else oracle.bk_label)(*prob)
        assert (lab == rlab).all(), scene
