"""NAPSAC (grid neighbours) and LO-RANSAC -- CPU oracle checks.

Pins: the grid neighbour lists equal a brute-force restatement of
nearest_neighbors.cpp:160-202 (same 4-D cell, other points, ascending index); every NAPSAC
sample lies in one cell; LO never lowers the best score it is given and reports its
iteration counters like RansacOutput::getLOIters."""
import numpy as np
import pytest

from ransac_amd import synthetic


def test_grid_neighbors_brute_force(oracle):
    pts, _, _ = synthetic.homography_points(n=3000, inlier_ratio=0.3, seed=4, cluster=(400, 600, 120))
    nb = oracle.grid_neighbors(pts, 50)
    cells = (pts / np.float32(50)).astype(np.int32)  # fp32 division, truncation
    keys = {}
    for i, c in enumerate(map(tuple, cells)):
        keys.setdefault(c, []).append(i)
    for i, c in enumerate(map(tuple, cells)):
        want = [j for j in keys[c] if j != i]
        assert nb[i].tolist() == want
    assert max(len(x) for x in nb) > 10


def test_napsac_samples_share_a_cell(oracle, usac):
    pts, _, _ = synthetic.homography_points(n=3000, inlier_ratio=0.3, seed=5, cluster=(400, 600, 120))
    r = oracle.ransac_run(oracle.HOMOGRAPHY, pts, 2.0, 0.95, 1, sampler=oracle.SAMPLER_NAPSAC, max_iters=300)
    assert r["ret"] == 0
    # the loop consumed only cell-local samples: rebuild them through the oracle sampler
    cells = (pts / np.float32(50)).astype(np.int32)
    import ctypes
    L = oracle.lib()
    L.orc_grid_new.restype = ctypes.c_void_p
    L.orc_grid_new.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_uint, ctypes.c_int]
    L.orc_napsac_new.restype = ctypes.c_void_p
    L.orc_napsac_new.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_uint]
    L.orc_napsac_sample.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
    L.orc_napsac_free.argtypes = [ctypes.c_void_p]
    L.orc_grid_free.argtypes = [ctypes.c_void_p]
    g = L.orc_grid_new(pts.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), len(pts), 50)
    s = L.orc_napsac_new(g, len(pts), 4)
    L.orc_srandom(ctypes.c_uint(7))
    smp = np.zeros(4, np.int32)
    for _ in range(500):
        L.orc_napsac_sample(s, smp.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
        assert len(set(smp.tolist())) == 4
        assert (cells[smp] == cells[smp[0]]).all()
    L.orc_napsac_free(s)
    L.orc_grid_free(g)


@pytest.mark.parametrize("lo", [1, 2])
def test_lo_improves_and_counts(oracle, lo):
    pts, H, inl = synthetic.homography_points(n=4000, inlier_ratio=0.2, seed=6, cluster=(500, 500, 150))
    a = oracle.ransac_run(oracle.HOMOGRAPHY, pts, 2.0, 0.95, 3)
    b = oracle.ransac_run(oracle.HOMOGRAPHY, pts, 2.0, 0.95, 3, lo=lo)
    assert b["ret"] == 0 and b["lo_inner_iters"] > 0
    # LO runs inside the loop: the best minimal score it hands to the polish is never lower
    assert b["minimal_inliers"] >= a["records"][0][1]
    assert b["inliers"] >= 0.95 * a["inliers"]


def test_grid_csr_restatement_matches_oracle(oracle):
    """The numpy CSR the device grid is checked against (tests/helpers/grid_ref.py) gives every
    point the oracle's neighbour list (orc_grid), negative coordinates included."""
    from ransac_amd import synthetic
    from tests.helpers.grid_ref import grid_csr

    pts, _, _ = synthetic.homography_points(n=6000, inlier_ratio=0.2, seed=3, cluster=(500, 500, 150))
    pts[::4, 1] -= 800.0
    for cs in (50, 9):
        g = grid_csr(pts, cs, 4)
        lists = oracle.grid_neighbors(pts, cs)
        for i in range(len(pts)):
            c = g["cell"][i]
            mem = g["members"][g["start"][c]:g["start"][c + 1]]
            assert g["members"][g["start"][c] + g["rank"][i]] == i
            np.testing.assert_array_equal(mem[mem != i], lists[i])
        assert (np.array([len(x) for x in lists])[g["eligible"]] >= 4).all()
