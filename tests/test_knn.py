"""KNN neighbours and the NAPSAC KNN sampler -- CPU oracle checks.

Pins: orc_knn equals a numpy brute force of nanoflann's float L2 distance
(nearest_neighbors.cpp:69-128 via nanoflann L2_Adaptor::evalMetric: ((d0^2 + d1^2) + d2^2) +
d3^2 in float, self excluded, ascending distance; equal distances by ascending index --
nanoflann's own tie order follows its KD-tree and is unpinned); the NAPSAC KNN sampler walks
the neighbour row from the farthest backwards, cyclically (napsac_sampler.hpp:76-98), with the
initial point from the glibc ArrayRandomGenerator pool -- restated here in Python over libc's
random()."""
import ctypes

import numpy as np
import pytest

from ransac_amd import synthetic


def brute_knn(pts, k):
    pts = np.asarray(pts, np.float32)
    n, cols = pts.shape
    idx = np.full((n, k), -1, np.int32)
    d2 = np.full((n, k), np.inf, np.float32)
    for p in range(n):
        d = pts[p] - pts
        if cols == 4:
            r = ((d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]) + d[:, 3] * d[:, 3]
        else:
            r = d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]
        r = r.astype(np.float32)
        r[p] = np.nan
        order = [j for j in np.argsort(r, kind="stable") if not np.isnan(r[j])][:k]
        idx[p, : len(order)] = order
        d2[p, : len(order)] = r[order]
    return idx, d2


@pytest.mark.parametrize("cols,k", [(4, 7), (4, 1), (2, 5), (2, 13), (4, 32)])
def test_knn_brute_force(oracle, cols, k):
    rng = np.random.default_rng(cols * 100 + k)
    pts = rng.uniform(0, 50, (400, cols)).astype(np.float32)
    pts[10:20] = pts[0]          # exact duplicates: distance-0 ties, ascending index
    pts[30:40] = np.round(pts[30:40])  # many equal distances
    idx, d2 = oracle.knn(pts, k)
    bi, bd = brute_knn(pts, k)
    assert (idx == bi).all()
    assert (d2.view(np.int32) == bd.view(np.int32)).all()


def test_knn_fewer_points_than_k(oracle):
    pts = np.arange(20, dtype=np.float32).reshape(5, 4)
    idx, d2 = oracle.knn(pts, 7)
    assert (idx[:, 4:] == -1).all() and np.isinf(d2[:, 4:]).all()
    assert sorted(idx[0, :4].tolist()) == [1, 2, 3, 4]


def test_napsac_knn_sampler_walk(oracle):
    """oracle loop samples == a Python restatement of generateSampleKNN over libc random()."""
    pts, _, _ = synthetic.homography_points(n=600, inlier_ratio=0.3, seed=3, cluster=(400, 600, 120))
    knn = 7
    nb, _ = oracle.knn(pts, knn)
    libc = ctypes.CDLL("libc.so.6")
    libc.random.restype = ctypes.c_long
    libc.srandom(9)
    n, m = len(pts), 4
    arr = list(range(n))
    mx = 0
    nxt = [0] * n
    want = []
    for _ in range(50):
        if mx == 0:
            mx = n
        r = libc.random() % mx
        init = arr[r]
        mx -= 1
        arr[r], arr[mx] = arr[mx], init
        smp = [init]
        for _i in range(1, m):
            smp.append(int(nb[init, nxt[init] + knn - 1]))
            nxt[init] -= 1
            if nxt[init] == -knn:
                nxt[init] = 0
        want.append(smp)
    # the sampler's draws are the loop's first samples: the first record's sample is sample 0
    L = oracle.lib()
    L.orc_napsac_knn_new.restype = ctypes.c_void_p
    L.orc_napsac_knn_new.argtypes = [ctypes.POINTER(ctypes.c_int32), ctypes.c_uint, ctypes.c_uint, ctypes.c_uint]
    L.orc_napsac_knn_sample.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32)]
    L.orc_napsac_knn_free.argtypes = [ctypes.c_void_p]
    nbc = np.ascontiguousarray(nb)
    s = L.orc_napsac_knn_new(nbc.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), n, m, knn)
    libc.srandom(9)
    got = []
    buf = np.zeros(m, np.int32)
    for _ in range(50):
        L.orc_napsac_knn_sample(s, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
        got.append(buf.tolist())
    L.orc_napsac_knn_free(s)
    assert got == want


def test_napsac_knn_loop_runs(oracle):
    pts, _, _ = synthetic.homography_points(n=2000, inlier_ratio=0.2, seed=7, cluster=(500, 500, 150))
    r = oracle.ransac_run(oracle.HOMOGRAPHY, pts, 2.0, 0.95, 5, sampler=oracle.SAMPLER_NAPSAC, lo=1, max_iters=3000,
                          neighbors=oracle.NEIGHBORS_NANOFLANN, knn=7)
    assert r["ret"] == 0 and r["inliers"] > 300
