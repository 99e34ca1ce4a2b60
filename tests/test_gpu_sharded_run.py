"""Hypothesis-sharded Ransac::run (usac_ransac_run_sharded): two fresh child
processes share the GPU, each solving and scoring half of every batch, with the per-batch
all-gather over gloo; both ranks' outputs -- iterations, best-score records, LO counters, SPRT
rejections / histories, model bits, inlier list -- must equal the single-rank run's.  With SPRT
each rank computes the pool-order inlier words of its slice and every rank replays the
sequential SPRT walk over the gathered words."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from ransac_amd import synthetic

HERE = os.path.dirname(os.path.abspath(__file__))


def make_case(usac, case):
    if case == "h_napsac_lo":  # cfg5 shape at reduced size: clustered inliers, NAPSAC grid, LO-RANSAC
        pts, _, _ = synthetic.homography_points(n=20000, inlier_ratio=0.2, seed=11, cluster=(500, 500, 150))
        mdl = usac.Model(2.0, 4, 0.95, 7, usac.ESTIMATOR.Homography, usac.SAMPLER.Napsac)
        mdl.setNeighborsType(usac.NeighborsSearch.Grid)
        mdl.lo = usac.LocOpt.InItLORsc
    elif case == "e_uniform":  # cfg4 shape at reduced size
        pts, _, _ = synthetic.fundamental_points(n=5000, inlier_ratio=0.5, seed=9, normalized=True,
                                                 prosac_order=False)
        mdl = usac.Model(0.002, 5, 0.95, 7, usac.ESTIMATOR.Essential, usac.SAMPLER.Uniform)
    elif case == "f_prosac_sprt":  # cfg3 shape at reduced size: F 7-pt + PROSAC + SPRT
        pts, _, _ = synthetic.fundamental_points(n=4000, inlier_ratio=0.3, seed=4, prosac_order=True)
        mdl = usac.Model(2.0, 7, 0.99, 7, usac.ESTIMATOR.Fundamental, usac.SAMPLER.Prosac)
        mdl.setSprt(True)
    elif case == "h_uniform_sprt":  # homography + Uniform + SPRT (unlisted slots)
        pts, _, _ = synthetic.homography_points(n=5000, inlier_ratio=0.15, seed=8)
        mdl = usac.Model(2.0, 4, 0.99, 7, usac.ESTIMATOR.Homography, usac.SAMPLER.Uniform)
        mdl.setSprt(True)
    else:  # "f_gc": fundamental, uniform, graph-cut LO with KNN neighbours
        pts, _, _ = synthetic.fundamental_points(n=3000, inlier_ratio=0.4, seed=5, prosac_order=False)
        mdl = usac.Model(2.0, 7, 0.95, 7, usac.ESTIMATOR.Fundamental, usac.SAMPLER.Uniform)
        mdl.lo = usac.LocOpt.GC
    mdl.ResetRandomGenerator(False)
    mdl.setSeed(3)
    mdl.max_iterations = 3000
    mdl.batch = 1000  # several batches, each split 500 / 500 across the two ranks
    if case.endswith("_sprt"):
        mdl.batch = 250  # SPRT runs end early: still several batches (125 / 125 samples per rank)
    return pts, mdl


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["h_napsac_lo", "e_uniform", "f_gc", "f_prosac_sprt", "h_uniform_sprt"])
def test_sharded_run_equals_single_rank(usac, tmp_path, case):
    pts, mdl = make_case(usac, case)
    r = usac.Ransac(mdl, pts)
    r.run()
    ref = r.getRansacOutput()
    port = _free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "helpers", "shard_child.py"), str(k), "2",
                               str(port), str(tmp_path / ("r%d.npz" % k)), case], env=env)
             for k in range(2)]
    for p in procs:
        assert p.wait(timeout=240) == 0
    for k in range(2):
        z = np.load(tmp_path / ("r%d.npz" % k))
        assert int(z["iters"]) == ref.getNumberOfMainIterations(), (k, case)
        assert int(z["lo"]) == ref.getLOIters()
        assert np.array_equal(z["records"], np.array(r.records, dtype=np.float64).reshape(-1, 3))
        assert (z["model"].view(np.int32) == np.asarray(ref.getModel(), np.float32).view(np.int32)).all()
        assert np.array_equal(z["inliers"], ref.getInliers())
        assert int(z["batches"]) == ref.raw["batches"]
        assert int(z["sprt_rejected"]) == ref.raw["sprt_rejected"]
        assert int(z["sprt_histories"]) == ref.raw["sprt_histories"]
    if case.endswith("_sprt"):  # the SPRT walk actually rejected models
        assert ref.raw["sprt_rejected"] > 0
    if case == "h_napsac_lo":  # LO chains split over the ranks: same rounds, the fits partitioned
        z = [np.load(tmp_path / ("r%d.npz" % k)) for k in range(2)]
        assert ref.raw["lo_fits"] > 0
        assert all(int(zk["lo_rounds"]) == ref.raw["lo_rounds"] for zk in z)
        assert sum(int(zk["lo_fits"]) for zk in z) == ref.raw["lo_fits"]
        assert all(int(zk["lo_fits"]) < ref.raw["lo_fits"] for zk in z)


@pytest.mark.gpu
def test_sharded_run_failing_gather_fails(usac):
    """A gather callback that raises fails the run (usac_last_error), never hangs it."""
    pts, mdl = make_case(usac, "e_uniform")
    r = usac.Ransac(mdl, pts)

    def bad(b):
        raise RuntimeError("peer lost")
    with pytest.raises(usac.UsacError):
        r.run(shard=(2, 0, bad))
