"""Timings of the widened rows on one GPU: device KNN at 100k points,
full USAC runs with NAPSAC-KNN + LO and with the graph-cut LO.  Prints one JSON object."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import ransac_amd as usac  # noqa: E402
from ransac_amd import synthetic  # noqa: E402


def knn_time(pts, k, reps=5):
    with usac.Context(usac.ESTIMATOR.Homography, pts, device=0) as ctx:
        ctx.knn(k)
        t = time.perf_counter()
        for _ in range(reps):
            ctx.knn(k, distances=False)
        return (time.perf_counter() - t) / reps * 1e3


def run(pts, sampler, lo, neigh, seeds):
    out = []
    for s in seeds:
        mdl = usac.Model(2.0, 4, 0.95, 7, usac.ESTIMATOR.Homography, sampler)
        mdl.ResetRandomGenerator(False)
        mdl.setSeed(s)
        mdl.lo = usac.LocOpt(lo)
        mdl.max_iterations = 5000
        mdl.setNeighborsType(neigh)
        r = usac.Ransac(mdl, pts)
        t = time.perf_counter()
        r.run()
        dt = time.perf_counter() - t
        o = r.getRansacOutput()
        out.append({"ms": dt * 1e3, "iters": o.getNumberOfMainIterations(), "inliers": o.getNumberOfInliers(),
                    "lo_iters": o.getLOIters(), "labelings_or_iterative": o.raw["lo_iterative_iters"],
                    "time_us": o.getTimeMicroSeconds()})
    return out


def main():
    pts, _, _ = synthetic.homography_points(n=100000, inlier_ratio=0.2, seed=11, cluster=(500, 500, 150))
    res = {"knn7_100k_ms": knn_time(pts, 7), "knn13_100k_ms": knn_time(pts, 13)}
    res["napsac_knn_lo"] = run(pts, usac.SAMPLER.Napsac, 1, usac.NeighborsSearch.Nanoflann, [5, 6, 7])
    res["uniform_gc_knn"] = run(pts, usac.SAMPLER.Uniform, 3, usac.NeighborsSearch.Nanoflann, [5, 6])
    res["uniform_gc_grid"] = run(pts, usac.SAMPLER.Uniform, 3, usac.NeighborsSearch.Grid, [5, 6])
    print(json.dumps(res))


if __name__ == "__main__":
    main()
