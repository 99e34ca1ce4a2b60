"""Per-seed cfg5 run statistics (the bench's 100 seeds): mean wall per run, main iterations,
loop batches, LO stages -- separates a slower run path from runs that simply do more work
(a solver spec change moves the runs' trajectories).  python tools/cfg5_stats.py [runs]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import ransac_amd as usac  # noqa: E402
from ransac_amd import synthetic  # noqa: E402

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 100
pts, _, _ = synthetic.homography_points(n=100000, inlier_ratio=0.2, seed=1, cluster=(500, 500, 150))


def one(seed):
    mdl = usac.Model(2.0, 4, 0.95, 7, usac.ESTIMATOR.Homography, usac.SAMPLER.Napsac)
    mdl.ResetRandomGenerator(False)
    mdl.setSeed(seed)
    mdl.lo = usac.LocOpt(1)
    mdl.max_iterations = 5000
    mdl.setNeighborsType(usac.NeighborsSearch.Grid)
    r = usac.Ransac(mdl, pts)
    t0 = time.perf_counter()
    r.run()
    t = time.perf_counter() - t0
    o = r.getRansacOutput()
    r.ctx.close()
    return t, o.getNumberOfMainIterations(), int(o.raw["batches"]), int(o.raw["lo_stages"]), int(o.getTimeMicroSeconds())


for i in range(5):
    one(10_000 + i)
rows = np.array([one(1 + s) for s in range(runs)], dtype=np.float64)
print("runs %d: wall %.3f ms, inside %.3f ms, iterations %.1f, batches %.2f, lo_stages %.2f" %
      (runs, 1e3 * rows[:, 0].mean(), 1e-3 * rows[:, 4].mean(), rows[:, 1].mean(), rows[:, 2].mean(), rows[:, 3].mean()))
