"""Wall-time split of cfg5 runs (context creation, Ransac::run phases via USAC_PROFILE, context
release) -- where a bench step's milliseconds go.  python tools/cfg5_split.py [runs]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import ransac_amd as usac  # noqa: E402
from ransac_amd import synthetic  # noqa: E402

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 20
pts, _, _ = synthetic.homography_points(n=100000, inlier_ratio=0.2, seed=1, cluster=(500, 500, 150))
t_create, t_run, t_del, t_in = [], [], [], []
for i in range(runs + 3):
    mdl = usac.Model(2.0, 4, 0.95, 7, usac.ESTIMATOR.Homography, usac.SAMPLER.Napsac)
    mdl.ResetRandomGenerator(False)
    mdl.setSeed(1 + i)
    mdl.lo = usac.LocOpt(1)
    mdl.max_iterations = 5000
    mdl.setNeighborsType(usac.NeighborsSearch.Grid)
    t0 = time.perf_counter()
    r = usac.Ransac(mdl, pts)
    t1 = time.perf_counter()
    r.run()
    t2 = time.perf_counter()
    out = r.getRansacOutput()
    r.ctx.close()
    t3 = time.perf_counter()
    if i >= 3:
        t_create.append(t1 - t0)
        t_run.append(t2 - t1)
        t_del.append(t3 - t2)
        t_in.append(out.getTimeMicroSeconds() * 1e-6)
f = lambda v: "%.3f" % (1e3 * float(np.mean(v)))  # noqa: E731
print("ms per run: create %s  run %s (inside usac_ransac_run %s)  release %s" % (f(t_create), f(t_run), f(t_in),
                                                                                   f(t_del)))
