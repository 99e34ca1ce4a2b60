"""Wall time of the NAPSAC grid (build + download) for fresh contexts over the cfg5 points:
python tools/grid_time.py [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import ransac_amd as usac  # noqa: E402
from ransac_amd import synthetic  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
pts, _, _ = synthetic.homography_points(n=100000, inlier_ratio=0.2, seed=1, cluster=(500, 500, 150))
ts = []
for i in range(reps + 3):
    with usac.Context(usac.ESTIMATOR.Homography, pts) as ctx:
        t0 = time.perf_counter()
        ctx.grid_neighbors(50)
        t1 = time.perf_counter()
    if i >= 3:
        ts.append(t1 - t0)
print("grid build + download: %.3f ms (median of %d)" % (1e3 * float(np.median(ts)), reps))
