"""Homography score-kernel time vs the data's inlier ratio (tail effect of the few good
hypotheses, whose points mostly pass stage A)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import ransac_amd as usac
from ransac_amd import synthetic

B = 65536
for ratio in (0.0, 0.05, 0.1, 0.3, 0.5):
    pts, _, _ = synthetic.homography_points(n=10000, inlier_ratio=ratio, seed=1)
    with usac.Context(usac.ESTIMATOR.Homography, pts) as ctx:
        ctx.set_score_chunks(8)
        ms = []
        for r in range(8):
            ctx.hypothesize_async(B, 1, r * B, 2.0)
            ctx.fetch_best()
            ms.append(ctx.last_timings()["score_ms"])
        print("inlier_ratio %.2f  score_ms med %.4f min %.4f" % (ratio, np.median(ms[2:]), min(ms[2:])))
