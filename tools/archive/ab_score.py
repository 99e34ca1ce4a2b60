"""A/B the score-kernel variants in one process (interleaved rounds, median ms)."""
import sys, os, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import ransac_amd as usac
from ransac_amd import synthetic

pts, _, _ = synthetic.homography_points(n=int(os.environ.get("NPTS", 10000)), inlier_ratio=0.3, seed=1)
ctx = usac.Context(usac.ESTIMATOR.Homography, pts)
variants = [(c, v) for v in (0, 2) for c in (4, 8)] + [(1, 0), (8, 1)]
res = {k: [] for k in variants}
B = 65536
for rnd in range(6):
    for (c, v) in variants:
        ctx.set_score_chunks(c); ctx.set_score_variant(v)
        ctx.hypothesize_async(B, 1, rnd * B, 2.0)
        ctx.fetch_best()
        t = ctx.last_timings()
        res[(c, v)].append((t["score_ms"], t["solve_ms"], t["batch_ms"]))
for k, v in res.items():
    a = np.array(v[1:])
    print("chunks=%d variant=%d score_ms med %.4f min %.4f | solve %.4f | batch %.4f" % (k[0], k[1], np.median(a[:,0]), a[:,0].min(), np.median(a[:,1]), np.median(a[:,2])))
