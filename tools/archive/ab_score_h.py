"""cfg2 score / solve stage times of one library build (RANSAC_AMD_LIB): median over rounds of
ctx.last_timings() for one 65536-hypothesis batch at a time (presorted fast kernel, 8 chunks)."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import ransac_amd as usac
from ransac_amd import synthetic

pts, _, _ = synthetic.homography_points(n=10000, inlier_ratio=0.3, seed=1)
ctx = usac.Context(usac.ESTIMATOR.Homography, pts)
ctx.set_score_chunks(8)
B = 65536
v = []
for rnd in range(25):
    ctx.hypothesize_async(B, 1, rnd * B, 2.0)
    ctx.fetch_best()
    t = ctx.last_timings()
    v.append((t["score_ms"], t["solve_ms"]))
a = np.array(v[3:])
print(json.dumps({"lib": os.path.basename(os.environ.get("RANSAC_AMD_LIB", "libransac_amd.so")),
                  "score_ms_med": float(np.median(a[:, 0])), "score_ms_min": float(a[:, 0].min()),
                  "solve_ms_med": float(np.median(a[:, 1]))}))
