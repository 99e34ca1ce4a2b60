"""cfg4 score / solve stage times of one library build (RANSAC_AMD_LIB) over score-chunk counts:
median over rounds of ctx.last_timings() for one 65536-sample batch at a time."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import ransac_amd as usac
from ransac_amd import synthetic

pts, _, _ = synthetic.fundamental_points(n=50000, inlier_ratio=0.3, seed=1, normalized=True)
ctx = usac.Context(usac.ESTIMATOR.Essential, pts)
B, thr = int(os.environ.get("B", 65536)), 0.002
chunks = [int(c) for c in os.environ.get("CHUNKS", "96").split(",")]
res = {c: [] for c in chunks}
for rnd in range(7):
    for c in chunks:
        ctx.set_score_chunks(c)
        ctx.hypothesize_async(B, 1, rnd * B, thr)
        ctx.fetch_best()
        t = ctx.last_timings()
        res[c].append((t["score_ms"], t["solve_ms"], t["batch_ms"]))
out = {}
for c, v in res.items():
    a = np.array(v[1:])
    out[c] = {"score_ms": float(np.median(a[:, 0])), "solve_ms": float(np.median(a[:, 1])),
              "batch_ms": float(np.median(a[:, 2]))}
print(json.dumps({"lib": os.path.basename(os.environ.get("RANSAC_AMD_LIB", "libransac_amd.so")), "B": B,
                  "chunks": out}))
