"""cfg4 batch phases on one context (no pipelining): solve / score / batch ms per 65 536-sample batch,
for the matrix-core e16 scorer and the lanes-over-models k_score_f2 (USAC_E16=0).  Usage: python tools/e_phase.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import ransac_amd as usac  # noqa: E402
from ransac_amd import synthetic  # noqa: E402

pts, _, _ = synthetic.fundamental_points(n=50000, inlier_ratio=0.3, seed=1, normalized=True)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
for flag in ("1", "0"):
    os.environ["USAC_E16"] = flag
    with usac.Context(usac.ESTIMATOR.Essential, pts) as ctx:
        ctx.set_score_chunks(96)
        t = []
        for i in range(12):
            ctx.hypothesize_async(B, 1, i * B, 0.002)
            rec = ctx.fetch_best()
            if i >= 2:
                t.append(ctx.last_timings())
    print("USAC_E16=%s: batch %.3f ms, solve %.3f ms, score %.3f ms (best %d inliers)" % (
        flag, np.mean([x["batch_ms"] for x in t]), np.mean([x["solve_ms"] for x in t]),
        np.mean([x["score_ms"] for x in t]), rec.inliers), flush=True)
os.environ.pop("USAC_E16", None)
