"""cfg4 throughput batches scored by the e16 matrix-core scorer only (PMC passes: rocprofv3 -- python tools/e16_only.py)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
os.environ["USAC_E16"] = "1"
import ransac_amd as usac  # noqa: E402
from ransac_amd import synthetic  # noqa: E402

pts, _, _ = synthetic.fundamental_points(n=50000, inlier_ratio=0.3, seed=1, normalized=True)
with usac.Context(usac.ESTIMATOR.Essential, pts) as ctx:
    ctx.set_score_chunks(96)
    for i in range(4):
        ctx.hypothesize_async(65536, 1, i * 65536, 0.002)
        ctx.fetch_best()
print("ok")
