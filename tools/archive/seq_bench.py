"""Σerr chain micro-bench (kernels_seqsum.hip): usac_get_inliers on a line context whose
residuals are a chosen float sequence (model (0, 1, 0): residual |y|), repeated; run under
rocprofv3 --kernel-trace --stats (tools/seq_bench.sh)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import ransac_amd as usac  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
rng = np.random.default_rng(0)
errs = rng.uniform(0, 2, n).astype(np.float32)
pts = np.stack([rng.uniform(-500, 500, n).astype(np.float32), errs], 1)
with usac.Context(usac.ESTIMATOR.Line2d, np.ascontiguousarray(pts)) as ctx:
    m = np.array([0, 1, 0], np.float32)
    for _ in range(10):
        ctx.get_inliers(m, 3.0e38)
    t0 = time.perf_counter()
    for _ in range(reps):
        c, s, _ = ctx.get_inliers(m, 3.0e38)
    dt = time.perf_counter() - t0
ref = np.add.accumulate(errs, dtype=np.float32)[-1]
print("n %d: %.1f us per get_inliers, sum equal %s" % (n, dt / reps * 1e6, np.float32(s).view(np.int32) == ref.view(np.int32)))
