"""Latency of the sequential-sum kernels against the chain length: usac_nonminimal (NormalizedDLT
on n points -> k_seq_seg / k_seq_link over n elements) repeated per n, one n after the other, so
a --kernel-trace shows each kernel's duration per n in launch order.
python tools/seq_micro.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import ransac_amd as usac  # noqa: E402
from ransac_amd import synthetic  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
pts, _, _ = synthetic.homography_points(n=100000, inlier_ratio=0.2, seed=1, cluster=(500, 500, 150))
with usac.Context(usac.ESTIMATOR.Homography, pts) as ctx:
    for n in (1000, 4000, 8000, 12000, 16000, 20000, 40000):
        idx = np.arange(n, dtype=np.int32)
        for _ in range(reps):
            ctx.nonminimal(idx)
        print(n, flush=True)
