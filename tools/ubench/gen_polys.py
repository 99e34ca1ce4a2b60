"""8192 degree-10 polynomials of the 5-point solver (cfg4 samples, the oracle's det M(z)) and their
JT work units (oracle restatement instrumented offline) -> tools/ubench/polys.bin for jt_bench.hip."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from oracle import oracle  # noqa: E402
from ransac_amd import synthetic  # noqa: E402

pts, _, _ = synthetic.fundamental_points(n=50000, inlier_ratio=0.3, seed=1, normalized=True)
est = oracle.Estimator(oracle.ESSENTIAL, pts)
A = np.array([oracle.e5_poly(est, s) for s in oracle.uniform_samples(13, len(pts), 5, 8192)])
A.astype(np.float64).tofile(os.path.join(os.path.dirname(os.path.abspath(__file__)), "polys.bin"))
print(A.shape)
