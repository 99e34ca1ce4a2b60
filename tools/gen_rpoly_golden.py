"""Generate tests/golden/rpoly_ref.npz: the reference's own rpoly_ak1 (usac/estimator/essential/rpoly.cpp,
compiled where it lies into oracle/_ref/librpoly_ref.so by oracle/Makefile) on 400 degree-10 polynomials of
the 5-point solver (the oracle's det M(z) of cfg4 samples) and 400 random polynomials of degree 3-10.
Stored: the coefficients (ascending), the reference's zeros (real, imaginary; its order) and its degree.
Run here, where the reference is present; the fixture pins the oracle's restatement on boxes without it."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from oracle import oracle  # noqa: E402
from ransac_amd import synthetic  # noqa: E402

assert oracle.rpoly_ref_available(), "oracle/_ref/librpoly_ref.so missing: run make -C oracle with the reference present"
pts, _, _ = synthetic.fundamental_points(n=50000, inlier_ratio=0.3, seed=1, normalized=True)
est = oracle.Estimator(oracle.ESSENTIAL, pts)
polys = [oracle.e5_poly(est, s) for s in oracle.uniform_samples(17, len(pts), 5, 400)]
rng = np.random.default_rng(21)
for _ in range(400):
    n = int(rng.integers(3, 11))
    a = np.zeros(11)
    a[: n + 1] = (rng.uniform(size=n + 1) - 0.5) * 10.0 ** ((rng.uniform(size=n + 1) - 0.5) * 8)
    polys.append(a)
A = np.array(polys)
deg = np.array([int(np.max(np.nonzero(a)[0])) for a in A], np.int32)
ZR = np.zeros((len(A), 10))
ZI = np.zeros((len(A), 10))
K = np.zeros(len(A), np.int32)
for i, a in enumerate(A):
    zr, zi = oracle.rpoly_ref_zeros(a[: deg[i] + 1])
    K[i] = len(zr)
    ZR[i, : len(zr)] = zr
    ZI[i, : len(zi)] = zi
out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "rpoly_ref.npz")
np.savez_compressed(out, coeffs=A, degree=deg, zr=ZR, zi=ZI, nzeros=K)
print("wrote", out, len(A))
