"""cfg3 exact runs: iterations, batches, PROSAC rewinds and records per run (diagnostic)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import ransac_amd as usac  # noqa: E402
from ransac_amd import synthetic  # noqa: E402

pts, _, _ = synthetic.fundamental_points(n=10000, inlier_ratio=0.3, seed=1)
ctx = usac.Context(usac.ESTIMATOR.Fundamental, pts)
for seed in range(1, 21):
    m = usac.Model(2.0, 7, 0.95, 7, usac.ESTIMATOR.Fundamental, usac.SAMPLER.Prosac)
    m.ResetRandomGenerator(False)
    m.setSeed(seed)
    m.setSprt(True)
    r = usac.Ransac(m, pts, ctx=ctx)
    r.run()
    o = r.getRansacOutput()
    print(seed, "iters", o.getNumberOfMainIterations(), "batches", o.raw["batches"], "rewinds", o.raw["rollbacks"],
          "term_len", o.raw["prosac_term_len"], "records", [(i, c) for i, c, _ in r.records])
