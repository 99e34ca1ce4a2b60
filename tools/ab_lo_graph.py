"""Same-process A/B of the LO stage graphs (USAC_LO_GRAPH, read at context creation): cfg5 runs
(100 k clustered points, NAPSAC grid + InItLORsc) alternating the two settings, USAC_PROFILE split
of each run parsed from stderr.  python tools/ab_lo_graph.py [runs]"""
import os
import re
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import ransac_amd as usac  # noqa: E402
from ransac_amd import synthetic  # noqa: E402

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 40
pts, _, _ = synthetic.homography_points(n=100000, inlier_ratio=0.2, seed=1, cluster=(500, 500, 150))
os.environ["USAC_PROFILE"] = "1"
err = tempfile.TemporaryFile(mode="w+")
os.dup2(err.fileno(), 2)
res = {0: [], 1: []}
for i in range(runs + 4):
    g = i % 2
    os.environ["USAC_LO_GRAPH"] = str(g)
    mdl = usac.Model(2.0, 4, 0.95, 7, usac.ESTIMATOR.Homography, usac.SAMPLER.Napsac)
    mdl.ResetRandomGenerator(False)
    mdl.setSeed(1 + i // 2)  # both arms run the same seeds
    mdl.lo = usac.LocOpt(1)
    mdl.max_iterations = 5000
    mdl.setNeighborsType(usac.NeighborsSearch.Grid)
    t0 = time.perf_counter()
    r = usac.Ransac(mdl, pts)
    r.run()
    r.ctx.close()
    dt = time.perf_counter() - t0
    if i >= 4:
        res[g].append(dt * 1e3)
err.seek(0)
lines = [ln for ln in err.read().splitlines() if ln.startswith("usac_ransac_run ms")]
lo = {0: [], 1: []}
built = {0: [], 1: []}
for i, ln in enumerate(lines):
    m = re.search(r"lo ([\d.]+) .*stages (\d+)", ln)
    gb = re.search(r"graphs (\d+)", ln)
    if m and i >= 4:
        lo[i % 2].append(float(m.group(1)) / max(1, int(m.group(2))) * 1e3)
        built[i % 2].append(int(gb.group(1)) if gb else 0)
for g in (0, 1):
    print("graph=%d  ms/run mean %.3f median %.3f  LO us/stage mean %.1f  graphs captured/run %.2f (last 10: %s)"
          " (%d runs)" % (g, np.mean(res[g]), np.median(res[g]), np.mean(lo[g]) if lo[g] else float("nan"),
                          np.mean(built[g]) if built[g] else 0, built[g][-10:], len(res[g])),
        file=sys.stdout, flush=True)
