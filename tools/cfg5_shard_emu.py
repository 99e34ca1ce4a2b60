"""cfg5 sharded-run rehearsal on ONE GPU: R ranks as R threads of one process, each with its own
context (stream) on the same device, exchanging through an in-process all-gather (the library's
gather callback).  LO stages are latency-bound and use a few dozen workgroups, so R concurrent
streams on one MI355X approximate R GPUs for the LO part; the batched verify is shared.
Prints per-R wall time per run, per-rank LO fits / stages and the USAC_PROFILE split.

  python tools/cfg5_shard_emu.py [--ranks 1 2 4] [--runs 20]
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import ransac_amd as usac  # noqa: E402
from ransac_amd import synthetic  # noqa: E402


def model(seed, lo):
    m = usac.Model(2.0, 4, 0.95, 7, usac.ESTIMATOR.Homography, usac.SAMPLER.Napsac)
    m.ResetRandomGenerator(False)
    m.setSeed(seed)
    m.lo = usac.LocOpt(lo)
    m.max_iterations = 5000
    m.setNeighborsType(usac.NeighborsSearch.Grid)
    return m


class Gather:
    def __init__(self, R):
        self.R = R
        self.slots = [None] * R
        self.bar = threading.Barrier(R)

    def fn(self, k):
        def g(b):
            self.slots[k] = b
            self.bar.wait()
            out = list(self.slots)
            self.bar.wait()
            return out
        return g


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--runs", type=int, default=20)
    ap.add_argument("--lo", type=int, default=1)
    ap.add_argument("--points", type=int, default=100000)
    a = ap.parse_args()
    pts, _, _ = synthetic.homography_points(n=a.points, inlier_ratio=0.2, seed=1, cluster=(500, 500, 150))
    res = {}
    ref = None
    for R in a.ranks:
        ctxs = [usac.Context(usac.ESTIMATOR.Homography, pts) for _ in range(R)]
        outs = [None] * R

        def rank_runs(k, seeds, g):
            o = []
            for s in seeds:
                r = usac.Ransac(model(s, a.lo), pts, ctx=ctxs[k])
                if R == 1:
                    r.run()
                else:
                    r.run(shard=(R, k, g.fn(k)))
                o.append(r.getRansacOutput())
            outs[k] = o

        def batch(seeds):
            g = Gather(R)
            th = [threading.Thread(target=rank_runs, args=(k, seeds, g)) for k in range(R)]
            t0 = time.perf_counter()
            for t in th:
                t.start()
            for t in th:
                t.join()
            return time.perf_counter() - t0

        batch(list(range(1000, 1003)))  # warm-up
        seeds = list(range(1, 1 + a.runs))
        dt = batch(seeds)
        o0 = outs[0]
        if ref is None:
            ref = [(x.getNumberOfMainIterations(), x.getModel().tobytes(), x.getInliers().tobytes()) for x in o0]
        same = all((x.getNumberOfMainIterations(), x.getModel().tobytes(), x.getInliers().tobytes()) == ref[i]
                   for k in range(R) for i, x in enumerate(outs[k]))
        res[R] = {"ms_per_run": dt / a.runs * 1e3, "equal_to_1_rank": same,
                  "lo_fits_per_rank": [int(np.mean([x.raw["lo_fits"] for x in outs[k]])) for k in range(R)],
                  "lo_stages_per_rank": [int(np.mean([x.raw["lo_stages"] for x in outs[k]])) for k in range(R)],
                  "lo_rounds": int(np.mean([x.raw["lo_rounds"] for x in o0])),
                  "iters": int(np.mean([x.getNumberOfMainIterations() for x in o0]))}
        print(json.dumps({R: res[R]}), flush=True)
        for c in ctxs:
            c.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
