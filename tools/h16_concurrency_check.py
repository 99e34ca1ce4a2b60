"""Concurrency check of the homography scorers: P contexts with batches in flight on their own
streams (bench.py's pipeline), each batch's counts compared with the same batch scored alone by
the exact one-chunk kernel (score variant 1).  Usage: python tools/h16_concurrency_check.py [P]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import ransac_amd as usac  # noqa: E402
from ransac_amd import synthetic  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 3
B, N, thr, seed = 65536, 24, 2.0, 1
pts, _, _ = synthetic.homography_points(n=10000, inlier_ratio=0.3, seed=seed)
ctxs = [usac.Context(usac.ESTIMATOR.Homography, pts) for _ in range(P)]
for c in ctxs:
    c.set_score_chunks(8)
got = {}
for i in range(N + P - 1):
    if i < N:
        ctxs[i % P].hypothesize_async(B, seed, i * B, thr)
    j = i - P + 1
    if j >= 0:
        c = ctxs[j % P]
        c.fetch_best()
        got[j] = c.last_counts(B)[0].copy()
ref = ctxs[0]
ref.set_score_variant(1)
bad = 0
for j in range(N):
    cnt, _, _ = ref.hypothesize_score(B=B, seed=seed, first_hyp=j * B, thr=thr)
    d = np.flatnonzero(got[j] != cnt)
    if len(d):
        bad += 1
        print("batch %d: %d hypotheses differ, e.g. %s" % (j, len(d), [(int(k), int(got[j][k]), int(cnt[k])) for k in d[:4]]))
print("P %d: %d of %d batches differ" % (P, bad, N))
sys.exit(1 if bad else 0)
