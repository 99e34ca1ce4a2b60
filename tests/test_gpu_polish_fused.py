"""The polish in one workgroup (k_polish_fused, kernels_nonmin.hip) against the oracle's polish
(ransac.cpp:157-207) and against the multi-launch passes it replaces: H, F and E runs whose best
models have a few hundred to a few thousand inliers give the oracle's polish passes, final
model bits and inlier list with the fused kernel on (USAC_POLISH_FUSED=1), off (the default) and
with a small list bound (USAC_POLISH_FUSED_MAX: the kernel stops at the first pass whose list
is longer and the host resumes that pass the multi-launch way) -- all identical."""
import os

import numpy as np
import pytest

from ransac_amd import synthetic

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.int32)


def _data(kind, n, ratio, seed):
    if kind == "H":
        return np.ascontiguousarray(synthetic.homography_points(n=n, inlier_ratio=ratio, seed=seed)[0])
    if kind == "F":
        return np.ascontiguousarray(synthetic.fundamental_points(n=n, inlier_ratio=ratio, seed=seed)[0])
    return np.ascontiguousarray(synthetic.fundamental_points(n=n, inlier_ratio=ratio, seed=seed, noise=0.5,
                                                             normalized=True)[0])


def _run(usac, kind, pts, thr, seed, env):
    est = {"H": usac.ESTIMATOR.Homography, "F": usac.ESTIMATOR.Fundamental, "E": usac.ESTIMATOR.Essential}[kind]
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        m = usac.Model(thr, {"H": 4, "F": 7, "E": 5}[kind], 0.95, 7, est, usac.SAMPLER.Uniform)
        m.ResetRandomGenerator(False)
        m.setSeed(seed)
        r = usac.Ransac(m, pts)
        r.run()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    o = r.getRansacOutput()
    return (o.raw["polish_passes"], _bits(o.getModel()).tolist(), o.getInliers().tolist(), r.records,
            o.getNumberOfMainIterations())


@pytest.mark.parametrize("kind,n,ratio", [("H", 3000, 0.3), ("H", 12000, 0.3), ("F", 3000, 0.3), ("F", 10000, 0.3),
                                          ("E", 4000, 0.4)])
def test_polish_fused_identical(usac, oracle, kind, n, ratio):
    thr = 0.002 if kind == "E" else 2.0
    okind = {"H": oracle.HOMOGRAPHY, "F": oracle.FUNDAMENTAL, "E": oracle.ESSENTIAL}[kind]
    passes = set()
    for seed in (1, 2):
        pts = _data(kind, n, ratio, seed)
        a = _run(usac, kind, pts, thr, seed, {"USAC_POLISH_FUSED": "1"})
        b = _run(usac, kind, pts, thr, seed, {})
        cut = str(max(9, len(a[2]) - 1))  # the list of the first accepted pass is longer: resume there
        c = _run(usac, kind, pts, thr, seed, {"USAC_POLISH_FUSED": "1", "USAC_POLISH_FUSED_MAX": cut})
        assert a == b, (kind, seed)
        assert a == c, (kind, seed)
        passes.add(a[0])
        if kind != "E" or n <= 4000:
            ref = oracle.ransac_run(okind, pts, thr, 0.95, seed)
            assert a[0] == ref["polish_passes"]
            assert a[1] == _bits(ref["model"]).tolist()
            assert a[2] == list(ref["inlier_idx"])
    assert max(passes) >= 1
