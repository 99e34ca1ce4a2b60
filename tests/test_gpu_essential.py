"""GPU parity, essential path (5-point solve + cheirality + epipolar-distance score + 8-point
polish) through the C-ABI against the CPU oracle: every E bit-exact, counts and sequential
sums exact, the whole loop identical (Uniform / PROSAC x SPRT)."""
import numpy as np
import pytest

from ransac_amd import synthetic

pytestmark = pytest.mark.gpu


def _cfg4(n=2000, seed=1, noise=0.5, prosac_order=False, ratio=0.3):
    return synthetic.fundamental_points(n=n, inlier_ratio=ratio, seed=seed, noise=noise, normalized=True,
                                        prosac_order=prosac_order)


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.int32)


def test_five_point_models_bit_exact(usac, oracle):
    pts, E, inl = _cfg4()
    rng = np.random.default_rng(0)
    idx = np.where(inl)[0]
    good = np.stack([rng.choice(idx, 5, replace=False) for _ in range(256)]).astype(np.int32)
    samples = np.concatenate([oracle.uniform_samples(31, len(pts), 5, 768), good])
    est = oracle.Estimator(oracle.ESSENTIAL, pts)
    om, onm = est.estimate_batch(samples)
    with usac.Context(usac.ESTIMATOR.Essential, pts) as ctx:
        gm, gnm = ctx.estimate_models(samples)
    assert (gnm == onm).all()
    assert onm.sum() > 500
    assert (_bits(gm[gnm == 1]) == _bits(om[onm == 1])).all()


def test_essential_score_inliers_nonminimal(usac, oracle):
    pts, E, inl = _cfg4(n=5000, seed=2)
    est = oracle.Estimator(oracle.ESSENTIAL, pts)
    samples = oracle.uniform_samples(32, len(pts), 5, 600)
    om, onm = est.estimate_batch(samples)
    models = np.concatenate([om[onm == 1], E.reshape(1, 9)])
    oc, osum = est.score_models(models, 0.002)
    with usac.Context(usac.ESTIMATOR.Essential, pts) as ctx:
        c, s = ctx.score_models(models, 0.002)
        assert (c == oc).all() and (_bits(s) == _bits(osum)).all()
        n, sm, idx = ctx.get_inliers(E, 0.002)
        on, osm, oidx = est.quality(E, 0.002, with_inliers=True)
        assert n == on and np.float32(sm) == np.float32(osm) and (idx == oidx).all()
        tidx = np.where(inl)[0].astype(np.int32)
        for k in (8, 9, 100, len(tidx)):
            assert (_bits(ctx.nonminimal(tidx[:k])) == _bits(est.nonminimal(tidx[:k]))).all(), k


@pytest.mark.parametrize("sampler", ["uniform", "prosac"])
@pytest.mark.parametrize("sprt", [False, True])
def test_essential_loop_identical(usac, oracle, sampler, sprt):
    pts, E, inl = _cfg4(n=2000, seed=3, prosac_order=(sampler == "prosac"), ratio=0.5)
    osmp = oracle.SAMPLER_PROSAC if sampler == "prosac" else oracle.SAMPLER_UNIFORM
    ref = oracle.ransac_run(oracle.ESSENTIAL, pts, 0.002, 0.95, 3, sampler=osmp, sprt=sprt, max_iters=3000)
    m = usac.Model(0.002, 5, 0.95, 7, usac.ESTIMATOR.Essential,
                   usac.SAMPLER.Prosac if sampler == "prosac" else usac.SAMPLER.Uniform)
    m.ResetRandomGenerator(False)
    m.setSeed(3)
    m.setSprt(sprt)
    m.max_iterations = 3000
    m.batch = 256
    r = usac.Ransac(m, pts)
    r.run()
    out = r.getRansacOutput()
    assert out.getNumberOfMainIterations() == ref["iters"]
    assert [(i, c) for i, c, _ in r.records] == [(i, c) for i, c, _ in ref["records"]]
    assert [np.float32(s) for _, _, s in r.records] == [np.float32(s) for _, _, s in ref["records"]]
    assert out.raw["sprt_rejected"] == ref["sprt_rejected"]
    assert (_bits(out.raw["minimal_model"]) == _bits(ref["minimal_model"])).all()
    assert (_bits(out.getModel()) == _bits(ref["model"])).all()
    assert (out.getInliers() == ref["inlier_idx"]).all()


def test_essential_throughput_batch(usac, oracle):
    pts, E, inl = _cfg4(n=20000, seed=4)
    est = oracle.Estimator(oracle.ESSENTIAL, pts)
    with usac.Context(usac.ESTIMATOR.Essential, pts) as ctx:
        ctx.set_score_chunks(8)
        c, s, best = ctx.hypothesize_score(B=4096, seed=9, first_hyp=0, thr=0.002)
        assert best["valid"] and best["inliers"] == c.max()
        oc, _ = est.quality(best["model"], 0.002)
        assert oc == best["inliers"]
        ctx.set_sprt(True, seed=2)
        c2, s2, best2 = ctx.hypothesize_score(B=4096, seed=9, first_hyp=0, thr=0.002)
        acc = c2 >= 0
        assert acc.sum() >= 1 and (c2[acc] == c[acc]).all()
