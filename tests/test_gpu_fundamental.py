"""GPU parity, fundamental path (7-point solve + oriented filter + Sampson score + 8-point
polish) through the C-ABI against the CPU oracle.  Bar: bit-exact -- number of models per
sample, every F, every count and every sequential fp32 Σerr; chunked (throughput) sums are
re-associated (rel 1e-5), counts still exact.
"""
import numpy as np
import pytest

from ransac_amd import synthetic

pytestmark = pytest.mark.gpu


def _cfg3(n=2000, seed=1, prosac_order=False, noise=0.5):
    pts, F, inl = synthetic.fundamental_points(n=n, inlier_ratio=0.3, seed=seed, noise=noise,
                                               prosac_order=prosac_order)
    return pts, F, inl


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.int32)


def test_seven_point_models_bit_exact(usac, oracle):
    pts, F, inl = _cfg3()
    samples = oracle.uniform_samples(11, len(pts), 7, 4096)
    # add all-inlier samples so the 2- and 3-root branches are exercised
    idx = np.where(inl)[0]
    rng = np.random.default_rng(0)
    good = np.stack([rng.choice(idx, 7, replace=False) for _ in range(1024)]).astype(np.int32)
    samples = np.concatenate([samples, good])
    est = oracle.Estimator(oracle.FUNDAMENTAL, pts)
    om, onm = est.estimate_batch(samples)
    with usac.Context(usac.ESTIMATOR.Fundamental, pts) as ctx:
        gm, gnm = ctx.estimate_models(samples)
    assert (gnm == onm).all()
    assert np.bincount(gnm, minlength=4)[2:].sum() > 50
    assert (_bits(gm) == _bits(om)).all()


def test_score_models_bit_exact(usac, oracle, kusvod2_scenes):
    pts, F, inl = _cfg3()
    est = oracle.Estimator(oracle.FUNDAMENTAL, pts)
    samples = oracle.uniform_samples(12, len(pts), 7, 2000)
    om, onm = est.estimate_batch(samples)
    models = np.concatenate([om[b, :onm[b]] for b in range(len(onm))] + [F.reshape(1, 9)])
    oc, osum = est.score_models(models, 2.0)
    with usac.Context(usac.ESTIMATOR.Fundamental, pts) as ctx:
        c, s = ctx.score_models(models, 2.0)
    assert (c == oc).all() and (_bits(s) == _bits(osum)).all()
    # real kusvod2 scenes with their GT F and F^T
    for scene, (p, Fg) in kusvod2_scenes.items():
        e = oracle.Estimator(oracle.FUNDAMENTAL, p)
        ms = np.stack([Fg, Fg.reshape(3, 3).T.reshape(9)])
        oc, osum = e.score_models(ms, 2.0)
        with usac.Context(usac.ESTIMATOR.Fundamental, p) as ctx:
            c, s = ctx.score_models(ms, 2.0)
        assert (c == oc).all() and (_bits(s) == _bits(osum)).all(), scene


def test_fused_batch_slots_and_best(usac, oracle):
    pts, F, inl = _cfg3(n=3000, seed=2)
    B = 3000
    samples = oracle.uniform_samples(13, len(pts), 7, B)
    est = oracle.Estimator(oracle.FUNDAMENTAL, pts)
    om, onm = est.estimate_batch(samples)
    with usac.Context(usac.ESTIMATOR.Fundamental, pts) as ctx:
        c, s, best = ctx.hypothesize_score(samples=samples, thr=2.0, first_hyp=100)
    c = c.reshape(B, 3)
    s = s.reshape(B, 3)
    order = []
    for b in range(B):
        assert (c[b, onm[b]:] == -1).all()
        if onm[b]:
            oc, osum = est.score_models(om[b, :onm[b]], 2.0)
            assert (c[b, :onm[b]] == oc).all()
            assert (_bits(s[b, :onm[b]]) == _bits(osum)).all()
            for j in range(onm[b]):
                order.append((-int(oc[j]), -float(osum[j]), b, j))
    order.sort()
    _, _, b0, j0 = order[0]
    assert best["valid"] and best["hyp_index"] == 100 + b0
    assert best["inliers"] == c[b0, j0]
    assert (_bits(best["model"]) == _bits(om[b0, j0])).all()


def test_nonminimal_eight_point_bit_exact(usac, oracle):
    pts, F, inl = _cfg3(n=3000, seed=3)
    est = oracle.Estimator(oracle.FUNDAMENTAL, pts)
    idx = np.where(inl)[0].astype(np.int32)
    with usac.Context(usac.ESTIMATOR.Fundamental, pts) as ctx:
        for n in (7, 8, 9, 64, 65, 500, len(idx)):
            g = ctx.nonminimal(idx[:n])
            o = est.nonminimal(idx[:n])
            assert (_bits(g) == _bits(o)).all(), n


def test_get_inliers_bit_exact(usac, oracle):
    pts, F, inl = _cfg3(n=5000, seed=4)
    est = oracle.Estimator(oracle.FUNDAMENTAL, pts)
    with usac.Context(usac.ESTIMATOR.Fundamental, pts) as ctx:
        n, s, idx = ctx.get_inliers(F, 2.0)
    on, osum, oidx = est.quality(F, 2.0, with_inliers=True)
    assert n == on and np.float32(s) == np.float32(osum) and (idx == oidx).all()


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_ransac_run_fundamental_identical(usac, oracle, seed):
    pts, F, inl = _cfg3(n=2000, seed=seed)
    ref = oracle.ransac_run(oracle.FUNDAMENTAL, pts, 2.0, 0.95, seed)
    m = usac.Model(2.0, 7, 0.95, 7, usac.ESTIMATOR.Fundamental, usac.SAMPLER.Uniform)
    m.ResetRandomGenerator(False)
    m.setSeed(seed)
    m.batch = 1024
    r = usac.Ransac(m, pts)
    r.run()
    out = r.getRansacOutput()
    assert out.getNumberOfMainIterations() == ref["iters"]
    assert [(i, c) for i, c, _ in r.records] == [(i, c) for i, c, _ in ref["records"]]
    assert [np.float32(s) for _, _, s in r.records] == [np.float32(s) for _, _, s in ref["records"]]
    assert (_bits(out.raw["minimal_model"]) == _bits(ref["minimal_model"])).all()
    assert out.raw["polish_passes"] == ref["polish_passes"]
    assert (_bits(out.getModel()) == _bits(ref["model"])).all()
    assert out.getNumberOfInliers() == ref["inliers"]
    assert (out.getInliers() == ref["inlier_idx"]).all()


def test_throughput_batch_full_size(usac, oracle):
    """cfg3 size (10k points, device sampler, chunked score): the batch best re-scored by the
    oracle has the same count; every slot count is either -1 or in [0, N]."""
    pts, F, inl = synthetic.fundamental_points(n=10000, inlier_ratio=0.3, seed=1)
    with usac.Context(usac.ESTIMATOR.Fundamental, pts) as ctx:
        ctx.set_score_chunks(8)
        B = 16384
        c, s, best = ctx.hypothesize_score(B=B, seed=5, first_hyp=0, thr=2.0)
        ctx.hypothesize_async(B, 5, 0, 2.0)
        rec = ctx.fetch_best()
    assert c.shape == (3 * B,) and c.min() >= -1 and c.max() <= len(pts)
    est = oracle.Estimator(oracle.FUNDAMENTAL, pts)
    oc, osum = est.quality(best["model"], 2.0)
    assert oc == best["inliers"] == c.max()
    # chunked Σ may reorder exact count ties; the count of the batch best is exact
    assert rec.inliers == best["inliers"]


@pytest.mark.parametrize("kind", ["F", "H"])
def test_batch_sprt_accepts_exact_counts(usac, oracle, kind):
    """Throughput SPRT: accepted models carry their exact full inlier count (score = count),
    rejected ones -1; good all-inlier samples survive, most random models are rejected."""
    if kind == "F":
        pts, M, inl = _cfg3(n=4000, seed=6)
        est_id, okind, m = usac.ESTIMATOR.Fundamental, oracle.FUNDAMENTAL, 7
    else:
        pts, M, inl = synthetic.homography_points(n=4000, inlier_ratio=0.3, seed=6)
        est_id, okind, m = usac.ESTIMATOR.Homography, oracle.HOMOGRAPHY, 4
    rng = np.random.default_rng(1)
    idx = np.where(inl)[0]
    good = np.stack([rng.choice(idx, m, replace=False) for _ in range(64)]).astype(np.int32)
    samples = np.concatenate([oracle.uniform_samples(21, len(pts), m, 4096), good])
    est = oracle.Estimator(okind, pts)
    with usac.Context(est_id, pts) as ctx:
        ctx.set_sprt(True, seed=1)
        c, s, best = ctx.hypothesize_score(samples=samples, thr=2.0)
        tested = ctx.sprt_tested()
        ctx.set_sprt(False)
        cf, sf, _ = ctx.hypothesize_score(samples=samples, thr=2.0)
    acc = c >= 0
    occupied = cf >= 0
    assert (acc <= occupied).all()
    assert (c[acc] == cf[acc]).all() and (s[acc] == c[acc].astype(np.float32)).all()
    assert acc.sum() >= 1 and acc.sum() <= 0.2 * occupied.sum()
    assert best["valid"] and best["inliers"] == c.max()
    oc, _ = est.quality(best["model"], 2.0)
    assert oc == best["inliers"]
    assert tested < 0.2 * occupied.sum() * len(pts)


@pytest.mark.parametrize("cert", ["default", "all_sequential", "low_climb"])
@pytest.mark.parametrize("kind", ["F", "H", "L"])
def test_batch_sprt_decisions_equal_reference_walk(usac, oracle, kind, cert, monkeypatch):
    """Every batch-SPRT decision equals the reference's fp64 lambda product walk from the model's
    start (kernels_sprt.hip's certificate): by default almost every walk is certified from counts;
    with the margin widened to 1e9 every walk takes the sequential product path, with the climb
    limit at 3 many do -- the decisions must not change."""
    from tests.helpers.sprt_check import batch_sprt_vs_oracle
    if cert == "all_sequential":
        monkeypatch.setenv("USAC_SPRT_CERT_MARGIN", "1e9")
    elif cert == "low_climb":
        monkeypatch.setenv("USAC_SPRT_CERT_CLIMB", "3")
    if kind == "F":
        pts, _, inl = _cfg3(n=4000, seed=7)
        est_id, okind, m, thr = usac.ESTIMATOR.Fundamental, oracle.FUNDAMENTAL, 7, 2.0
    elif kind == "H":
        pts, _, inl = synthetic.homography_points(n=4000, inlier_ratio=0.3, seed=7)
        est_id, okind, m, thr = usac.ESTIMATOR.Homography, oracle.HOMOGRAPHY, 4, 2.0
    else:
        pts, M = synthetic.line_points(n=3000, inlier_ratio=0.3, seed=7)
        inl = np.abs(pts @ M[:2] + M[2]) < 3.0
        est_id, okind, m, thr = usac.ESTIMATOR.Line2d, oracle.LINE2D, 2, 8.0
    rng = np.random.default_rng(2)
    idx = np.where(inl)[0]
    good = np.stack([rng.choice(idx, m, replace=False) for _ in range(48)]).astype(np.int32)
    samples = np.concatenate([oracle.uniform_samples(23, len(pts), m, 1000), good])
    with usac.Context(est_id, pts) as ctx:
        ctx.set_sprt(True, seed=3)
        c, _, _ = ctx.hypothesize_score(samples=samples, thr=thr)
        r = batch_sprt_vs_oracle(oracle, ctx, okind, pts, thr, samples, c, 3, m)
    assert r["accepted"] >= 1 and r["models"] > 100
    np.testing.assert_array_equal(r["device"], r["oracle"])
    assert r["empty_slots_ok"]
