"""The fast two-view scorer (packed stage A + LDS queues, `k_score_f2`) against the exact
oracle and the exact device kernel (score variant 1): counts and sequential sums bit-equal
on models built to stress the division-free rejection tests -- pairs exactly on the
threshold and on the next float, near-degenerate denominators, huge / tiny / NaN entries.
(DESIGN.md "Two-view stage A".)"""
import numpy as np
import pytest

from ransac_amd import synthetic

pytestmark = pytest.mark.gpu


def _models(rng, base):
    models = [base]
    for scale in (1e-6, 1e-4, 1e-2, 1.0):
        models += [base * (1 + scale * rng.standard_normal(9).astype(np.float32)) for _ in range(30)]
    models += [rng.standard_normal(9).astype(np.float32) * np.float32(10 ** rng.uniform(-20, 20)) for _ in range(60)]
    rank1 = np.outer(rng.standard_normal(3), rng.standard_normal(3)).reshape(9).astype(np.float32)
    z = base.copy()
    z[[0, 1, 3, 4]] = 0.0  # epipolar-line normals vanish on part of the data
    models += [rank1, z, base * np.float32(1e30), base * np.float32(1e-30), np.zeros(9, np.float32),
               np.full(9, np.nan, np.float32), np.where(np.arange(9) == 4, np.inf, base).astype(np.float32)]
    return np.stack(models).astype(np.float32)


@pytest.mark.parametrize("kind", ["F", "E"])
def test_fast_twoview_adversarial(usac, oracle, kind):
    rng = np.random.default_rng(5)
    if kind == "F":
        pts, F, _ = synthetic.fundamental_points(n=3001, inlier_ratio=0.4, seed=3, prosac_order=False)
        okind, est_id, thrs = oracle.FUNDAMENTAL, usac.ESTIMATOR.Fundamental, [2.0, 0.3, 11.0]
    else:
        pts, F, _ = synthetic.fundamental_points(n=3001, inlier_ratio=0.4, seed=3, normalized=True,
                                                 prosac_order=False)
        okind, est_id, thrs = oracle.ESSENTIAL, usac.ESTIMATOR.Essential, [0.002, 0.0004, 0.05]
    base = (np.asarray(F, np.float64) / np.abs(F).max()).reshape(9).astype(np.float32)
    models = _models(rng, base)
    est = oracle.Estimator(okind, pts)
    with usac.Context(est_id, pts) as ctx:
        for thr in thrs:
            oc, os_ = est.score_models(models, thr)
            gc, gs = ctx.score_models(models, thr)  # fast kernel
            np.testing.assert_array_equal(gc, oc)
            np.testing.assert_array_equal(gs.view(np.int32), os_.view(np.int32))
            ctx.set_score_variant(1)
            ec, es = ctx.score_models(models, thr)  # exact kernel
            ctx.set_score_variant(0)
            np.testing.assert_array_equal(ec, oc)
            np.testing.assert_array_equal(es.view(np.int32), os_.view(np.int32))
        # thresholds exactly on pairs' errors (and the next float up) for a few models
        for m in models[[0, 5, 40, 100]]:
            errs = est.errors(m)
            fin = np.sort(errs[np.isfinite(errs) & (errs > 0)])
            for e in fin[:: max(1, len(fin) // 6)][:6]:
                for tt in (float(e), float(np.nextafter(np.float32(e), np.float32(np.inf)))):
                    gc, gs = ctx.score_models(m[None], tt)
                    oc, os_ = est.score_models(m[None], tt)
                    assert gc[0] == oc[0], (kind, tt)
                    assert gs.view(np.int32)[0] == os_.view(np.int32)[0], (kind, tt)


@pytest.mark.parametrize("kind", ["F", "E"])
def test_fast_twoview_full_batch_equals_exact(usac, kind):
    """A whole device-sampled batch (B = 65536): fast vs exact kernel, one chunk and 64."""
    if kind == "F":
        pts, _, _ = synthetic.fundamental_points(n=10000, inlier_ratio=0.3, seed=1)
        est_id, thr = usac.ESTIMATOR.Fundamental, 2.0
    else:
        pts, _, _ = synthetic.fundamental_points(n=20000, inlier_ratio=0.3, seed=1, normalized=True)
        est_id, thr = usac.ESTIMATOR.Essential, 0.002
    with usac.Context(est_id, pts) as ctx:
        ctx.set_score_variant(1)
        ce, se, be = ctx.hypothesize_score(B=65536, seed=7, first_hyp=0, thr=thr)
        ctx.set_score_variant(0)
        cf, sf, bf = ctx.hypothesize_score(B=65536, seed=7, first_hyp=0, thr=thr)
        np.testing.assert_array_equal(cf, ce)
        np.testing.assert_array_equal(sf.view(np.int32), se.view(np.int32))
        assert bf["hyp_index"] == be["hyp_index"]
        ctx.set_score_chunks(64)
        ctx.hypothesize_async(65536, 7, 0, thr)
        rec = ctx.fetch_best()
        assert rec.inliers == be["inliers"]


def test_essential_guarded_drain(usac, oracle):
    """The throughput launches' essential drains take the guarded residual (kernels_fund.hip
    essential_error_guarded: v_rsq_f32 instead of the correctly rounded square roots and IEEE
    divisions, the exact expression inside a 2^-16 band around thr).  A device batch scored in
    8 chunks: every count equals the oracle's -- also with thr placed exactly on a pair's error
    and on the next float -- and each Σ is within the stated bound c thr 2^-18 + |Σ| c 2^-23."""
    pts, _, _ = synthetic.fundamental_points(n=20000, inlier_ratio=0.3, seed=3, normalized=True)
    B, seed = 512, 5
    est = oracle.Estimator(oracle.ESSENTIAL, pts)
    with usac.Context(usac.ESTIMATOR.Essential, pts) as ctx:
        ctx.set_score_chunks(8)
        smp = ctx.draw_samples(B, seed, 0)
        om, onm = est.estimate_batch(smp)
        occ = onm == 1
        assert occ.sum() > 100
        # thresholds on the exact errors of pairs of a model with many inliers, and the next floats
        good = np.flatnonzero(occ)[np.argmax(est.score_models(om[occ], 0.002)[0])]
        e = est.errors(om[good])
        near = np.sort(e[(e > 0.001) & (e < 0.004)])[:: max(1, int(((e > 0.001) & (e < 0.004)).sum()) // 3)][:3]
        thrs = [np.float32(0.002)]
        for v in near:
            thrs += [np.float32(v), np.nextafter(np.float32(v), np.float32(np.inf))]
        differ = 0
        for thr in thrs:
            ctx.hypothesize_async(B, seed, 0, float(thr))
            ctx.fetch_best()
            c, s = ctx.last_counts(B)
            oc, osum = est.score_models(om, float(thr))
            np.testing.assert_array_equal(c[occ], oc[occ], err_msg=str(thr))
            assert (c[~occ] < 0).all()
            cnt = oc[occ].astype(np.float64)
            bound = cnt * float(thr) * 2.0 ** -18 + np.abs(osum[occ].astype(np.float64)) * cnt * 2.0 ** -23
            err = np.abs(s[occ].astype(np.float64) - osum[occ])
            assert (err <= bound).all(), (thr, float((err / np.maximum(bound, 1e-30)).max()))
            differ += int((s[occ] != osum[occ]).sum())
        assert differ > 0  # the guarded terms are in use (Σ no longer bit-equal)
