"""The matrix-core prefilter scorer of essential matrices (kernels_e16.hip) against the exact-expression
kernel and the CPU oracle: counts exact on every (model, point) pair of a full-size cfg4 batch,
adversarial models (tiny / huge / rank-deficient / non-finite, pixel-scale coordinates), thresholds
placed exactly on pair errors, non-finite points, tiny point sets; Σ within the throughput bound
(|Σ| c 2^-23 + c thr 2^-18: guarded terms within 2^-19, fixed-point units 2^-38 thr)."""
import os

import numpy as np
import pytest

from ransac_amd import synthetic

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def e16_on(monkeypatch):
    """the scorer is the default (USAC_E16 unset or 1, read at context creation); pinned on here"""
    monkeypatch.setenv("USAC_E16", "1")


def _bound(sums_ref, counts, thr):
    c = np.maximum(counts, 0).astype(np.float64)
    return np.abs(sums_ref.astype(np.float64)) * c * 2.0 ** -23 + c * thr * 2.0 ** -18


def test_e16_counts_equal_exact_full_size(usac):
    """cfg4 size: N = 50k, B = 65536 samples, the bench's 96-chunk throughput batch: every occupied
    slot's count equals the one-chunk exact kernel's, the batch record is the same."""
    pts, _, _ = synthetic.fundamental_points(n=50000, inlier_ratio=0.3, seed=1, normalized=True)
    B, thr = 65536, 0.002
    with usac.Context(usac.ESTIMATOR.Essential, pts) as ctx:
        ctx.set_score_variant(1)
        ce, se, be = ctx.hypothesize_score(B=B, seed=5, first_hyp=0, thr=thr)
        ctx.set_score_variant(0)
        ctx.set_score_chunks(96)
        ctx.hypothesize_async(B, 5, 0, thr)
        rec = ctx.fetch_best()
        cf, sf = ctx.last_counts(B)
    occ = ce >= 0
    assert occ.sum() > 0.2 * B
    np.testing.assert_array_equal(cf[occ], ce[occ])
    err = np.abs(sf[occ].astype(np.float64) - se[occ].astype(np.float64))
    assert (err <= _bound(se[occ], ce[occ], thr)).all()
    assert rec.inliers == be["inliers"] and rec.hyp_index == be["hyp_index"]


def _adversarial_models(Egt, rng):
    base = (Egt / np.linalg.norm(Egt)).reshape(9).astype(np.float32)
    models = [base]
    for scale in (1e-6, 1e-4, 1e-2, 1.0):
        models += [base * (1 + scale * rng.standard_normal(9).astype(np.float32)) for _ in range(40)]
    models += [rng.standard_normal(9).astype(np.float32) * 10 ** rng.uniform(-20, 20) for _ in range(100)]
    rank1 = np.outer([1.0, 2.0, -1.0], [0.5, -1.0, 2.0]).reshape(9).astype(np.float32)
    models += [base * np.float32(1e30), base * np.float32(1e-30), base * np.float32(1e19), np.full(9, np.nan, np.float32),
               np.full(9, np.inf, np.float32), np.zeros(9, np.float32), rank1,
               np.array([0, 0, 0, 0, 0, 0, 0, 0, 1], np.float32), np.array([0, 0, 1, 0, 0, 0, 0, 0, 0], np.float32)]
    return base, np.stack(models).astype(np.float32)


@pytest.mark.parametrize("normalized", [True, False])
def test_e16_adversarial_models(usac, oracle, normalized):
    """Tiny / huge / rank-deficient / non-finite models on normalised and pixel-scale coordinates, and
    thresholds exactly on pair errors (and the next float): counts equal the oracle's through the
    matrix-core scorer (score variant 3)."""
    rng = np.random.default_rng(1)
    pts, Egt, _ = synthetic.fundamental_points(n=3000, inlier_ratio=0.3, seed=4, normalized=normalized)
    est = oracle.Estimator(oracle.ESSENTIAL, pts)
    base, models = _adversarial_models(Egt, rng)
    thrs = (0.002, 0.0005, 0.03) if normalized else (1.0, 0.25, 6.0)
    with usac.Context(usac.ESTIMATOR.Essential, pts) as ctx:
        ctx.set_score_variant(3)
        ctx.set_score_chunks(4)
        for thr in thrs:
            gc, gs = ctx.score_models(models, thr)
            oc, os_ = est.score_models(models, thr)
            np.testing.assert_array_equal(gc, oc)
            fin = np.isfinite(os_) & (oc > 0)
            assert (np.abs(gs[fin].astype(np.float64) - os_[fin]) <= _bound(os_[fin], oc[fin], thr)).all()
        errs = est.errors(base)
        for e in np.sort(errs[np.isfinite(errs)])[::47][:16]:
            for tt in (float(e), float(np.nextafter(np.float32(e), np.float32(np.inf)))):
                if not tt > 0:
                    continue
                gc, _ = ctx.score_models(base[None], tt)
                oc, _ = est.score_models(base[None], tt)
                assert gc[0] == oc[0], tt


def test_e16_nonfinite_and_tiny_point_sets(usac, oracle):
    """NaN / inf coordinates among the points (never inliers), and point sets of 1 .. 65 points
    (partial 32-point blocks)."""
    rng = np.random.default_rng(7)
    pts, Egt, _ = synthetic.fundamental_points(n=2000, inlier_ratio=0.4, seed=8, normalized=True)
    pts = pts.copy()
    bad = rng.choice(len(pts), 40, replace=False)
    pts[bad[:10], 0] = np.nan
    pts[bad[10:20], 3] = np.inf
    pts[bad[20:30], 1] = -np.inf
    pts[bad[30:], 2] = np.nan
    _, models = _adversarial_models(Egt, rng)
    for sub in (pts, pts[:1], pts[:31], pts[:33], pts[:65]):
        est = oracle.Estimator(oracle.ESSENTIAL, sub)
        with usac.Context(usac.ESTIMATOR.Essential, sub) as ctx:
            ctx.set_score_variant(3)
            ctx.set_score_chunks(4)
            gc, _ = ctx.score_models(models, 0.002)
        oc, _ = est.score_models(models, 0.002)
        np.testing.assert_array_equal(gc, oc)


def test_e16_off_equals_on(usac):
    """USAC_E16=0 (the lanes-over-models k_score_f2 for every throughput batch) gives the same counts."""
    pts, _, _ = synthetic.fundamental_points(n=20000, inlier_ratio=0.3, seed=9, normalized=True)
    out = []
    for flag in ("1", "0"):
        os.environ["USAC_E16"] = flag
        try:
            with usac.Context(usac.ESTIMATOR.Essential, pts) as ctx:
                ctx.set_score_chunks(32)
                ctx.hypothesize_async(16384, 3, 0, 0.002)
                rec = ctx.fetch_best()
                out.append((ctx.last_counts(16384)[0], rec.inliers, rec.hyp_index))
        finally:
            os.environ.pop("USAC_E16", None)
    np.testing.assert_array_equal(out[0][0], out[1][0])
    assert out[0][1:] == out[1][1:]
