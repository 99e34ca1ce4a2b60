"""The matrix-core prefilter scorer of homographies (kernels_h16.hip) against the exact-expression
kernel and the CPU oracle: counts exact on every (hypothesis, point) pair of full-size batches,
adversarial models, thresholds placed on pair errors, non-finite points, tiny point sets; Σ within
the throughput bound (timed_kernel_parity's: |Σ| c 2^-23 + c (2^-22 Mp + 2^-18 thr))."""
import os

import numpy as np
import pytest

from ransac_amd import synthetic

pytestmark = pytest.mark.gpu


def _bound(sums_ref, counts, pts, thr):
    c = np.maximum(counts, 0).astype(np.float64)
    mp = float(np.abs(pts[np.isfinite(pts).all(1)].astype(np.float64)).sum(1).max())
    return np.abs(sums_ref.astype(np.float64)) * c * 2.0 ** -23 + c * (2.0 ** -22 * mp + 2.0 ** -18 * thr)


@pytest.mark.parametrize("dlt", [0, 1])
def test_h16_counts_equal_exact_full_size(usac, dlt):
    """cfg2 size: N = 10k, B = 65536; every hypothesis' count equals the exact kernel's."""
    pts, _, _ = synthetic.homography_points(n=10000, inlier_ratio=0.3, seed=2)
    B, thr = 65536, 2.0
    with usac.Context(usac.ESTIMATOR.Homography, pts) as ctx:
        ctx.set_dlt_mode(dlt)
        ctx.set_score_variant(1)
        ce, se, be = ctx.hypothesize_score(B=B, seed=99, first_hyp=0, thr=thr)
        ctx.set_score_variant(0)
        ctx.set_score_chunks(8)
        ctx.hypothesize_async(B, 99, 0, thr)
        rec = ctx.fetch_best()
        cf, sf = ctx.last_counts(B)
    np.testing.assert_array_equal(cf, ce)
    err = np.abs(sf.astype(np.float64) - se.astype(np.float64))
    assert (err <= _bound(se, ce, pts, thr)).all()
    assert rec.inliers == be["inliers"]


def test_h16_loop_batch_clustered_100k(usac):
    """cfg5-shaped batches through the hypothesize API: 8192 hypotheses over 100k clustered points (many point chunks)."""
    pts, _, _ = synthetic.homography_points(n=100000, inlier_ratio=0.2, seed=3, cluster=(500, 500, 150))
    B, thr = 8192, 2.0
    with usac.Context(usac.ESTIMATOR.Homography, pts) as ctx:
        ctx.set_score_variant(1)
        ce, se, _ = ctx.hypothesize_score(B=B, seed=5, first_hyp=0, thr=thr)
        ctx.set_score_variant(0)
        ctx.set_score_chunks(8)
        ctx.hypothesize_async(B, 5, 0, thr)
        ctx.fetch_best()
        cf, sf = ctx.last_counts(B)
    np.testing.assert_array_equal(cf, ce)
    assert (np.abs(sf.astype(np.float64) - se) <= _bound(se, ce, pts, thr)).all()


def _adversarial_models(Hgt, rng):
    base = (Hgt / Hgt[2, 2]).reshape(9).astype(np.float32)
    models = [base]
    for scale in (1e-6, 1e-4, 1e-2, 1.0):
        models += [base * (1 + scale * rng.standard_normal(9).astype(np.float32)) for _ in range(40)]
    models += [rng.standard_normal(9).astype(np.float32) * 10 ** rng.uniform(-20, 20) for _ in range(100)]
    tiny = base.copy()
    tiny[6:] = [1e-30, -1e-30, 1e-38]
    singular = np.array([1, 2, 3, 2, 4, 6, 1e-3, 2e-3, 3e-3], np.float32)
    models += [tiny, base * np.float32(1e30), base * np.float32(1e-30), np.full(9, np.nan, np.float32),
               np.full(9, np.inf, np.float32), np.zeros(9, np.float32), singular]
    return base, np.stack(models).astype(np.float32)


def test_h16_adversarial_models(usac, oracle):
    """Tiny / huge / singular / non-finite models and thresholds exactly on pair errors (and the next
    float): counts equal the oracle's through the multi-chunk scorer (score variant 3)."""
    rng = np.random.default_rng(0)
    pts, Hgt, _ = synthetic.homography_points(n=3000, inlier_ratio=0.3, seed=4)
    est = oracle.Estimator(oracle.HOMOGRAPHY, pts)
    base, models = _adversarial_models(Hgt, rng)
    with usac.Context(usac.ESTIMATOR.Homography, pts) as ctx:
        ctx.set_score_variant(3)
        ctx.set_score_chunks(4)
        for thr in (2.0, 0.5, 7.3):
            gc, gs = ctx.score_models(models, thr)
            oc, os_ = est.score_models(models, thr)
            np.testing.assert_array_equal(gc, oc)
            fin = np.isfinite(os_)
            assert (np.abs(gs[fin].astype(np.float64) - os_[fin]) <= _bound(os_[fin], oc[fin], pts, thr)).all()
        errs = est.errors(base)
        for e in np.sort(errs[np.isfinite(errs)])[::61][:12]:
            for tt in (float(e), float(np.nextafter(np.float32(e), np.float32(np.inf)))):
                gc, _ = ctx.score_models(base[None], tt)
                oc, _ = est.score_models(base[None], tt)
                assert gc[0] == oc[0], tt


def test_h16_nonfinite_and_tiny_point_sets(usac, oracle):
    """NaN / inf coordinates among the points (never inliers), and point sets of 1 .. 65 points
    (partial 32-point blocks)."""
    rng = np.random.default_rng(7)
    pts, Hgt, _ = synthetic.homography_points(n=2000, inlier_ratio=0.4, seed=8)
    pts = pts.copy()
    bad = rng.choice(len(pts), 40, replace=False)
    pts[bad[:10], 0] = np.nan
    pts[bad[10:20], 3] = np.inf
    pts[bad[20:30], 1] = -np.inf
    pts[bad[30:], 2] = np.nan
    _, models = _adversarial_models(Hgt, rng)
    for sub in (pts, pts[:1], pts[:31], pts[:33], pts[:65]):
        est = oracle.Estimator(oracle.HOMOGRAPHY, sub)
        with usac.Context(usac.ESTIMATOR.Homography, sub) as ctx:
            ctx.set_score_variant(3)
            ctx.set_score_chunks(4)
            gc, _ = ctx.score_models(models, 2.0)
        oc, _ = est.score_models(models, 2.0)
        np.testing.assert_array_equal(gc, oc)


def test_h16_off_equals_on(usac):
    """USAC_H16=0 (the lanes-over-hypotheses k_score_hf for every batch) gives the same counts."""
    pts, _, _ = synthetic.homography_points(n=10000, inlier_ratio=0.3, seed=9)
    out = []
    for flag in ("1", "0"):
        os.environ["USAC_H16"] = flag
        try:
            with usac.Context(usac.ESTIMATOR.Homography, pts) as ctx:
                ctx.set_score_chunks(8)
                ctx.hypothesize_async(16384, 3, 0, 2.0)
                rec = ctx.fetch_best()
                out.append((ctx.last_counts(16384)[0], rec.inliers, rec.hyp_index))
        finally:
            os.environ.pop("USAC_H16", None)
    np.testing.assert_array_equal(out[0][0], out[1][0])
    assert out[0][1:] == out[1][1:]


def test_h16_pipelined_contexts(usac):
    """bench.py's pipeline: three contexts with batches in flight on their own streams; every batch's
    counts equal the same batch scored alone by the exact one-chunk kernel (tools/h16_concurrency_check.py)."""
    pts, _, _ = synthetic.homography_points(n=10000, inlier_ratio=0.3, seed=1)
    B, N, P, thr = 16384, 9, 3, 2.0
    ctxs = [usac.Context(usac.ESTIMATOR.Homography, pts) for _ in range(P)]
    try:
        for c in ctxs:
            c.set_score_chunks(8)
        got = {}
        for i in range(N + P - 1):
            if i < N:
                ctxs[i % P].hypothesize_async(B, 1, i * B, thr)
            j = i - P + 1
            if j >= 0:
                ctxs[j % P].fetch_best()
                got[j] = ctxs[j % P].last_counts(B)[0].copy()
        ctxs[0].set_score_variant(1)
        for j in range(N):
            cnt, _, _ = ctxs[0].hypothesize_score(B=B, seed=1, first_hyp=j * B, thr=thr)
            np.testing.assert_array_equal(got[j], cnt)
    finally:
        for c in ctxs:
            c.close()
