"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle on the same inputs.

Bar: integer outputs (inlier counts, indices, iteration counts, record lists) bit-exact;
fp32 models and sums bit-exact too -- the device kernels evaluate the same IEEE
operation sequence as the oracle (no FMA contraction, correctly-rounded div/sqrt).  The
one declared tolerance: the throughput-mode score kernel splits the point range into
chunks, so its Σerr is a re-associated fp32 sum (rel 1e-5) while counts stay exact.
"""
import numpy as np
import pytest

from ransac_amd import synthetic

pytestmark = pytest.mark.gpu

H = 2  # ESTIMATOR.Homography
L2 = 1  # ESTIMATOR.Line2d


def _cfg2(n=2000, seed=1):
    pts, Hgt, inl = synthetic.homography_points(n=n, inlier_ratio=0.3, seed=seed)
    return pts, Hgt


# ----------------------------------------------------------------------------- scoring
def test_score_gt_models_real_scenes(usac, oracle, homography_scenes):
    """Golden: GT models on the reference's 12 scenes -> published GT inlier counts."""
    for scene, (pts, model, gt) in homography_scenes.items():
        ctx = usac.Context(usac.ESTIMATOR.Homography, pts)
        inv, _ = oracle.inv3x3(model)
        c, s = ctx.score_models(np.stack([model, inv]), 2.0)
        assert max(c) == gt, scene
        est = oracle.Estimator(oracle.HOMOGRAPHY, pts)
        for k, m in enumerate((model, inv)):
            oc, osum = est.quality(m, 2.0)
            assert c[k] == oc and np.float32(s[k]) == np.float32(osum), scene
        ctx.close()


def test_score_random_models_bit_exact(usac, oracle):
    pts, Hgt = _cfg2(3000)
    est = oracle.Estimator(oracle.HOMOGRAPHY, pts)
    samples = oracle.uniform_samples(5, len(pts), 4, 512)
    models, _ = est.estimate_batch(samples)
    models[::7] = models[::7] + np.float32(1e-3)      # perturbed, still near-valid
    models[3] = 0.0                                     # singular -> zero inverse, NaN errors
    oc, os_ = est.score_models(models, 2.0)
    with usac.Context(usac.ESTIMATOR.Homography, pts) as ctx:
        gc, gs = ctx.score_models(models, 2.0)
    np.testing.assert_array_equal(gc, oc)
    np.testing.assert_array_equal(gs.view(np.int32), os_.view(np.int32))


def test_score_line2d_bit_exact(usac, oracle, line2d_scenes):
    pts, gt, _ = next(iter(sorted(line2d_scenes.items())))[1]
    est = oracle.Estimator(oracle.LINE2D, pts)
    samples = oracle.uniform_samples(3, len(pts), 2, 256)
    models, _ = est.estimate_batch(samples)
    oc, os_ = est.score_models(models, 10.0)
    with usac.Context(usac.ESTIMATOR.Line2d, pts) as ctx:
        gc, gs = ctx.score_models(models[:, :3], 10.0)
        gm, _ = ctx.estimate_models(samples)
    np.testing.assert_array_equal(gc, oc)
    np.testing.assert_array_equal(gs.view(np.int32), os_.view(np.int32))
    np.testing.assert_array_equal(gm.view(np.int32), models.view(np.int32))


# ----------------------------------------------------------------------------- solver
@pytest.mark.parametrize("mode", [0, 1])
def test_dlt4_models_bit_exact(usac, oracle, homography_scenes, mode):
    cases = [_cfg2(2000)[0], homography_scenes["adam"][0], homography_scenes["Brussels"][0]]
    for pts in cases:
        est = oracle.Estimator(oracle.HOMOGRAPHY, pts, mode)
        samples = oracle.uniform_samples(9, len(pts), 4, 1024)
        om, _ = est.estimate_batch(samples)
        with usac.Context(usac.ESTIMATOR.Homography, pts) as ctx:
            ctx.set_dlt_mode(mode)
            gm, nm = ctx.estimate_models(samples)
        assert (nm == 1).all()
        same = (gm.view(np.int32) == om.view(np.int32)) | (np.isnan(gm) & np.isnan(om))
        assert same.all(), "first mismatch at sample %d" % int(np.argmin(same.all(1)))


def test_dlt4_qr_fallbacks_bit_exact(usac, oracle):
    """The thin DLT's QR + inverse-iteration spec and its row-Jacobi fall-back (k_solve_h4 ->
    k_solve_h4_jac over the fall-back list): a full cfg2-size batch (~2.4e-4 of its samples fall
    back on a close sigma_7 / sigma_8 pair) plus degenerate samples (repeated points: rank-
    deficient rows; all-zero points: a zero column norm; a non-finite point)."""
    pts, _ = _cfg2(10000, seed=4)
    pts = pts.copy()
    pts[17] = 0.0
    pts[18] = 0.0
    pts[19] = [np.inf, 1.0, 2.0, 3.0]
    samples = oracle.uniform_samples(11, len(pts), 4, 65536)
    samples[:64] = [[5, 5, 9, 13], [17, 18, 17, 18], [17, 18, 20, 21], [19, 1, 2, 3]] * 16
    samples[64:128, 1] = samples[64:128, 0]
    est = oracle.Estimator(oracle.HOMOGRAPHY, pts)
    om, _ = est.estimate_batch(samples)
    with usac.Context(usac.ESTIMATOR.Homography, pts) as ctx:
        for _ in range(2):  # the second solve starts from the counters the first one reset
            gm, nm = ctx.estimate_models(samples)
            assert (nm == 1).all()
            same = (gm.view(np.int32) == om.view(np.int32)) | (np.isnan(gm) & np.isnan(om))
            assert same.all(), "first mismatch at sample %d" % int(np.argmin(same.all(1)))


def test_fused_batch_matches_oracle(usac, oracle):
    pts, _ = _cfg2(4000)
    samples = oracle.uniform_samples(21, len(pts), 4, 4096)
    est = oracle.Estimator(oracle.HOMOGRAPHY, pts)
    om, _ = est.estimate_batch(samples)
    oc, os_ = est.score_models(om, 2.0)
    with usac.Context(usac.ESTIMATOR.Homography, pts) as ctx:
        c, s, best = ctx.hypothesize_score(samples=samples, thr=2.0, first_hyp=100)
    np.testing.assert_array_equal(c, oc)
    np.testing.assert_array_equal(s.view(np.int32), os_.view(np.int32))
    # batch best: Score::bigger, earliest index on exact ties
    order = sorted(range(len(oc)), key=lambda i: (-oc[i], -os_[i], i))
    assert best["hyp_index"] == 100 + order[0] and best["inliers"] == oc[order[0]]
    np.testing.assert_array_equal(best["model"], om[order[0]])


# ----------------------------------------------------------------------------- inliers / LSQ
def test_get_inliers_exact(usac, oracle, homography_scenes):
    est = oracle.Estimator(oracle.HOMOGRAPHY, homography_scenes["Boston"][0])
    with usac.Context(usac.ESTIMATOR.Homography, homography_scenes["Boston"][0]) as ctx:
        for scene in ("Boston", "Boston", "graf", "city"):
            pts, model, gt = homography_scenes[scene]
            if scene != "Boston":
                ctx.close()
                ctx = usac.Context(usac.ESTIMATOR.Homography, pts)
                est = oracle.Estimator(oracle.HOMOGRAPHY, pts)
            for m in (model, oracle.inv3x3(model)[0]):
                oc, os_, oidx = est.quality(m, 2.0, with_inliers=True)
                c, s, idx = ctx.get_inliers(m, 2.0)
                assert c == oc and np.float32(s) == np.float32(os_)
                np.testing.assert_array_equal(idx, oidx)


def test_nonminimal_matches_oracle(usac, oracle, homography_scenes):
    pts, model, gt = homography_scenes["Boston"]
    est = oracle.Estimator(oracle.HOMOGRAPHY, pts)
    inv, _ = oracle.inv3x3(model)
    cands = [est.quality(m, 2.0, with_inliers=True) for m in (model, inv)]
    idx = max(cands, key=lambda r: r[0])[2]
    assert len(idx) == gt
    with usac.Context(usac.ESTIMATOR.Homography, pts) as ctx:
        for sub in (idx, idx[:4], idx[:3], idx[:57], idx[:200]):
            g = ctx.nonminimal(sub)
            o = est.nonminimal(sub)
            np.testing.assert_array_equal(g.view(np.int32), o.view(np.int32))


def test_nonminimal_line_matches_oracle(usac, oracle, line2d_scenes):
    pts, gt, _ = next(iter(sorted(line2d_scenes.items())))[1]
    est = oracle.Estimator(oracle.LINE2D, pts)
    _, _, idx = est.quality(gt, 10.0, with_inliers=True)
    with usac.Context(usac.ESTIMATOR.Line2d, pts) as ctx:
        g = ctx.nonminimal(idx)
    o = est.nonminimal(idx)
    np.testing.assert_array_equal(g[:3].view(np.int32), o[:3].view(np.int32))


# ----------------------------------------------------------------------------- Ransac::run
@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("mode", [0, 1])
def test_ransac_run_homography_identical(usac, oracle, homography_scenes, seed, mode):
    for pts in (homography_scenes["adam"][0], _cfg2(3000, seed=seed)[0]):
        o = oracle.ransac_run(oracle.HOMOGRAPHY, pts, 2.0, 0.95, seed, dlt_mode=mode)
        model = usac.Model(2.0, 4, 0.95, 7, usac.ESTIMATOR.Homography, usac.SAMPLER.Uniform)
        model.ResetRandomGenerator(False)
        model.setSeed(seed)
        model.setDLTMode(mode)
        model.batch = 512
        r = usac.Ransac(model, pts)
        r.run()
        out = r.getRansacOutput()
        assert r.records == o["records"]
        assert out.getNumberOfMainIterations() == o["iters"]
        assert out.getNumberOfInliers() == o["inliers"]
        np.testing.assert_array_equal(out.getModel().view(np.int32), o["model"].view(np.int32))
        np.testing.assert_array_equal(out.getInliers(), o["inlier_idx"])


@pytest.mark.parametrize("seed", [1, 5])
def test_ransac_run_line2d_identical(usac, oracle, line2d_scenes, seed):
    pts, gt, _ = next(iter(sorted(line2d_scenes.items())))[1]
    o = oracle.ransac_run(oracle.LINE2D, pts, 10.0, 0.99, seed)
    model = usac.Model(10.0, 2, 0.99, 7, usac.ESTIMATOR.Line2d, usac.SAMPLER.Uniform)
    model.setSeed(seed)
    model.ResetRandomGenerator(False)
    r = usac.Ransac(model, pts)
    r.run()
    out = r.getRansacOutput()
    assert r.records == o["records"]
    assert out.getNumberOfMainIterations() == o["iters"]
    assert out.getNumberOfInliers() == o["inliers"]
    np.testing.assert_array_equal(out.getInliers(), o["inlier_idx"])


# ----------------------------------------------------------------------------- guard band
def test_fast_kernel_equals_exact_kernel_full_size(usac):
    """Guard-band fast path vs the exact-expression kernel on every (hypothesis, point)
    pair of a BASELINE-size batch (N = 10k, B = 65536): identical counts (chunked and
    sequential), identical sequential sums."""
    pts, _ = _cfg2(10000, seed=2)
    with usac.Context(usac.ESTIMATOR.Homography, pts) as ctx:
        for mode in (0, 1):
            ctx.set_dlt_mode(mode)
            ctx.set_score_variant(1)
            ce, se, be = ctx.hypothesize_score(B=65536, seed=99, first_hyp=0, thr=2.0)
            ctx.set_score_variant(0)
            cf, sf, bf = ctx.hypothesize_score(B=65536, seed=99, first_hyp=0, thr=2.0)
            np.testing.assert_array_equal(cf, ce)
            np.testing.assert_array_equal(sf.view(np.int32), se.view(np.int32))
            assert bf["hyp_index"] == be["hyp_index"]
            for chunks in (2, 4, 8):
                ctx.set_score_chunks(chunks)
                ctx.hypothesize_async(65536, 99, 0, 2.0)
                rec = ctx.fetch_best()
                assert rec.inliers == be["inliers"]


def test_fast_kernel_adversarial_models(usac, oracle):
    """Models built to put pairs on the threshold, near-zero denominators, huge entries."""
    rng = np.random.default_rng(0)
    pts, Hgt = _cfg2(2000, seed=4)
    est = oracle.Estimator(oracle.HOMOGRAPHY, pts)
    base = (Hgt / Hgt[2, 2]).reshape(9).astype(np.float32)
    models = [base]
    for scale in (1e-6, 1e-4, 1e-2, 1.0):
        models += [base * (1 + scale * rng.standard_normal(9).astype(np.float32)) for _ in range(40)]
    models += [rng.standard_normal(9).astype(np.float32) * 10 ** rng.uniform(-20, 20) for _ in range(100)]
    tiny = base.copy(); tiny[6:] = [1e-30, -1e-30, 1e-38]
    models += [tiny, base * np.float32(1e30), base * np.float32(1e-30), np.full(9, np.nan, np.float32)]
    models = np.stack(models).astype(np.float32)
    thresholds = [2.0, 0.5, 7.3]
    with usac.Context(usac.ESTIMATOR.Homography, pts) as ctx:
        for thr in thresholds:
            gc, gs = ctx.score_models(models, thr)
            oc, os_ = est.score_models(models, thr)
            np.testing.assert_array_equal(gc, oc)
            np.testing.assert_array_equal(gs.view(np.int32), os_.view(np.int32))
            # put points exactly on the threshold: thr := the exact error of some pairs
            errs = est.errors(base)
            for e in np.sort(errs[np.isfinite(errs)])[::97][:8]:
                t = float(e)
                for tt in (t, float(np.nextafter(np.float32(t), np.float32(np.inf)))):
                    gc, _ = ctx.score_models(base[None], tt)
                    oc, _ = est.score_models(base[None], tt)
                    assert gc[0] == oc[0], tt


# ----------------------------------------------------------------------------- full size
def test_full_size_device_sampler_properties(usac, oracle):
    """BASELINE cfg2 size (N = 10k, B = 65536), device sampler: size-independent checks."""
    pts, Hgt = _cfg2(10000, seed=1)
    B = 65536
    with usac.Context(usac.ESTIMATOR.Homography, pts) as ctx:
        c, s, best = ctx.hypothesize_score(B=B, seed=1234, first_hyp=0, thr=2.0)
        c2, s2, best2 = ctx.hypothesize_score(B=B, seed=1234, first_hyp=0, thr=2.0)
        ctx.hypothesize_async(B, 1234, 0, 2.0)
        ab = ctx.fetch_best()
        n, ssum, idx = ctx.get_inliers(best["model"], 2.0)
    np.testing.assert_array_equal(c, c2)                         # deterministic sampler
    assert best["hyp_index"] == best2["hyp_index"] and best["inliers"] == best2["inliers"]
    assert (c >= 0).all() and (c <= len(pts)).all()
    assert best["inliers"] == c.max() == n                       # argmax + exact recount
    assert ab.inliers == best["inliers"]                         # chunked kernel: same counts
    assert abs(ab.score - best["score"]) <= 1e-5 * max(1.0, best["score"])
    est = oracle.Estimator(oracle.HOMOGRAPHY, pts)
    oc, os_ = est.quality(best["model"], 2.0)
    assert oc == n and np.float32(os_) == np.float32(ssum)
    assert (idx[1:] > idx[:-1]).all()                              # ascending, unique


@pytest.mark.parametrize("kind", ["H", "F"])
def test_nonminimal_sizes_bit_exact(usac, oracle, kind):
    """Non-minimal fits on both sides of the one-workgroup small-fit kernel (<= 256 points), the
    64-point block and 4096-point superblock edges, on clean inlier subsets (inverse iteration)
    and on outlier-contaminated ones (the Jacobi fall-back of the eigen spec)."""
    from ransac_amd import synthetic as syn
    if kind == "H":
        pts, _, inl = syn.homography_points(n=12000, inlier_ratio=0.5, seed=21)
        est_o, est_u = oracle.HOMOGRAPHY, usac.ESTIMATOR.Homography
    else:
        pts, _, inl = syn.fundamental_points(n=12000, inlier_ratio=0.5, seed=21, prosac_order=False)
        est_o, est_u = oracle.FUNDAMENTAL, usac.ESTIMATOR.Fundamental
    inliers = np.flatnonzero(inl)
    est = oracle.Estimator(est_o, pts)
    rng = np.random.default_rng(5)
    with usac.Context(est_u, pts) as ctx:
        for k in (5, 9, 14, 63, 64, 65, 255, 256, 257, 4096, 4097, 9000):
            for contaminated in (False, True):
                pool = inliers if not contaminated else np.arange(12000)
                idx = np.sort(rng.choice(pool, size=min(k, len(pool)), replace=False)).astype(np.int32)
                g = ctx.nonminimal(idx)
                o = est.nonminimal(idx)
                np.testing.assert_array_equal(g.view(np.int32), o.view(np.int32), err_msg="%s %d %s" % (kind, k, contaminated))
