"""The stateful plugin handles (include/usac_gpu.h ABI 11) through the Python mirror: each one's
state stream equals the oracle's restatement of the reference plugin, and the reference loop body
(ransac.cpp:58-139) written in Python against them -- one call per plugin, or batches walked by
SPRT.replay (usac_sprt_replay) -- equals the oracle's run: records, iterations, model bits,
inliers."""
import numpy as np
import pytest

from ransac_amd import synthetic

pytestmark = pytest.mark.gpu


def _model(usac, est, thr, sampler, seed, sprt=False, lo=0, nb=0):
    m = {usac.ESTIMATOR.Line2d: 2, usac.ESTIMATOR.Homography: 4, usac.ESTIMATOR.Fundamental: 7}[est]
    mdl = usac.Model(thr, m, 0.95, 7, est, sampler)
    mdl.ResetRandomGenerator(False)
    mdl.setSeed(seed)
    mdl.setSprt(sprt)
    mdl.lo = usac.LocOpt(lo)
    mdl.setNeighborsType(usac.NeighborsSearch(nb))
    return mdl


def test_uniform_sampler_handle_stream(usac, oracle):
    pts = synthetic.homography_points(n=997, inlier_ratio=0.3, seed=2)[0]
    with usac.Context(usac.ESTIMATOR.Homography, pts) as ctx:
        rng = usac.RandomGenerator(13)
        s = usac.Sampler(ctx, _model(usac, usac.ESTIMATOR.Homography, 2.0, usac.SAMPLER.Uniform, 13), rng)
        got = [s.generateSample() for _ in range(100)]  # one call at a time, then batches
        got += list(s.generateSamples(400))
        got += [s.generateSample() for _ in range(10)]
        assert s.state()["drawn"] == 510
        np.testing.assert_array_equal(np.array(got), oracle.uniform_samples(13, 997, 4, 510))
        s.close()
        rng.close()


def test_prosac_sampler_and_termination_handles(usac, oracle):
    pts = synthetic.fundamental_points(n=3000, inlier_ratio=0.4, seed=5)[0]
    with usac.Context(usac.ESTIMATOR.Fundamental, pts) as ctx:
        mdl = _model(usac, usac.ESTIMATOR.Fundamental, 2.0, usac.SAMPLER.Prosac, 21)
        s = usac.Sampler(ctx, mdl)
        t = usac.TerminationCriteria(ctx, mdl, s)
        got = s.generateSamples(700)
        ref, growth, largest = oracle.prosac_samples(21, 3000, 7, 700)
        np.testing.assert_array_equal(got, ref)
        assert s.state()["largest_sample_size"] == largest
        # the standard overloads
        for inl in (0, 100, 1000, 2500):
            assert t.getUpBoundIterations(inl) == oracle.std_termination(inl, 3000, 7, 0.95)
        t.close()
        s.close()


def test_sprt_handle_pool_and_bound(usac, oracle):
    pts = synthetic.homography_points(n=2000, inlier_ratio=0.3, seed=3)[0]
    with usac.Context(usac.ESTIMATOR.Homography, pts) as ctx:
        rng = usac.RandomGenerator(5)
        sp = usac.SPRT(ctx, _model(usac, usac.ESTIMATOR.Homography, 2.0, usac.SAMPLER.Uniform, 5, sprt=True), rng)
        # the pool shuffle consumed n draws of the shared stream: the next draw is glibc's n-th
        assert rng.next() == int(oracle.glibc_stream(5, 2001)[2000])
        assert sp.stats() == {"histories": 1, "rejected": 0}
        assert sp.getUpperBoundIterations(0) >= 0
        sp.close()
        rng.close()


def _python_loop(usac, ctx, mdl, batched):
    """ransac.cpp:14-214 in Python over the plugin handles (Ransac ctor order)."""
    rng = usac.RandomGenerator(mdl.seed)
    sampler = usac.Sampler(ctx, mdl, rng)
    lo = usac.LocalOptimization(ctx, mdl) if int(mdl.lo) else None
    prosac = mdl.sampler == usac.SAMPLER.Prosac
    term = usac.TerminationCriteria(ctx, mdl, sampler if prosac else None)
    sprt = usac.SPRT(ctx, mdl, rng) if mdl.sprt else None
    best, cur = usac.Score(), usac.Score()
    best_model = np.zeros(9, np.float32)
    iters, max_iters = 0, mdl.max_iterations
    records = []

    def new_best(model):
        nonlocal max_iters, best_model
        mm = np.array(model, np.float32).reshape(-1)
        if lo is not None:
            lo.GetModelScore(mm, cur)
        best.inlier_number, best.score = cur.inlier_number, cur.score
        best_model = mm.copy()
        max_iters = term.getUpBoundIterations(iters, best_model) if prosac else term.getUpBoundIterations(
            best.inlier_number)
        if sprt is not None:
            max_iters = min(max_iters, sprt.getUpperBoundIterations(best.inlier_number))
        records.append((iters, best.inlier_number, int(np.float32(best.score).view(np.int32))))

    S = ctx.spk
    if not batched:
        while iters < max_iters:
            smp = sampler.generateSample()
            models, nm = ctx.estimate_models(smp[None])
            models = models.reshape(-1, 9)
            for i in range(int(nm[0])):
                if sprt is not None:
                    good = sprt.verifyModelAndGetModelScore(models[i], iters, best.inlier_number, cur)
                    if not good and iters >= 20:
                        iters += 1
                        continue
                else:
                    c, s = ctx.score_models(models[i], mdl.threshold)
                    cur.inlier_number, cur.score = int(c[0]), float(s[0])
                if cur.bigger(best):
                    new_best(models[i])
            iters += 1
    else:
        B = 1 if prosac else 48
        while iters < max_iters:
            models, nm = ctx.estimate_models(sampler.generateSamples(B))
            models = np.ascontiguousarray(models.reshape(B, S, 9))
            st = usac.SprtState()
            st.iters = iters
            while True:
                st.max_iters, st.best_inliers, st.best_score = max_iters, best.inlier_number, best.score
                if not sprt.replay(models, nm, st):
                    break
                iters = st.iters
                cur.inlier_number, cur.score = st.inliers, st.score
                new_best(models[st.found_sample, st.found_slot])
            iters = st.iters
    for h in (sprt, term, lo, sampler, rng):
        if h is not None:
            h.close()
    return records, iters, best, best_model


@pytest.mark.parametrize("batched", [False, True])
@pytest.mark.parametrize("case", ["H_sprt", "F_prosac_sprt", "L_sprt_lo"])
def test_python_loop_over_plugins_equals_oracle(usac, oracle, case, batched):
    if case == "H_sprt":
        pts = synthetic.homography_points(n=3000, inlier_ratio=0.3, seed=8)[0]
        est, okind, thr, smp, lo = usac.ESTIMATOR.Homography, oracle.HOMOGRAPHY, 2.0, usac.SAMPLER.Uniform, 0
    elif case == "F_prosac_sprt":
        pts = synthetic.fundamental_points(n=3000, inlier_ratio=0.4, seed=8)[0]
        est, okind, thr, smp, lo = usac.ESTIMATOR.Fundamental, oracle.FUNDAMENTAL, 2.0, usac.SAMPLER.Prosac, 0
    else:
        pts = synthetic.line_points(n=1000, inlier_ratio=0.2, seed=8)[0]
        est, okind, thr, smp, lo = usac.ESTIMATOR.Line2d, oracle.LINE2D, 8.0, usac.SAMPLER.Uniform, 1
    seed = 6
    mdl = _model(usac, est, thr, smp, seed, sprt=True, lo=lo)
    with usac.Context(est, pts) as ctx:
        records, iters, best, best_model = _python_loop(usac, ctx, mdl, batched)
    osmp = oracle.SAMPLER_PROSAC if smp == usac.SAMPLER.Prosac else oracle.SAMPLER_UNIFORM
    ref = oracle.ransac_run(okind, pts, thr, 0.95, seed, sampler=osmp, sprt=True, lo=lo)
    assert records == [(i, c, int(np.float32(s).view(np.int32))) for i, c, s in ref["records"]]
    assert iters == ref["iters"]
    nm = 3 if est == usac.ESTIMATOR.Line2d else 9
    assert (best_model[:nm].view(np.int32) == ref["minimal_model"][:nm].view(np.int32)).all()
    assert best.inlier_number == ref["minimal_inliers"]
