"""GPU parity of the whole Ransac::run loop (usac_ransac_run) against the oracle for every
sampler x SPRT x estimator combination of ABI v2: iteration count (SPRT double counting
included), the sequence of best-score updates (iteration, count, fp32 score bits), the
minimal model, the polish, the final model and inlier list, SPRT rejections / history
length and PROSAC's final termination length -- all exact.
"""
import numpy as np
import pytest

from ransac_amd import synthetic

pytestmark = pytest.mark.gpu


def _data(kind, seed, prosac):
    if kind == "F":
        pts, _, _ = synthetic.fundamental_points(n=3000, inlier_ratio=0.3, seed=seed, prosac_order=prosac)
    elif kind == "H":
        pts, _, inl = synthetic.homography_points(n=3000, inlier_ratio=0.3, seed=seed)
        if prosac:  # PROSAC expects quality-sorted correspondences: inliers first (noisy order)
            q = np.random.default_rng(seed).uniform(0, 1, len(pts)) + 0.5 * inl
            pts = pts[np.argsort(-q, kind="stable")]
    else:
        pts, _ = synthetic.line_points(n=1000, inlier_ratio=0.2, seed=seed)
    return np.ascontiguousarray(pts)


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.int32)


@pytest.mark.parametrize("kind", ["H", "F", "L"])
@pytest.mark.parametrize("sampler", ["uniform", "prosac"])
@pytest.mark.parametrize("sprt", [False, True])
@pytest.mark.parametrize("seed", [1, 2])
def test_loop_identical(usac, oracle, kind, sampler, sprt, seed):
    pts = _data(kind, seed, sampler == "prosac")
    okind = {"H": oracle.HOMOGRAPHY, "F": oracle.FUNDAMENTAL, "L": oracle.LINE2D}[kind]
    est = {"H": usac.ESTIMATOR.Homography, "F": usac.ESTIMATOR.Fundamental, "L": usac.ESTIMATOR.Line2d}[kind]
    thr = 2.0 if kind != "L" else 8.0
    osmp = oracle.SAMPLER_PROSAC if sampler == "prosac" else oracle.SAMPLER_UNIFORM
    ref = oracle.ransac_run(okind, pts, thr, 0.95, seed, sampler=osmp, sprt=sprt)
    m = usac.Model(thr, {"H": 4, "F": 7, "L": 2}[kind], 0.95, 7, est,
                   usac.SAMPLER.Prosac if sampler == "prosac" else usac.SAMPLER.Uniform)
    m.ResetRandomGenerator(False)
    m.setSeed(seed)
    m.setSprt(sprt)
    m.batch = 512
    r = usac.Ransac(m, pts)
    r.run()
    out = r.getRansacOutput()
    assert out.getNumberOfMainIterations() == ref["iters"]
    assert [(i, c) for i, c, _ in r.records] == [(i, c) for i, c, _ in ref["records"]]
    assert [np.float32(s) for _, _, s in r.records] == [np.float32(s) for _, _, s in ref["records"]]
    assert out.raw["sprt_rejected"] == ref["sprt_rejected"]
    assert out.raw["sprt_histories"] == ref["sprt_histories"]
    assert out.raw["prosac_term_len"] == ref["prosac_term_len"]
    assert (_bits(out.raw["minimal_model"]) == _bits(ref["minimal_model"])).all()
    assert out.raw["polish_passes"] == ref["polish_passes"]
    assert (_bits(out.getModel()) == _bits(ref["model"])).all()
    assert out.getNumberOfInliers() == ref["inliers"]
    assert (out.getInliers() == ref["inlier_idx"]).all()


def test_prosac_speculative_batches_roll_back(usac, oracle):
    """Large speculative batches must give the same run as batch 1 (every rollback path)."""
    pts = _data("F", 3, True)
    outs = []
    for batch in (1, 7, 4096):
        m = usac.Model(2.0, 7, 0.99, 7, usac.ESTIMATOR.Fundamental, usac.SAMPLER.Prosac)
        m.ResetRandomGenerator(False)
        m.setSeed(3)
        m.batch = batch
        r = usac.Ransac(m, pts)
        r.run()
        o = r.getRansacOutput()
        outs.append((o.getNumberOfMainIterations(), r.records, _bits(o.getModel()).tolist(), o.raw["rollbacks"]))
    assert outs[0][:3] == outs[1][:3] == outs[2][:3]
    ref = oracle.ransac_run(oracle.FUNDAMENTAL, pts, 2.0, 0.99, 3, sampler=oracle.SAMPLER_PROSAC)
    assert outs[0][0] == ref["iters"]


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_cfg1_generator_loop_identical(usac, oracle, seed):
    """cfg1 (BASELINE configs[0]): Line2d + Uniform on 1 000 points from the reference's own
    generator (Generate2DLinePoints restated; it rewrites dataset/line2d bit for bit at the
    printed digits, test_oracle.py) -- the device loop equals the oracle's run."""
    pts, gt = oracle.generate_line2d(seed, 3.0, 100, 900, 1000, 1000)
    ref = oracle.ransac_run(oracle.LINE2D, pts, 10.0, 0.99, seed)
    m = usac.Model(10.0, 2, 0.99, 7, usac.ESTIMATOR.Line2d, usac.SAMPLER.Uniform)
    m.ResetRandomGenerator(False)
    m.setSeed(seed)
    r = usac.Ransac(m, pts)
    r.run()
    out = r.getRansacOutput()
    assert out.getNumberOfMainIterations() == ref["iters"]
    assert [(i, c) for i, c, _ in r.records] == [(i, c) for i, c, _ in ref["records"]]
    assert (_bits(out.getModel()) == _bits(ref["model"])).all()
    assert out.getNumberOfInliers() == ref["inliers"]
    assert (out.getInliers() == ref["inlier_idx"]).all()
    # the generator's line is found: |cos| between normals ~1
    mdl = out.getModel()[:2]
    assert abs(float(np.dot(mdl, gt[:2]))) / float(np.linalg.norm(mdl)) > 0.99


def _run_loop(usac, pts, est, sampler, thr, seed, lo, spec):
    import os
    mdl = usac.Model(thr, 4 if est == usac.ESTIMATOR.Homography else 2, 0.99, 7, est, sampler)
    mdl.ResetRandomGenerator(False)
    mdl.setSeed(seed)
    mdl.lo = usac.LocOpt(lo)
    mdl.max_iterations = 20000
    mdl.setNeighborsType(usac.NeighborsSearch.Grid)
    if spec:
        os.environ.pop("USAC_NO_SPECULATION", None)
    else:
        os.environ["USAC_NO_SPECULATION"] = "1"
    try:
        r = usac.Ransac(mdl, pts)
        r.run()
    finally:
        os.environ.pop("USAC_NO_SPECULATION", None)
    return r.getRansacOutput(), r.records


@pytest.mark.parametrize("loop_h16", ["0", "1"])
def test_speculation_on_off_identical(usac, loop_h16, monkeypatch):
    """The loop's next batch drawn and solved ahead of the replay: with the library's
    ramping batches, runs with and without the speculation give the same records, iterations,
    model bits and inliers -- Uniform and NAPSAC, with and without LO -- and the journal rollback
    (a speculative batch cut short by a new termination bound) is exercised.  loop_h16 = "1"
    (USAC_LOOP_H16): the speculative batches scored by the matrix-core k_score_h16 beside the main
    stream's exact recount and LO kernels -- the configuration that miscounted in round 5 (packed
    fp32 beside MFMA waves)."""
    monkeypatch.setenv("USAC_LOOP_H16", loop_h16)
    rollbacks = batches = 0
    for kind, sampler, lo in [("H", usac.SAMPLER.Uniform, 0), ("H", usac.SAMPLER.Uniform, 1),
                              ("Hc", usac.SAMPLER.Napsac, 0), ("Hc", usac.SAMPLER.Napsac, 1),
                              ("L", usac.SAMPLER.Uniform, 0)]:
        for seed in (1, 2, 3):
            if kind == "H":
                pts = synthetic.homography_points(n=6000, inlier_ratio=0.25, seed=seed)[0]
            elif kind == "Hc":
                pts = synthetic.homography_points(n=20000, inlier_ratio=0.15, seed=seed, cluster=(500, 500, 150))[0]
            else:
                pts = synthetic.line_points(n=3000, inlier_ratio=0.05, seed=seed)[0]
            est = usac.ESTIMATOR.Line2d if kind == "L" else usac.ESTIMATOR.Homography
            thr = 8.0 if kind == "L" else 2.0
            a, ra = _run_loop(usac, pts, est, sampler, thr, seed, lo, True)
            b, rb = _run_loop(usac, pts, est, sampler, thr, seed, lo, False)
            assert ra == rb, (kind, lo, seed)
            assert a.getNumberOfMainIterations() == b.getNumberOfMainIterations()
            assert (_bits(a.getModel()) == _bits(b.getModel())).all()
            assert np.array_equal(a.getInliers(), b.getInliers())
            assert a.getLOIters() == b.getLOIters()
            assert b.raw["spec_batches"] == 0
            batches += a.raw["spec_batches"]
            rollbacks += a.raw["spec_rollbacks"]
    assert batches > 0 and rollbacks > 0, (batches, rollbacks)


@pytest.mark.parametrize("kind", ["H", "F", "L"])
def test_polish_groups_identical(usac, oracle, kind):
    """The polish passes go out in groups (USAC_POLISH_GROUP; k_polish_prep takes each pass's
    acceptance on the device): one pass per submission, two, and all four give the oracle's
    polish -- passes, final model bits, inlier list."""
    import os
    okind = {"H": oracle.HOMOGRAPHY, "F": oracle.FUNDAMENTAL, "L": oracle.LINE2D}[kind]
    est = {"H": usac.ESTIMATOR.Homography, "F": usac.ESTIMATOR.Fundamental, "L": usac.ESTIMATOR.Line2d}[kind]
    thr = 2.0 if kind != "L" else 8.0
    passes = set()
    for seed in (1, 2, 3, 4):
        pts = _data(kind, seed, False)
        ref = oracle.ransac_run(okind, pts, thr, 0.95, seed)
        passes.add(ref["polish_passes"])
        for g in ("1", "2", "4"):
            os.environ["USAC_POLISH_GROUP"] = g
            try:
                m = usac.Model(thr, {"H": 4, "F": 7, "L": 2}[kind], 0.95, 7, est, usac.SAMPLER.Uniform)
                m.ResetRandomGenerator(False)
                m.setSeed(seed)
                r = usac.Ransac(m, pts)
                r.run()
            finally:
                os.environ.pop("USAC_POLISH_GROUP", None)
            out = r.getRansacOutput()
            assert out.raw["polish_passes"] == ref["polish_passes"], (seed, g)
            assert (_bits(out.getModel()) == _bits(ref["model"])).all(), (seed, g)
            assert (out.getInliers() == ref["inlier_idx"]).all(), (seed, g)
    assert max(passes) >= 1


@pytest.mark.parametrize("kind", ["F", "L"])
def test_prosac_sprt_mask_inlier_lists(usac, oracle, kind):
    """PROSAC + SPRT: a new best's inlier list (PROSAC's termination input) is decoded from the
    model's SPRT mask row on the host; USAC_CHECK_MASK_LIST=1 makes the library also run the
    device getInliers at every update and fail the run on any difference.  The runs equal the
    oracle's, and the device-list path (USAC_DEVICE_INLIERS=1) gives the same runs."""
    import os
    okind = {"F": oracle.FUNDAMENTAL, "L": oracle.LINE2D}[kind]
    est = {"F": usac.ESTIMATOR.Fundamental, "L": usac.ESTIMATOR.Line2d}[kind]
    thr = 2.0 if kind != "L" else 8.0
    for seed in (1, 2, 3):
        pts = _data(kind, seed, True)
        ref = oracle.ransac_run(okind, pts, thr, 0.95, seed, sampler=oracle.SAMPLER_PROSAC, sprt=True)
        runs = []
        for env in ("USAC_CHECK_MASK_LIST", "USAC_DEVICE_INLIERS"):
            os.environ[env] = "1"
            try:
                m = usac.Model(thr, {"F": 7, "L": 2}[kind], 0.95, 7, est, usac.SAMPLER.Prosac)
                m.ResetRandomGenerator(False)
                m.setSeed(seed)
                m.setSprt(True)
                m.batch = 64
                r = usac.Ransac(m, pts)
                r.run()
            finally:
                os.environ.pop(env, None)
            out = r.getRansacOutput()
            runs.append((out.getNumberOfMainIterations(), r.records, out.raw["prosac_term_len"]))
        assert runs[0] == runs[1], seed
        assert runs[0][0] == ref["iters"] and runs[0][2] == ref["prosac_term_len"], seed


def test_sprt_batch_copy_paths_identical(usac, oracle):
    """PROSAC + SPRT runs with the round-5 host paths switched off one by one -- the batch's
    counts / list / models copied behind its mask words (USAC_NO_POOL_TAIL), the pool shuffle
    behind the first solve (USAC_NO_DEFER_POOL), the inlier lists decoded from the masks
    (USAC_DEVICE_INLIERS), the word-run SPRT walk (USAC_SPRT_PLAIN_WALK) -- give the same runs,
    equal to the oracle's; batches of 64 and 1024 (the split and the whole mask copy)."""
    import os
    for seed in (1, 2):
        pts = _data("F", seed, True)
        ref = oracle.ransac_run(oracle.FUNDAMENTAL, pts, 2.0, 0.95, seed, sampler=oracle.SAMPLER_PROSAC, sprt=True)
        for batch in (64, 1024):
            runs = []
            for env in (None, "USAC_NO_POOL_TAIL", "USAC_NO_DEFER_POOL", "USAC_DEVICE_INLIERS", "USAC_SPRT_PLAIN_WALK"):
                if env:
                    os.environ[env] = "1"
                try:
                    m = usac.Model(2.0, 7, 0.95, 7, usac.ESTIMATOR.Fundamental, usac.SAMPLER.Prosac)
                    m.ResetRandomGenerator(False)
                    m.setSeed(seed)
                    m.setSprt(True)
                    m.batch = batch
                    r = usac.Ransac(m, pts)
                    r.run()
                finally:
                    if env:
                        os.environ.pop(env, None)
                o = r.getRansacOutput()
                runs.append((o.getNumberOfMainIterations(), r.records, o.raw["sprt_rejected"],
                             o.raw["prosac_term_len"], _bits(o.getModel()).tolist(), o.getInliers().tolist()))
            assert all(x == runs[0] for x in runs[1:]), (seed, batch)
            assert runs[0][0] == ref["iters"] and runs[0][3] == ref["prosac_term_len"], (seed, batch)
            assert runs[0][5] == list(ref["inlier_idx"]), (seed, batch)
