"""Statistical pins of the oracle against the reference's own published results.

The reference cannot be built here (OpenCV + contrib, Eigen3, nanoflann: SURVEY §8c), so
nothing compares a single run bit for bit with it.  What it does publish are multi-run
statistics (test/tests.h getStatisticalResults): per scene the average / standard deviation of
the final inlier count, the main-loop iterations and the average error of the final model on
the ground-truth inliers (quality.hpp:134-146).  These tests run the oracle the same number of
seeded times on the same scenes (tests/golden/*_scenes.npz, the reference's data files) and
require every pinned average to agree within four combined standard errors,

    |mean_ours - mean_ref| <= 4 sqrt(sd_ref^2 / n_ref + sd_ours^2 / n_ours) + floor,

the floor (half a percent of the mean, at least one inlier; 0.002 px for errors) covering
the reference side's unreproducible randomness (random_device / time seeds) and values the
CSV rounds.  The device path equals the oracle bit for bit (tests/test_gpu_*.py), so these pins
hold for it too; tests/test_gpu_reference_statistics.py re-runs a subset through the library.

What is pinned, and what is not (DESIGN.md §3 lists the same):
  * homography, Uniform + graph-cut LO (+ SPRT), 12 real scenes: final inliers and GT error --
    the thin-SVD 4-point DLT (Q1), the homography residual, GC-LO, SPRT and the NormalizedDLT
    polish end to end.  Not pinned: iterations (e.g. adam 16 published vs 3 here -- the
    termination bound of 133/153 inliers at p = 0.95 is 3; the CSV predates the current loop).
  * fundamental, Uniform + graph-cut LO (+ SPRT), kusvod2 scenes: final inliers -- the 7-point
    solver, Sampson error, GC-LO -- with the rank-2 8-point polish of the revision that wrote
    the CSVs (oracle.set_f8_rank2; the current eight_points.cpp:58-68 comments it out).
  * homography, EVD (results/EVD, 15 wide-baseline scenes): graph-cut LO with KNN or grid
    neighbours, Uniform and PROSAC, with and without SPRT -- final inliers (PROSAC: 14 of 15
    scenes, EVD_SKIP).
  * line2d (results/line2d): Uniform (inliers + iterations), LO-RANSAC and NAPSAC (inliers),
    SPRT (inliers + iterations, below), graph-cut LO (inliers).  Not pinned: PROSAC and the
    iteration counts with LO / graph cut (LINE2D_NOT_PINNED).

Time-seeded runs (the "harness lens").  Every Ransac the reference's harness constructs calls
srand(time(NULL)) (model.hpp:45 reset_random_generator defaults to true; uniform_sampler.hpp:22-26,
sprt.hpp:90), and getStatisticalResults builds one Ransac per run back to back (tests.h:144-147).
All runs that start within the same wall-clock second therefore draw the same glibc stream and
return the same result: a CSV row of R runs at an average of tau seconds each holds only about
R*tau + 1 distinct runs.  The CSVs show it -- kusvod2 `shout` (100 runs at 6.9 ms) publishes
78.0 +- 0.0 inliers and 137 +- 0 iterations, identical runs.  Where that matters (fast runs, so
one to three distinct runs per row) the pins below simulate the harness: runs start at
phase + i*tau (phase uniform in [0, 1) s, tau = the row's "Avg time"), runs in the same second
share one oracle run drawn from a pool of seeded oracle runs, and the published average must lie
within the central 99 % of the simulated 50- / 100-run averages (lens_p >= 0.005).
"""
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
STATS = json.load(open(os.path.join(HERE, "golden", "reference_stats.json")))["files"]

INL, SD_INL = "Avg num inl/gt", "Std dev num inl"
ITS, SD_ITS = "Avg num iters", "Std dev num iters"
ERR, SD_ERR = "Avg err", "Std dev err"

# Scenes whose published averages the oracle does not reproduce, with the measured gap (oracle
# mean vs published mean over the seeds used here).  They stay in the report, not in the pins.
EXCEPTIONS = {
    ("homography/uniform_gc_Grid_c_sz_50.csv", "graf", INL):
        "bimodal: some runs converge to a 210-inlier plane (225.6 +- 7.2 vs 233.0 +- 2.8)",
    ("homography/uniform_gc_Grid_c_sz_50.csv", "graf", ERR): "follows the bimodal inlier count",
    ("homography/uniform_gc_Grid_c_sz_50.csv", "BruggeSquare", ERR):
        "29 GT inliers, heavy-tailed error (2.6 +- 1.1 vs 1.8 +- 0.5)",
    ("homography/uniform_gc_sprt_Grid_c_sz_50.csv", "graf", INL): "bimodal as without SPRT",
    ("homography/uniform_gc_sprt_Grid_c_sz_50.csv", "graf", ERR): "bimodal as without SPRT",
    ("homography/uniform_gc_sprt_Grid_c_sz_50.csv", "BruggeSquare", ERR): "heavy-tailed as without SPRT",
}


def agree(ours, ref_mean, ref_sd, ref_n, floor):
    ours = np.asarray(ours, dtype=np.float64)
    se = np.sqrt(ref_sd ** 2 / ref_n + ours.std(ddof=1) ** 2 / len(ours)) if len(ours) > 1 else ref_sd
    return abs(ours.mean() - ref_mean) <= 4.0 * se + floor, ours.mean()


def check(rel, results, keys, floors):
    """results: scene -> {key: list of per-run values}; returns the pinned (scene, key) pairs."""
    table = STATS[rel]
    n_ref = table["settings"]["Runs for each image"]
    pinned, failures = [], []
    for scene, vals in results.items():
        row = table["scenes"][scene]
        for key, sdk in keys:
            if (rel, scene, key) in EXCEPTIONS:
                continue
            ok, m = agree(vals[key], row[key], row[sdk], n_ref, floors[key](row[key]))
            (pinned if ok else failures).append((scene, key, round(m, 4), row[key], row[sdk]))
    assert not failures, (rel, failures)
    return pinned


def lens_p(vals, row, key, runs, sims=4000, seed=0):
    """Harness lens (module docstring): two-sided tail probability of the published average
    `row[key]` among simulated time-seeded averages of `runs` runs built from `vals` (one
    value per independent seeded oracle run)."""
    rng = np.random.default_rng(seed)
    vals = np.asarray(vals, dtype=np.float64)
    tau = row["Avg time (mcs)"] * 1e-6
    means = np.empty(sims)
    for i in range(sims):
        grp = np.floor(rng.random() + tau * np.arange(runs)).astype(np.int64)
        grp -= grp[0]
        pick = rng.choice(len(vals), grp[-1] + 1, replace=len(vals) <= grp[-1])
        means[i] = vals[pick[grp]].mean()
    x = row[key]
    return min(float((means <= x + 1e-9).mean()), float((means >= x - 1e-9).mean()))


def lens_check(rel, results, keys, min_p=0.005):
    """results: scene -> {key: per-run values}; returns {(scene, key): p}, asserting p >= min_p."""
    table = STATS[rel]
    runs = int(table["settings"]["Runs for each image"])
    ps = {(scene, key): lens_p(vals[key], table["scenes"][scene], key, runs)
          for scene, vals in results.items() for key in keys}
    bad = {k: v for k, v in ps.items() if v < min_p}
    assert not bad, (rel, bad)
    return ps


def inl_floor(mean):
    return max(1.0, 0.005 * mean)


def gt_inliers(oracle, est, pts, model, thr):
    """GetImage.h:250-277: GT inliers of the GT model or of its inverse, whichever has more."""
    e1 = est.errors(model)
    e2 = est.errors(oracle.inv3x3(model)[0])
    g1, g2 = np.nonzero(e1 < thr)[0], np.nonzero(e2 < thr)[0]
    return g2 if len(g2) > len(g1) else g1


def gt_error(est, model, gt):
    """Quality::getErrorGT_inl (quality.hpp:134-146): sequential fp32 mean over the GT inliers."""
    e = est.errors(model)[gt]
    acc = np.float32(0)
    for v in e:
        acc = np.float32(acc + v)
    return float(acc / np.float32(len(gt)))


@pytest.mark.parametrize("rel", ["homography/uniform_gc_Grid_c_sz_50.csv",
                                 "homography/uniform_gc_sprt_Grid_c_sz_50.csv"])
def test_homography_gc_statistics(oracle, homography_scenes, rel):
    runs = 50
    sprt = "sprt" in rel
    z = homography_scenes
    results = {}
    for scene, (pts, model, _) in z.items():
        est = oracle.Estimator(oracle.HOMOGRAPHY, pts)
        gt = gt_inliers(oracle, est, pts, model, 2.0)
        inl, err = [], []
        for seed in range(1, runs + 1):
            r = oracle.ransac_run(oracle.HOMOGRAPHY, pts, 2.0, 0.95, seed, lo=oracle.LO_GC,
                                  neighbors=oracle.NEIGHBORS_GRID, cell_size=50, sprt=sprt)
            assert r["ret"] == 0
            inl.append(r["inliers"])
            err.append(gt_error(est, r["model"], gt))
        results[scene] = {INL: inl, ERR: err}
    pinned = check(rel, results, [(INL, SD_INL), (ERR, SD_ERR)],
                   {INL: inl_floor, ERR: lambda m: max(0.002, 0.005 * m)})
    assert len(pinned) >= 21, pinned  # 12 scenes x 2 quantities, 3 documented exceptions


@pytest.mark.parametrize("rel", ["kusvod2/uniform_gc_Grid_c_sz_50.csv",
                                 "kusvod2/uniform_gc_sprt_Grid_c_sz_50.csv"])
def test_fundamental_gc_statistics(oracle, kusvod2_scenes, rel):
    runs = 30
    sprt = "sprt" in rel
    results = {}
    oracle.set_f8_rank2(True)
    try:
        for scene, (pts, _) in kusvod2_scenes.items():
            if scene not in STATS[rel]["scenes"] or scene in KUSVOD2_SKIP or (sprt and scene in KUSVOD2_SPRT_SKIP):
                continue
            inl = []
            for seed in range(1, runs + 1):
                r = oracle.ransac_run(oracle.FUNDAMENTAL, pts, 2.0, 0.95, seed, lo=oracle.LO_GC,
                                      neighbors=oracle.NEIGHBORS_GRID, cell_size=50, sprt=sprt)
                inl.append(r["inliers"] if r["ret"] == 0 else 0)
            results[scene] = {INL: inl}
    finally:
        oracle.set_f8_rank2(False)
    pinned = check(rel, results, [(INL, SD_INL)], {INL: inl_floor})
    assert len(pinned) >= 10, pinned


# kusvod2 scenes the rank-2 oracle does not reproduce (measured, 20 runs: oracle vs published
# average inliers) -- the older revision differs beyond the 8-point polish there.
KUSVOD2_SKIP = {
    "box": "160.4 +- 6.7 vs 153.9 +- 4.2",
    "castle": "153.2 +- 2.8 vs 149.3 +- 4.2",
    "graff": "46 points, 10000 iterations: 10.7 +- 0.7 vs 12.9 +- 1.1",
    "leafs": "73.2 +- 4.4 vs 67.4 +- 1.6",
    "shout": "74.6 +- 5.7 vs 78.0 +- 0.0",
}
KUSVOD2_SPRT_SKIP = {"kampa": "with SPRT 103.7 +- 2.5 vs 99.2 +- 2.0 (pinned without SPRT)"}


@pytest.fixture(scope="module")
def evd_scenes():
    z = np.load(os.path.join(HERE, "golden", "evd_scenes.npz"))
    return {k[:-4]: z[k] for k in z.files}


# EVD (wide-baseline homographies, 83 - 1164 tentatives, 15 - 80 true correspondences): the
# reference's EVD statistics are graph-cut runs with KNN (nanoflann, k = 7) or grid
# neighbours, Uniform or PROSAC (the tentatives file is already in quality order, so the
# sorted points are the points: dataset/GetImage.h:122-136), with and without SPRT; the CSVs
# cap the iterations at 15 000 (the runs that never meet the termination bound report 15000).
# Final inliers are pinned; iterations are not (the CSVs predate the current loop, as the
# homography ones: adam 1467 published vs ~1250 here).
EVD_CASES = [("EVD/uniform_gc_Nanoflann_c_sz_50.csv", "uniform", False, "knn"),
             ("EVD/uniform_gc_sprt_Nanoflann_c_sz_50.csv", "uniform", True, "knn"),
             ("EVD/prosac_gc_Nanoflann_c_sz_50.csv", "prosac", False, "knn"),
             ("EVD/prosac_gc_sprt_Nanoflann_c_sz_50.csv", "prosac", True, "knn"),
             ("EVD/prosac_gc_sprt_Grid_c_sz_50.csv", "prosac", True, "grid")]
# PROSAC scenes the oracle does not reproduce (12 runs, oracle vs published average inliers):
# here PROSAC finds the 40-inlier plane of `grand` / `pkk` in most runs, the published runs
# far less often (large published spread: the reference's PROSAC fails on them in many runs).
# Uniform sampling on the same scenes agrees, so the gap is in the PROSAC schedule (the
# reference seeds it from std::random_device, and which libstdc++ uniform_int_distribution it
# ran is unknown -- DESIGN.md §3).  Reported, not pinned.
EVD_SKIP = {
    ("EVD/prosac_gc_Nanoflann_c_sz_50.csv", "grand"): "41.0 vs 29.6 +- 9.3",
    ("EVD/prosac_gc_sprt_Nanoflann_c_sz_50.csv", "grand"): "36.4 vs 12.9 +- 11.9",
    ("EVD/prosac_gc_sprt_Grid_c_sz_50.csv", "pkk"): "28.5 vs 13.3 +- 13.4",
}


@pytest.mark.parametrize("rel,sampler,sprt,nb", EVD_CASES)
def test_evd_gc_statistics(oracle, evd_scenes, rel, sampler, sprt, nb):
    runs = 12
    results = {}
    for scene, pts in sorted(evd_scenes.items()):
        if scene not in STATS[rel]["scenes"] or (rel, scene) in EVD_SKIP:
            continue
        inl = []
        for seed in range(1, runs + 1):
            r = oracle.ransac_run(oracle.HOMOGRAPHY, pts, 2.0, 0.95, seed, max_iters=15000,
                                  sampler=oracle.SAMPLER_PROSAC if sampler == "prosac" else oracle.SAMPLER_UNIFORM,
                                  sprt=sprt, lo=oracle.LO_GC, cell_size=50, knn=7,
                                  neighbors=oracle.NEIGHBORS_NANOFLANN if nb == "knn" else oracle.NEIGHBORS_GRID)
            inl.append(r["inliers"] if r["ret"] == 0 else 0)
        results[scene] = {INL: inl}
    pinned = check(rel, results, [(INL, SD_INL)], {INL: inl_floor})
    assert len(pinned) >= 12, pinned


def _line2d_runs(oracle, pts, runs, **kw):
    inl, its = [], []
    for seed in range(1, runs + 1):
        r = oracle.ransac_run(oracle.LINE2D, pts, 10.0, 0.99, seed, **kw)
        assert r["ret"] == 0
        inl.append(r["inliers"])
        its.append(r["iters"])
    return {INL: inl, ITS: its}


def test_line2d_lo_statistics(oracle, line2d_scenes):
    """results/line2d/uniform_100.csv: InItLORsc (model.hpp:27-30 defaults).  Inliers pinned;
    the published iteration counts with LO exceed those without (2608 vs 2548 on the first
    scene) -- the revision that wrote the CSV counted differently -- so they are not pinned."""
    rel = "line2d/uniform_100.csv"
    results = {name: _line2d_runs(oracle, pts, 30, lo=oracle.LO_INITLORSC)
               for name, (pts, _, _) in sorted(line2d_scenes.items())}
    pinned = check(rel, results, [(INL, SD_INL)], {INL: inl_floor})
    assert len(pinned) == 8


def test_line2d_napsac_statistics(oracle, line2d_scenes):
    """results/line2d/napsac_000.csv: NAPSAC with nanoflann KNN neighbours (the Ransac ctor
    builds KNN for any neighbour type but Grid, ransac.hpp:60-78; k = 8 as store_results_line2d)."""
    rel = "line2d/napsac_000.csv"
    results = {name: _line2d_runs(oracle, pts, 16, sampler=oracle.SAMPLER_NAPSAC,
                                  neighbors=oracle.NEIGHBORS_NANOFLANN, knn=8)
               for name, (pts, _, _) in sorted(line2d_scenes.items())[:3]}
    pinned = check(rel, results, [(INL, SD_INL)], {INL: inl_floor})
    assert len(pinned) == 3


def test_dlt4_thin_row_matches_numpy_svd(oracle, homography_scenes):
    """Q1 (dlt.cpp:43-48): the 4-point model is row 7 of the thin 8x9 SVD's V^T -- checked against
    LAPACK (numpy) on 2000 random samples of a real scene: median relative difference ~4e-8."""
    pts, _, _ = homography_scenes["Brussels"]
    rng = np.random.default_rng(5)
    est = oracle.Estimator(oracle.HOMOGRAPHY, pts, oracle.DLT_THIN)
    rels = []
    for _ in range(2000):
        s = rng.choice(len(pts), 4, replace=False).astype(np.int32)
        models, nm = est.estimate_batch(s[None, :])
        if nm[0] == 0:
            continue
        A = []
        for i in s:
            x1, y1, x2, y2 = (float(v) for v in pts[i])
            A.append([-x1, -y1, -1, 0, 0, 0, x2 * x1, x2 * y1, x2])
            A.append([0, 0, 0, -x1, -y1, -1, y2 * x1, y2 * y1, y2])
        A = np.array(A, dtype=np.float32).astype(np.float64)
        vt = np.linalg.svd(A, full_matrices=False)[2]
        h = vt[7] / vt[7][8]
        m = models.reshape(-1, 9)[0].astype(np.float64)
        rels.append(np.abs(m - h).max() / np.abs(h).max())
    rels = np.array(rels)
    assert len(rels) > 1900
    assert np.median(rels) < 1e-6, np.median(rels)
    assert np.quantile(rels, 0.99) < 1e-4, np.quantile(rels, 0.99)


@pytest.fixture(scope="module")
def line2d_sprt_pools(oracle, line2d_scenes):
    """100 seeded oracle runs per scene, SPRT on (sprt.hpp semantics as written: shuffled,
    rolling pool) and with the CSV revision's point order (oracle.set_sprt_file_order)."""
    pools = {}
    for file_order in (False, True):
        oracle.set_sprt_file_order(file_order)
        try:
            pools[file_order] = {name: _line2d_runs(oracle, pts, 100, sprt=True)
                                 for name, (pts, _, _) in sorted(line2d_scenes.items())}
        finally:
            oracle.set_sprt_file_order(False)
    return pools


def test_line2d_sprt_statistics(line2d_sprt_pools):
    """results/line2d/uniform_001.csv (Uniform + SPRT, 50 runs of 14-40 ms: 2-3 distinct runs
    per row under the harness's time seeding).  With the points tested in file order from
    point 0 -- the SPRT of the revision that wrote this CSV (oracle.set_sprt_file_order) --
    all 8 scenes' average inliers and iterations are pinned under the harness lens: the
    published SPRT runs are longer and worse than without SPRT (2628 vs 2548 iterations,
    411.6 +- 45 vs 438.2 inliers on the first scene) because the line2d files hold their
    inliers last, so a true line is often rejected on the outlier prefix."""
    ps = lens_check("line2d/uniform_001.csv", line2d_sprt_pools[True], [INL, ITS])
    assert len(ps) == 16


def test_line2d_sprt_statistics_current_pool(line2d_sprt_pools):
    """The same CSV against sprt.hpp as written (shuffled pool, rolling index: the semantics
    the product and its bit-exact parity tests follow).  The four I=200 scenes agree under
    the harness lens; the four I=500 scenes cannot: with a shuffled pool the true line
    (6.7-7.1 % inliers) is almost never rejected, so runs end at ~700-725 inliers after
    ~700 iterations, while the CSV's rows sit at 473-702 +- 83-168 inliers and 1313-2734
    iterations -- outside the central 99 % of the simulated 50-run averages (the file-order
    revision above reproduces them).  Asserted both ways so a change on either side shows."""
    rel = "line2d/uniform_001.csv"
    pools = line2d_sprt_pools[False]
    i200 = {k: v for k, v in pools.items() if "I=200" in k}
    i500 = {k: v for k, v in pools.items() if "I=500" in k}
    assert len(lens_check(rel, i200, [INL, ITS])) == 8
    runs = int(STATS[rel]["settings"]["Runs for each image"])
    rejected = [scene for scene, vals in i500.items()
                if min(lens_p(vals[k], STATS[rel]["scenes"][scene], k, runs) for k in (INL, ITS)) < 0.005]
    assert len(rejected) >= 2, rejected


# line2d CSVs (results/line2d) with numbers the oracle does not reproduce, and why.
LINE2D_NOT_PINNED = {
    "prosac_000.csv iterations": "seed-insensitive in the CSV (5, 1.04, 4, 1.04, 9, 1.04, 7.02, 1.02 "
                                 "per scene, std 0-0.28) but 2-9 here with the densitySort order "
                                 "(utils.cpp:8-32 restated with the exact KNN, k = 13): the PROSAC "
                                 "termination of that revision stops after one sample on the I=500 "
                                 "scenes, the current prosac_termination_criteria.hpp does not",
    "uniform_010.csv iterations": "graph-cut runs 3-9 % shorter here (2418 vs 2507 on the first scene) "
                                  "-- a graph-cut revision difference; inliers are pinned",
    "uniform_010.csv w=1200_h=1000_I=200 inliers": "468.0 +- 3.0 vs 457.2 +- 7.2",
    "uniform_100.csv iterations": "LO runs longer than no-LO in the CSV (2608 vs 2548): that revision "
                                  "counted differently",
}


def test_line2d_gc_statistics(oracle, line2d_scenes):
    """results/line2d/uniform_010.csv: Uniform + graph-cut LO (KNN neighbours, k = 8 as the
    line2d harness; Grid is invalid for 2-D points, Q17).  Average inliers pinned by the plain
    rule (four combined standard errors + floor; ~230 ms per published run, so ~12 distinct
    runs per row), one scene excepted (LINE2D_NOT_PINNED)."""
    rel = "line2d/uniform_010.csv"
    results = {}
    for name, (pts, _, _) in sorted(line2d_scenes.items()):
        if "uniform_010.csv %s inliers" % name.replace("_n=3.000000", "").replace("_N=10200", "") in LINE2D_NOT_PINNED:
            continue
        results[name] = _line2d_runs(oracle, pts, 5, lo=oracle.LO_GC, neighbors=oracle.NEIGHBORS_NANOFLANN, knn=8)
    assert len(results) == 7
    assert len(check(rel, results, [(INL, SD_INL)], {INL: inl_floor})) == 7


# kusvod2 scenes excluded from the plain pins above, re-examined under the harness lens: 100
# runs of 3-8 ms are one or two distinct runs per row, so the published average is one or two
# draws of the run distribution (box / castle / leafs / shout / kampa).  Still not pinned:
# graff (10 000 iterations per run, ~10-14 distinct runs; 10.7 vs 12.9 inliers) and castle
# with SPRT (147.75 published, the oracle's runs give 150-156).
KUSVOD2_LENS = [("kusvod2/uniform_gc_Grid_c_sz_50.csv", ["box", "castle", "leafs", "shout"]),
                ("kusvod2/uniform_gc_sprt_Grid_c_sz_50.csv", ["box", "leafs", "shout", "kampa"])]


@pytest.mark.parametrize("rel,scenes", KUSVOD2_LENS)
def test_fundamental_gc_statistics_lens(oracle, kusvod2_scenes, rel, scenes):
    sprt = "sprt" in rel
    results = {}
    oracle.set_f8_rank2(True)
    try:
        for scene in scenes:
            pts, _ = kusvod2_scenes[scene]
            inl = []
            for seed in range(1, 31):
                r = oracle.ransac_run(oracle.FUNDAMENTAL, pts, 2.0, 0.95, seed, lo=oracle.LO_GC,
                                      neighbors=oracle.NEIGHBORS_GRID, cell_size=50, sprt=sprt)
                inl.append(r["inliers"] if r["ret"] == 0 else 0)
            results[scene] = {INL: inl}
    finally:
        oracle.set_f8_rank2(False)
    assert len(lens_check(rel, results, [INL])) == len(scenes)
