"""PROSAC sampler / termination and SPRT -- no GPU.

Pins:
  * std::mt19937: the C++ standard's known answer (10000th output of the default seed 5489
    is 4123659995) and numpy's legacy RandomState(seed) raw 32-bit stream;
  * uniform_int_distribution<int>: libstdc++'s classic downscaling, restated independently
    here in Python from the raw stream;
  * SPRT: the decision thresholds A0 the reference's defaults give (SURVEY §8 a15:
    H 18.1658, F 10.9713, E 10.3862, line 1.3933);
  * the PROSAC growth function's "+1 per hypothesis" regime.
The reference seeds PROSAC's mt19937 from std::random_device (not reproducible); this build
seeds it with the run seed -- the stream semantics, not the seed, are what is pinned.
The host library (libransac_amd.so) must reproduce the oracle's streams exactly.
"""
import numpy as np
import pytest

from ransac_amd import synthetic


def test_mt19937_known_answers(oracle):
    assert int(oracle.mt19937_stream(5489, 10000)[-1]) == 4123659995
    for seed in (1, 5489, 123456789):
        ref = np.random.RandomState(seed).randint(0, 2 ** 32, size=64, dtype=np.uint64)
        np.testing.assert_array_equal(oracle.mt19937_stream(seed, 64), ref)


@pytest.mark.parametrize("hi", [0, 1, 5, 6, 1000, 9998, 2 ** 31 - 1])
def test_uniform_int_downscaling(oracle, hi):
    raw = oracle.mt19937_stream(77, 4000).astype(np.uint64)
    buckets = hi + 1
    scale = 0xFFFFFFFF // buckets
    limit = buckets * scale
    ref = [int(r // scale) for r in raw if r < limit]
    got = oracle.mt19937_uniform(77, hi, len(ref))
    np.testing.assert_array_equal(got, np.array(ref[: len(got)]))
    assert got.min() >= 0 and got.max() <= hi


def test_sprt_thresholds_match_reference_defaults(oracle, usac):
    want = {oracle.HOMOGRAPHY: 18.1658, oracle.FUNDAMENTAL: 10.9713, oracle.ESSENTIAL: 10.3862,
            oracle.LINE2D: 1.3933}
    for kind, A in want.items():
        pool, A0 = oracle.sprt_pool(1, kind, 500, 4)
        assert A0 == pytest.approx(A, abs=5e-5)
        hpool, hA0 = usac.sprt_pool(1, kind, 500, 4)
        assert hA0 == A0
        np.testing.assert_array_equal(hpool, pool)
        assert sorted(pool.tolist()) == list(range(500))


def test_sprt_pool_consumes_glibc_stream_before_sampler(oracle):
    # the shuffle is the reference's pool swap over srandom(seed)'s first n draws
    n = 50
    r = oracle.glibc_stream(9, n)
    pool = list(range(n))
    mx = n
    for i in range(n):
        k = int(r[i]) % mx
        mx -= 1
        pool[k], pool[mx] = pool[mx], pool[k]
    np.testing.assert_array_equal(oracle.sprt_pool(9, oracle.HOMOGRAPHY, n, 4)[0], np.array(pool))


def test_prosac_growth_and_samples(oracle, usac):
    n, m = 10000, 7
    s, growth, largest = oracle.prosac_samples(3, n, m, 3000)
    # T_n is tiny for N >> m, so g(n) grows by one per hypothesis
    assert growth[m - 1] == 1 and growth[m] == 2 and growth[m + 100] == 102
    assert (np.diff(growth[m:2000]) == 1).all()
    # the last point of a PROSAC sample is the newest point of the progressive pool
    for t in range(1, 3000):
        pool = s[t, -1] + 1
        assert s[t, :-1].max() <= pool - 2
        assert len(set(s[t].tolist())) == m
    assert largest == s[:, -1].max() + 1
    np.testing.assert_array_equal(usac.prosac_samples(3, n, m, 3000), s)
    # termination_length below the pool size: uniform draws from the CLOSED range <0; t> (Q15)
    s2, _, _ = oracle.prosac_samples(5, 200, 4, 500, term_len=30)
    np.testing.assert_array_equal(usac.prosac_samples(5, 200, 4, 500, termination_length=30), s2)
    assert s2[300:].max() <= 30


@pytest.mark.parametrize("sprt", [False, True])
def test_oracle_prosac_fundamental_run(oracle, sprt):
    pts, F, inl = synthetic.fundamental_points(n=3000, inlier_ratio=0.3, seed=2, prosac_order=True)
    r = oracle.ransac_run(oracle.FUNDAMENTAL, pts, 2.0, 0.95, 1, sampler=oracle.SAMPLER_PROSAC, sprt=sprt)
    assert r["ret"] == 0
    found = set(r["inlier_idx"].tolist())
    truth = set(np.where(inl)[0].tolist())
    assert len(found & truth) >= 0.75 * len(truth)  # PROSAC stops after a handful of samples
    assert r["prosac_term_len"] <= 3000


def test_oracle_sprt_rejects_and_counts(oracle):
    pts, H, inl = synthetic.homography_points(n=2000, inlier_ratio=0.3, seed=3)
    a = oracle.ransac_run(oracle.HOMOGRAPHY, pts, 2.0, 0.95, 1, sprt=False)
    b = oracle.ransac_run(oracle.HOMOGRAPHY, pts, 2.0, 0.95, 1, sprt=True)
    assert b["ret"] == 0 and b["sprt_rejected"] > 0 and b["sprt_histories"] >= 1
    # SPRT scores are counts: every record's score equals its inlier count
    assert all(float(s) == float(c) for _, c, s in b["records"])
    assert abs(b["inliers"] - a["inliers"]) <= 0.05 * a["inliers"]
