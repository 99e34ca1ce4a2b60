"""CPU oracle, essential path, no GPU.

The reference's 5-point solver goes through OpenCV SVD/determinant/inv and the rpoly
Jenkins-Traub root finder (five_points.cpp:13-274).  Two of its steps are pinned against the
reference's own code compiled where it lies (oracle/_ref): the polynomial matrix M(z)
(mblock.hpp) and the root step (rpoly.cpp's rpoly_ak1, restated operation for operation: the
same zeros in the same order, which decides the selected candidate), plus a committed fixture of
rpoly's outputs for boxes without the reference.  The OpenCV steps (null basis, determinant
interpolation, triangulation SVD) are not reproducible here, and the oracle's restatement of
them is pinned by identities: on exact two-view data
the generating E is among the solver's candidates and passes its cheirality test, the
returned E satisfies the essential-matrix constraints, and the residual equals the textbook
point-to-epipolar-line distance.
"""
import numpy as np
import pytest

from ransac_amd import synthetic


def _dist(m, E):
    a = m.reshape(-1) / np.linalg.norm(m)
    b = E.reshape(-1) / np.linalg.norm(E)
    return min(np.linalg.norm(a - b), np.linalg.norm(a + b))


def test_real_roots_match_numpy(oracle):
    """The root step (usac_oracle.c jt_rpoly, the reference's Jenkins-Traub rpoly_ak1 restated)
    finds every real zero of well-separated polynomials and reports no complex one."""
    rng = np.random.default_rng(0)
    for _ in range(200):
        roots = np.sort(rng.uniform(-4, 4, size=rng.integers(1, 11)))
        if len(roots) > 1 and np.min(np.diff(roots)) < 1e-2:
            continue
        poly = np.poly(roots)[::-1] * rng.uniform(0.5, 2)
        got = np.sort(oracle.real_roots(poly))
        np.testing.assert_allclose(got, roots, rtol=0, atol=1e-7)
    # complex pairs are not reported
    got = np.sort(oracle.real_roots(np.poly([1.0, -2.0, 1 + 1j, 1 - 1j]).real[::-1]))
    np.testing.assert_allclose(got, [-2.0, 1.0], atol=1e-9)


def test_real_roots_wide_range(oracle):
    """Roots spread over six decades, both signs: none lost (rpoly's scaling and its
    lower-bound shifts), every one to ~1e-9."""
    rng = np.random.default_rng(1)
    worst, tested = 0.0, 0
    for _ in range(800):
        k = int(rng.integers(2, 11))
        roots = np.sort(rng.choice([-1.0, 1.0], k) * 10 ** rng.uniform(-3, 3, k))
        if np.min(np.diff(roots) / np.maximum(1.0, np.abs(roots[1:]))) < 1e-3:
            continue
        got = np.sort(oracle.real_roots(np.poly(roots)[::-1]))
        assert len(got) == len(roots)
        worst = max(worst, float(np.max(np.abs(got - roots) / np.maximum(np.abs(roots), 1e-3))))
        tested += 1
    assert tested > 600 and worst < 1e-8, worst


def test_jt_log_exp_correctly_rounded(oracle):
    """The restatement's portable log / exp (the two libm calls in rpoly.cpp:82,98) are the
    correctly rounded values (checked with 60-digit decimal arithmetic); the device repeats them
    bit for bit.  glibc's own differ on a small fraction (its exp is not correctly rounded)."""
    import math
    from decimal import Decimal, getcontext

    getcontext().prec = 60

    def cr(v):
        f = float(v)
        c = [math.nextafter(f, -math.inf), f, math.nextafter(f, math.inf)]
        return min(c, key=lambda x: abs(Decimal(x) - v))

    rng = np.random.default_rng(4)
    for x in np.ldexp(rng.uniform(0.5, 1.0, 400), rng.integers(-1000, 1000, 400)):
        assert oracle.jt_log(x) == cr(Decimal(float(x)).ln()), x
    for y in np.r_[rng.uniform(-700, 700, 300), rng.uniform(-5, 5, 300)]:
        assert oracle.jt_exp(y) == cr(Decimal(float(y)).exp()), y
    assert oracle.jt_log(1.0) == 0.0 and oracle.jt_exp(0.0) == 1.0


def test_rpoly_restatement_matches_reference_random(oracle):
    """The restatement against the reference's rpoly_ak1 compiled where it lies (oracle/_ref):
    20 000 random polynomials of degree 3-10 over eight decades of coefficient size give the
    same zeros, bit for bit and in the same order, on all but a handful (measured 3 in 200 000):
    those are the arguments where glibc's exp / log misround and the root bound's last bits
    differ; there the degree and the order agree and the zeros agree to 1e-9."""
    if not oracle.rpoly_ref_available():
        pytest.skip("oracle/_ref/librpoly_ref.so not built (the reference is absent)")
    rng = np.random.default_rng(3)
    exact = near = 0
    for t in range(20000):
        n = int(rng.integers(3, 11))
        a = (rng.uniform(size=n + 1) - 0.5) * 10.0 ** ((rng.uniform(size=n + 1) - 0.5) * 8)
        zr, zi = oracle.rpoly_zeros(a)
        rr, ri = oracle.rpoly_ref_zeros(a)
        assert len(zr) == len(rr), (a, zr, rr)
        if np.array_equal(zr, rr) and np.array_equal(zi, ri):
            exact += 1
            continue
        near += 1
        z, r = zr + 1j * zi, rr + 1j * ri
        assert np.all(np.abs(z - r) <= 1e-9 * np.maximum(np.abs(r), 1.0)), (a, z, r)
    assert near <= 5, near


def test_essential_error_closed_form(oracle):
    pts, E, inl = synthetic.fundamental_points(n=500, inlier_ratio=0.5, seed=2, normalized=True)
    est = oracle.Estimator(oracle.ESSENTIAL, pts)
    e = est.errors(E).astype(np.float64)
    Ed = E.astype(np.float64).reshape(3, 3)
    x1 = np.c_[pts[:, :2], np.ones(len(pts))].astype(np.float64)
    x2 = np.c_[pts[:, 2:], np.ones(len(pts))].astype(np.float64)
    l = x2 @ Ed      # epipolar lines in image 1
    t = x1 @ Ed.T    # epipolar lines in image 2
    d1 = np.abs(np.einsum("ij,ij->i", l, x1)) / np.hypot(l[:, 0], l[:, 1])
    d2 = np.abs(np.einsum("ij,ij->i", t, x2)) / np.hypot(t[:, 0], t[:, 1])
    np.testing.assert_allclose(e, (d1 + d2) / 2, rtol=1e-3, atol=1e-6)


def test_five_point_candidates_contain_exact_E(oracle):
    pts, E, inl = synthetic.fundamental_points(n=2000, inlier_ratio=0.3, seed=1, noise=0.0, normalized=True)
    est = oracle.Estimator(oracle.ESSENTIAL, pts)
    idx = np.where(inl)[0]
    rng = np.random.default_rng(0)
    hit = returned = 0
    for _ in range(100):
        s = rng.choice(idx, 5, replace=False).astype(np.int32)
        cand, ok = est.e5_candidates(s)
        assert len(cand) <= 10
        d = [_dist(m, E) for m in cand]
        if d and min(d) < 1e-4 and ok[int(np.argmin(d))]:
            hit += 1
        ms = est.estimate(s)
        if len(ms):
            returned += 1
            M = ms[0].reshape(3, 3).astype(np.float64)
            sv = np.linalg.svd(M, compute_uv=False)
            # 1e-3: the selected zero may be a late one of rpoly's deflation order, whose value
            # (and E) carries the deflation's larger error -- as in the reference
            assert sv[2] <= 1e-3 * sv[0] and abs(sv[0] - sv[1]) <= 1e-3 * sv[0]
            # the returned E is a passing candidate -- the only one when one passes (the order among
            # several: test_e5_selection_follows_reference_rpoly_order)
            hits = [k for k in range(len(cand)) if ok[k] and np.array_equal(ms[0], cand[k])]
            assert hits and (ok.sum() > 1 or hits == [int(np.argmax(ok))])
    assert hit >= 95 and returned >= 95


def test_ransac_essential_finds_inliers(oracle):
    pts, E, inl = synthetic.fundamental_points(n=2000, inlier_ratio=0.5, seed=3, normalized=True,
                                               prosac_order=False)
    r = oracle.ransac_run(oracle.ESSENTIAL, pts, 0.002, 0.95, 1)
    assert r["ret"] == 0
    found = set(r["inlier_idx"].tolist())
    truth = set(np.where(inl)[0].tolist())
    assert len(found & truth) >= 0.9 * len(truth)


def test_e5_matrix_pinned_against_reference_mblock(oracle):
    """the oracle's M(z) -- the ten cubic constraints of E = x N0 + y N1 + z N2 + N3
    over the monomials [x^3, y^3, x^2 y, x y^2, x^2, y^2, x y, x, y, 1] (usac_oracle.c e5_matrix; the
    device's usac_device_e5.hpp follows it bit for bit) -- against the reference's own generated
    matrix, usac/estimator/essential/mblock.hpp compiled where it lies into oracle/_ref by
    oracle/Makefile (oracle/mblock_ref.cpp; the reference's Polynomial::Eval at z).  Every entry
    within 1e-12 of its row's largest magnitude: same rows, same columns, same polynomials."""
    if not oracle.mblock_ref_available():
        pytest.skip("oracle/_ref/libmblock_ref.so not built (the reference is absent)")
    rng = np.random.default_rng(5)
    worst = 0.0
    for t in range(300):
        N = rng.standard_normal((4, 9))
        if t % 3 == 0:  # null bases of real samples' scale: orthonormal rows
            N = np.linalg.qr(N.T)[0].T
        for z in (-5.0, -4.0, -1.0, 0.0, 0.25, 3.0, 5.0, float(rng.uniform(-20, 20))):
            a = oracle.e5_matrix(N, z)
            b = oracle.mblock_ref_eval(N, z)
            scale = np.abs(b).max(axis=1, keepdims=True)
            assert (scale > 0).all()
            worst = max(worst, float((np.abs(a - b) / scale).max()))
    assert worst <= 1e-12, worst


def _residual(a, x):
    """|p(x)| / sum |a_i| |x|^i evaluated exactly (rationals): the backward error of a root."""
    from fractions import Fraction

    X, v, s = Fraction(float(x)), Fraction(0), Fraction(0)
    for i, c in enumerate(a):
        t = Fraction(float(c)) * X ** i
        v += t
        s += abs(t)
    return float(abs(v) / s) if s else 0.0


def test_e5_roots_pinned_against_reference_rpoly(oracle):
    """the 5-point solver's root step follows the reference's rpoly_ak1
    (usac/estimator/essential/rpoly.cpp:7-750, restated in usac_oracle.c jt_rpoly; the reference
    compiled where it lies into oracle/_ref by oracle/Makefile).  On the oracle's degree-10
    polynomials of 10 000 cfg4 samples the restatement reports the same zeros in the same order,
    bit for bit, on >= 99.9 % of the samples (the rest: the root bound's last bits, where glibc's
    exp / log misround -- same order, zeros within 1e-9)."""
    if not oracle.rpoly_ref_available():
        pytest.skip("oracle/_ref/librpoly_ref.so not built (the reference is absent)")
    pts, _, _ = synthetic.fundamental_points(n=50000, inlier_ratio=0.3, seed=1, normalized=True)
    est = oracle.Estimator(oracle.ESSENTIAL, pts)
    samples = oracle.uniform_samples(11, len(pts), 5, 10000)
    n_exact = n_near = 0
    for s in samples:
        a = oracle.e5_poly(est, s)
        zr, zi = oracle.rpoly_zeros(a)
        rr, ri = oracle.rpoly_ref_zeros(a)
        assert len(zr) == len(rr), (s, zr, rr)
        if np.array_equal(zr, rr) and np.array_equal(zi, ri):
            n_exact += 1
        else:
            n_near += 1
            z, r = zr + 1j * zi, rr + 1j * ri
            assert np.all(np.abs(z - r) <= 1e-9 * np.maximum(np.abs(r), 1.0)), (s, z, r)
    print("rpoly pin: %d / %d samples bit-exact, %d within 1e-9" % (n_exact, len(samples), n_near))
    assert n_near <= 0.001 * len(samples)


def test_e5_selection_follows_reference_rpoly_order(oracle):
    """five_points.cpp:239-273 returns the first candidate in rpoly's order that passes cheirality.
    The solver's candidates are the real roots ascending (asc_real_roots); when several pass it walks
    the restatement's zeros in rpoly's order and takes the first whose nearest candidate passes.
    Against the reference's own rpoly (oracle/_ref): on 10 000 cfg4 samples the selected model is the
    candidate the reference's order selects on every sample with several passing candidates (VERDICT
    r5: round 5 scanned ascending and differed on 14.7 % of the samples with a passing candidate)."""
    if not oracle.rpoly_ref_available():
        pytest.skip("oracle/_ref/librpoly_ref.so not built (the reference is absent)")
    pts, _, _ = synthetic.fundamental_points(n=50000, inlier_ratio=0.3, seed=1, normalized=True)
    est = oracle.Estimator(oracle.ESSENTIAL, pts)
    n_multi = n_diff = n_one = 0
    for s in oracle.uniform_samples(11, len(pts), 5, 10000):
        cand, ok = est.e5_candidates(s)
        if ok.sum() == 0:
            continue
        ms = est.estimate(s)
        assert len(ms) == 1
        mine = [k for k in range(len(cand)) if ok[k] and np.array_equal(ms[0], cand[k])]
        assert mine
        a = oracle.e5_poly(est, s)
        roots = oracle.asc_roots(a)
        if len(roots) != len(cand):  # a candidate without a null vector (not reported): skip the mapping
            continue
        if ok.sum() == 1:
            n_one += 1
            continue
        n_multi += 1
        rr, ri = oracle.rpoly_ref_zeros(a)
        ref_pick = None
        for z in rr[ri == 0]:  # the reference: its zeros in order, the first whose candidate passes
            k = int(np.argmin(np.abs(roots - z)))
            if ok[k]:
                ref_pick = k
                break
        n_diff += ref_pick != mine[0]
    print("selection: %d samples with several passing candidates, %d differ from the reference's order "
          "(%d with one)" % (n_multi, n_diff, n_one))
    assert n_multi > 500 and n_diff == 0


def test_rpoly_restatement_matches_golden(oracle):
    """The same pin without the reference present: tests/golden/rpoly_ref.npz holds the
    reference's rpoly_ak1 zeros (its order) for 400 of the solver's degree-10 polynomials and 400
    random ones (tools/gen_rpoly_golden.py, run where oracle/_ref is built).  The restatement
    reports the same number of zeros and the same zeros, bit for bit, on all but the rare
    polynomials whose root bound meets a misrounded glibc exp / log (<= 2 here), and within 1e-9
    in the same order on those."""
    import os

    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rpoly_ref.npz"))
    near = 0
    for a, d, zr_ref, zi_ref, k in zip(g["coeffs"], g["degree"], g["zr"], g["zi"], g["nzeros"]):
        zr, zi = oracle.rpoly_zeros(a[: d + 1])
        assert len(zr) == k
        if np.array_equal(zr, zr_ref[:k]) and np.array_equal(zi, zi_ref[:k]):
            continue
        near += 1
        z, r = zr + 1j * zi, zr_ref[:k] + 1j * zi_ref[:k]
        assert np.all(np.abs(z - r) <= 1e-9 * np.maximum(np.abs(r), 1.0))
    assert near <= 2, near
