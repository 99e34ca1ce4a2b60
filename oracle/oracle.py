"""ctypes binding of the CPU ORACLE (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the checker or the timed CPU baseline -- never by the product
(ransac_amd/).  See oracle/usac_oracle.h for what it restates and how it is pinned.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")

LINE2D, HOMOGRAPHY, FUNDAMENTAL, ESSENTIAL = 1, 2, 3, 4
DLT_THIN, DLT_NULLSPACE = 0, 1

_f32p = ctypes.POINTER(ctypes.c_float)
_i32p = ctypes.POINTER(ctypes.c_int)
_u32p = ctypes.POINTER(ctypes.c_uint)


class OrcResult(ctypes.Structure):
    _fields_ = [
        ("model", ctypes.c_float * 9),
        ("inliers", ctypes.c_int),
        ("iters", ctypes.c_uint),
        ("n_records", ctypes.c_int),
        ("polish_passes", ctypes.c_int),
        ("minimal_model", ctypes.c_float * 9),
        ("minimal_inliers", ctypes.c_int),
        ("sprt_rejected", ctypes.c_int),
        ("sprt_histories", ctypes.c_int),
        ("prosac_term_len", ctypes.c_uint),
        ("lo_inner_iters", ctypes.c_uint),
        ("lo_iterative_iters", ctypes.c_uint),
    ]


SAMPLER_UNIFORM, SAMPLER_NAPSAC, SAMPLER_PROSAC = 1, 3, 4  # usac/model.hpp:11


LO_NONE, LO_INITLORSC, LO_INITFLORSC, LO_GC = 0, 1, 2, 3  # usac/model.hpp:13
NEIGHBORS_NULL, NEIGHBORS_NANOFLANN, NEIGHBORS_GRID = 0, 1, 2  # usac/model.hpp:12 (NeighborsSearch)


class OrcConfig(ctypes.Structure):
    _fields_ = [("threshold", ctypes.c_float), ("desired_prob", ctypes.c_float), ("max_iterations", ctypes.c_uint),
                ("seed", ctypes.c_uint), ("dlt_mode", ctypes.c_int), ("sampler", ctypes.c_int), ("sprt", ctypes.c_int),
                ("lo", ctypes.c_int), ("lo_sample_size", ctypes.c_uint), ("lo_iterative_iterations", ctypes.c_uint),
                ("lo_inner_iterations", ctypes.c_uint), ("lo_threshold_multiplier", ctypes.c_uint),
                ("cell_size", ctypes.c_int), ("neighbors", ctypes.c_int), ("knn", ctypes.c_uint),
                ("spatial_coherence_gc", ctypes.c_float)]


class OrcMT(ctypes.Structure):
    _fields_ = [("mt", ctypes.c_uint32 * 624), ("i", ctypes.c_int)]


def build():
    """Compile the oracle with its own Makefile (plain gcc)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.orc_random.restype = ctypes.c_long
        L.orc_uniform_new.restype = ctypes.c_void_p
        L.orc_uniform_new.argtypes = [ctypes.c_uint, ctypes.c_uint]
        L.orc_uniform_free.argtypes = [ctypes.c_void_p]
        L.orc_uniform_samples.argtypes = [ctypes.c_void_p, _i32p, ctypes.c_int]
        L.orc_est_new.restype = ctypes.c_void_p
        L.orc_est_new.argtypes = [ctypes.c_int, _f32p, ctypes.c_uint, ctypes.c_int]
        L.orc_est_free.argtypes = [ctypes.c_void_p]
        L.orc_est_estimate.argtypes = [ctypes.c_void_p, _i32p, _f32p]
        L.orc_est_nonminimal.argtypes = [ctypes.c_void_p, _i32p, ctypes.c_uint, _f32p]
        L.orc_est_nonminimal_weighted.argtypes = [ctypes.c_void_p, _i32p, ctypes.c_uint, _f32p, _f32p]
        L.orc_sym_eig_min.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
        L.orc_est_set_model.argtypes = [ctypes.c_void_p, _f32p]
        L.orc_est_error.argtypes = [ctypes.c_void_p, ctypes.c_uint]
        L.orc_est_error.restype = ctypes.c_float
        L.orc_inv3x3.argtypes = [_f32p, _f32p]
        L.orc_quality.argtypes = [ctypes.c_void_p, _f32p, ctypes.c_float, _i32p, _f32p, _i32p]
        L.orc_score_models.argtypes = [ctypes.c_void_p, _f32p, ctypes.c_int, ctypes.c_float, _i32p, _f32p]
        L.orc_est_max_models.argtypes = [ctypes.c_void_p]
        L.orc_cubic_roots.argtypes = [ctypes.c_double] * 4 + [ctypes.POINTER(ctypes.c_double)]
        L.orc_real_roots.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
        L.orc_e5_candidates.argtypes = [ctypes.c_void_p, _i32p, _f32p, _i32p]
        L.orc_estimate_batch.argtypes = [ctypes.c_void_p, _i32p, ctypes.c_int, _f32p, _i32p]
        L.orc_gt_inliers_homography.argtypes = [_f32p, ctypes.c_uint, _f32p, ctypes.c_float]
        L.orc_std_termination.argtypes = [ctypes.c_uint, ctypes.c_uint, ctypes.c_uint, ctypes.c_float, ctypes.c_uint]
        L.orc_std_termination.restype = ctypes.c_uint
        L.orc_ransac_run.argtypes = [ctypes.c_int, _f32p, ctypes.c_uint, ctypes.c_float, ctypes.c_float,
                                     ctypes.c_uint, ctypes.c_uint, ctypes.c_int, ctypes.POINTER(OrcResult),
                                     _i32p, _u32p, _i32p, _f32p, ctypes.c_int]
        L.orc_ransac_run_cfg.argtypes = [ctypes.c_int, _f32p, ctypes.c_uint, ctypes.POINTER(OrcConfig),
                                         ctypes.POINTER(OrcResult), _i32p, _u32p, _i32p, _f32p, ctypes.c_int]
        L.orc_mt_seed.argtypes = [ctypes.POINTER(OrcMT), ctypes.c_uint32]
        L.orc_mt_next.argtypes = [ctypes.POINTER(OrcMT)]
        L.orc_mt_next.restype = ctypes.c_uint32
        L.orc_mt_uniform.argtypes = [ctypes.POINTER(OrcMT), ctypes.c_uint]
        L.orc_prosac_new.restype = ctypes.c_void_p
        L.orc_prosac_new.argtypes = [ctypes.c_uint, ctypes.c_uint, ctypes.c_uint32]
        L.orc_prosac_free.argtypes = [ctypes.c_void_p]
        L.orc_prosac_growth.argtypes = [ctypes.c_void_p]
        L.orc_prosac_growth.restype = _u32p
        L.orc_prosac_largest.argtypes = [ctypes.c_void_p]
        L.orc_prosac_largest.restype = ctypes.c_uint
        L.orc_prosac_set_term_len.argtypes = [ctypes.c_void_p, ctypes.c_uint]
        L.orc_prosac_sample.argtypes = [ctypes.c_void_p, _i32p]
        L.orc_prosac_term_new.restype = ctypes.c_void_p
        L.orc_prosac_term_new.argtypes = [_u32p, ctypes.c_uint, ctypes.c_uint, ctypes.c_float, ctypes.c_uint]
        L.orc_prosac_term_free.argtypes = [ctypes.c_void_p]
        L.orc_prosac_term_length.argtypes = [ctypes.c_void_p]
        L.orc_prosac_term_length.restype = ctypes.c_uint
        L.orc_prosac_term_update.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.POINTER(ctypes.c_uint8),
                                             ctypes.c_uint]
        L.orc_prosac_term_update.restype = ctypes.c_uint
        L.orc_sprt_new.restype = ctypes.c_void_p
        L.orc_sprt_new.argtypes = [ctypes.c_int, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint, ctypes.c_int]
        L.orc_sprt_free.argtypes = [ctypes.c_void_p]
        L.orc_sprt_pool.argtypes = [ctypes.c_void_p]
        L.orc_sprt_pool.restype = _u32p
        L.orc_sprt_A.argtypes = [ctypes.c_void_p]
        L.orc_sprt_A.restype = ctypes.c_double
        L.orc_sprt_upper_bound.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.orc_sprt_upper_bound.restype = ctypes.c_uint
        L.orc_hypothesis_loop.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_float, _f32p]
        L.orc_generate_line2d.argtypes = [ctypes.c_uint, ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, _f32p, _f32p]
        L.orc_generate_line2d_next.argtypes = [ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_int, _f32p, _f32p]
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t)


def glibc_stream(seed, n):
    L = lib()
    L.orc_srandom(ctypes.c_uint(seed))
    return np.array([L.orc_random() for _ in range(n)], dtype=np.int64)


def uniform_samples(seed, n_points, m, count):
    """glibc-seeded UniformSampler stream: count x m int32."""
    L = lib()
    L.orc_srandom(ctypes.c_uint(seed))
    s = L.orc_uniform_new(n_points, m)
    out = np.zeros((count, m), dtype=np.int32)
    L.orc_uniform_samples(s, _p(out, _i32p), count)
    L.orc_uniform_free(s)
    return out


class Estimator:
    def __init__(self, kind, points, dlt_mode=DLT_THIN):
        self.points = np.ascontiguousarray(points, dtype=np.float32)
        self.kind = kind
        self.n = self.points.shape[0]
        self._h = lib().orc_est_new(kind, _p(self.points, _f32p), self.n, dlt_mode)
        if not self._h:
            raise ValueError("oracle: unsupported estimator %r" % kind)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_est_free(self._h)
            self._h = None

    @property
    def m(self):
        return {LINE2D: 2, FUNDAMENTAL: 7, ESSENTIAL: 5}.get(self.kind, 4)

    @property
    def max_models(self):
        return 3 if self.kind == FUNDAMENTAL else 1

    def estimate(self, sample):
        sample = np.ascontiguousarray(sample, dtype=np.int32)
        out = np.zeros(27, dtype=np.float32)
        k = lib().orc_est_estimate(self._h, _p(sample, _i32p), _p(out, _f32p))
        return out[: 9 * k].reshape(k, 9)

    def e5_candidates(self, sample):
        sample = np.ascontiguousarray(sample, dtype=np.int32)
        cand = np.zeros((10, 9), dtype=np.float32)
        ok = np.zeros(10, dtype=np.int32)
        k = lib().orc_e5_candidates(self._h, _p(sample, _i32p), _p(cand, _f32p), _p(ok, _i32p))
        return cand[:k].copy(), ok[:k].astype(bool)

    def estimate_batch(self, samples):
        samples = np.ascontiguousarray(samples, dtype=np.int32)
        B = samples.shape[0]
        km = self.max_models
        models = np.zeros((B, km, 9), dtype=np.float32)
        nm = np.zeros(B, dtype=np.int32)
        lib().orc_estimate_batch(self._h, _p(samples, _i32p), B, _p(models, _f32p), _p(nm, _i32p))
        return (models[:, 0] if km == 1 else models), nm

    def nonminimal(self, idx):
        idx = np.ascontiguousarray(idx, dtype=np.int32)
        out = np.zeros(9, dtype=np.float32)
        ok = lib().orc_est_nonminimal(self._h, _p(idx, _i32p), len(idx), _p(out, _f32p))
        return out if ok else None

    def nonminimal_weighted(self, idx, weights):
        """weights: one float per point of the set (indexed by point index, as the reference)."""
        idx = np.ascontiguousarray(idx, dtype=np.int32)
        weights = np.ascontiguousarray(weights, dtype=np.float32)
        assert weights.size >= self.n
        out = np.zeros(9, dtype=np.float32)
        ok = lib().orc_est_nonminimal_weighted(self._h, _p(idx, _i32p), len(idx), _p(weights, _f32p), _p(out, _f32p))
        if ok < 0:
            raise NotImplementedError("weighted non-minimal fit: homography / fundamental only")
        return out if ok else None

    def errors(self, model):
        model = np.ascontiguousarray(model, dtype=np.float32).reshape(-1)
        full = np.zeros(9, dtype=np.float32)
        full[: model.size] = model
        L = lib()
        L.orc_est_set_model(self._h, _p(full, _f32p))
        return np.array([L.orc_est_error(self._h, i) for i in range(self.n)], dtype=np.float32)

    def quality(self, model, thr, with_inliers=False):
        model = np.ascontiguousarray(model, dtype=np.float32).reshape(-1)
        full = np.zeros(9, dtype=np.float32)
        full[: model.size] = model
        cnt = ctypes.c_int(0)
        s = ctypes.c_float(0)
        inl = np.zeros(max(self.n, 1), dtype=np.int32) if with_inliers else None
        lib().orc_quality(self._h, _p(full, _f32p), ctypes.c_float(thr), ctypes.byref(cnt), ctypes.byref(s),
                          _p(inl, _i32p) if inl is not None else None)
        if with_inliers:
            return cnt.value, s.value, inl[: cnt.value].copy()
        return cnt.value, s.value

    def score_models(self, models, thr):
        models = np.ascontiguousarray(models, dtype=np.float32).reshape(-1, 9)
        n = models.shape[0]
        c = np.zeros(n, dtype=np.int32)
        s = np.zeros(n, dtype=np.float32)
        lib().orc_score_models(self._h, _p(models, _f32p), n, ctypes.c_float(thr), _p(c, _i32p), _p(s, _f32p))
        return c, s


def sprt_fixed_batch(est, pool, thr, models, starts, epsilon, delta, A):
    """The throughput SPRT's per-model test (sprt.hpp:209-234's fp64 lambda walk, fixed epsilon /
    delta / A, each model from its own pool start) -> (good, count [-1 if rejected], tested)."""
    L = lib()
    models = np.ascontiguousarray(models, dtype=np.float32).reshape(-1, 9)
    pool = np.ascontiguousarray(pool, dtype=np.uint32)
    starts = np.ascontiguousarray(starts, dtype=np.uint32)
    K = models.shape[0]
    good = np.zeros(K, np.int32)
    cnt = np.zeros(K, np.int32)
    tested = np.zeros(K, np.uint32)
    _u = ctypes.POINTER(ctypes.c_uint)
    L.orc_sprt_fixed_batch.restype = None
    L.orc_sprt_fixed_batch.argtypes = [ctypes.c_void_p, _u, ctypes.c_uint, ctypes.c_float, _f32p, _u, ctypes.c_int,
                                       ctypes.c_double, ctypes.c_double, ctypes.c_double, _i32p, _i32p, _u]
    L.orc_sprt_fixed_batch(est._h, pool.ctypes.data_as(_u), len(pool), ctypes.c_float(thr), _p(models, _f32p),
                           starts.ctypes.data_as(_u), K, epsilon, delta, A, _p(good, _i32p), _p(cnt, _i32p),
                           tested.ctypes.data_as(_u))
    return good.astype(bool), cnt, tested


def e5_matrix(N, z):
    """The oracle's M(z) (usac_oracle.c e5_matrix) of a 4 x 9 null basis."""
    L = lib()
    N = np.ascontiguousarray(N, dtype=np.float64).reshape(36)
    M = np.zeros(100, np.float64)
    _d = ctypes.POINTER(ctypes.c_double)
    L.orc_e5_matrix.restype = None
    L.orc_e5_matrix.argtypes = [_d, ctypes.c_double, _d]
    L.orc_e5_matrix(N.ctypes.data_as(_d), float(z), M.ctypes.data_as(_d))
    return M.reshape(10, 10)


MBLOCK_REF_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_ref", "libmblock_ref.so")


def mblock_ref_available():
    return os.path.exists(MBLOCK_REF_PATH)


def mblock_ref_eval(N, z):
    """The reference's own mblock.hpp (compiled where it lies into oracle/_ref) evaluated at z."""
    L = ctypes.CDLL(MBLOCK_REF_PATH)
    _d = ctypes.POINTER(ctypes.c_double)
    L.mblock_ref_eval.restype = None
    L.mblock_ref_eval.argtypes = [_d, ctypes.c_double, _d]
    N = np.ascontiguousarray(N, dtype=np.float64).reshape(36)
    M = np.zeros(100, np.float64)
    L.mblock_ref_eval(N.ctypes.data_as(_d), float(z), M.ctypes.data_as(_d))
    return M.reshape(10, 10)


RPOLY_REF_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_ref", "librpoly_ref.so")


def rpoly_ref_available():
    return os.path.exists(RPOLY_REF_PATH)


def rpoly_ref_zeros(coeffs):
    """The reference's own rpoly_ak1 (usac/estimator/essential/rpoly.cpp:7-230, compiled where it
    lies into oracle/_ref by oracle/Makefile) on sum coeffs[i] z^i -> (real parts, imaginary
    parts) of the zeros it reports, in the order it found them (its degree shrinks when it fails
    after 20 shifts, rpoly.cpp:214-218)."""
    L = ctypes.CDLL(RPOLY_REF_PATH)
    _d = ctypes.POINTER(ctypes.c_double)
    L.rpoly_ref_zeros.restype = ctypes.c_int
    L.rpoly_ref_zeros.argtypes = [_d, ctypes.c_int, _d, _d]
    a = np.ascontiguousarray(coeffs, dtype=np.float64)
    zr = np.zeros(100)
    zi = np.zeros(100)
    k = L.rpoly_ref_zeros(a.ctypes.data_as(_d), len(a) - 1, zr.ctypes.data_as(_d), zi.ctypes.data_as(_d))
    k = max(k, 0)
    return zr[:k].copy(), zi[:k].copy()


def e5_poly(est, sample):
    """The degree-10 polynomial det M(z) of a 5-point sample, ascending powers: the input of the
    root step (usac_oracle.c e5_poly; five_points.cpp:113-148 interpolates the same polynomial)."""
    L = lib()
    _d = ctypes.POINTER(ctypes.c_double)
    L.orc_e5_poly.restype = None
    L.orc_e5_poly.argtypes = [ctypes.c_void_p, _i32p, _d]
    s = np.ascontiguousarray(sample, dtype=np.int32)
    a = np.zeros(11)
    L.orc_e5_poly(est._h, _p(s, _i32p), a.ctypes.data_as(_d))
    return a


def real_roots(coeffs):
    """real zeros of sum coeffs[i] z^i (degree <= 10) in the order the 5-pt solver's Jenkins-Traub
    root step finds them (usac_oracle.c jt_rpoly; five_points.cpp:143-157)"""
    a = np.ascontiguousarray(coeffs, dtype=np.float64)
    r = np.zeros(max(len(a) - 1, 1), dtype=np.float64)
    k = lib().orc_real_roots(a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), len(a) - 1,
                             r.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    return r[:k].copy()


def asc_roots(coeffs):
    """the 5-pt solver's candidate values: real roots of sum coeffs[i] z^i, ascending (usac_oracle.c asc_real_roots)"""
    a = np.ascontiguousarray(coeffs, dtype=np.float64)
    r = np.zeros(max(len(a) - 1, 1), dtype=np.float64)
    k = lib().orc_asc_roots(a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), len(a) - 1,
                            r.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    return r[:k].copy()


def rpoly_zeros(coeffs):
    """every zero the oracle's rpoly restatement reports (real, imaginary parts), in its order"""
    L = lib()
    _d = ctypes.POINTER(ctypes.c_double)
    L.orc_rpoly_zeros.restype = ctypes.c_int
    L.orc_rpoly_zeros.argtypes = [_d, ctypes.c_int, _d, _d]
    a = np.ascontiguousarray(coeffs, dtype=np.float64)
    zr = np.zeros(10)
    zi = np.zeros(10)
    k = max(L.orc_rpoly_zeros(a.ctypes.data_as(_d), len(a) - 1, zr.ctypes.data_as(_d), zi.ctypes.data_as(_d)), 0)
    return zr[:k].copy(), zi[:k].copy()


def jt_log(x):
    L = lib()
    L.orc_jt_log.restype = ctypes.c_double
    L.orc_jt_log.argtypes = [ctypes.c_double]
    return L.orc_jt_log(float(x))


def jt_exp(y):
    L = lib()
    L.orc_jt_exp.restype = ctypes.c_double
    L.orc_jt_exp.argtypes = [ctypes.c_double]
    return L.orc_jt_exp(float(y))


def cubic_roots(c0, c1, c2, c3):
    r = (ctypes.c_double * 3)()
    k = lib().orc_cubic_roots(c0, c1, c2, c3, r)
    return [r[i] for i in range(k)]


def inv3x3(m):
    m = np.ascontiguousarray(m, dtype=np.float32).reshape(9)
    out = np.zeros(9, dtype=np.float32)
    ok = lib().orc_inv3x3(_p(m, _f32p), _p(out, _f32p))
    return out, bool(ok)


def gt_inliers_homography(points, model, thr):
    points = np.ascontiguousarray(points, dtype=np.float32)
    model = np.ascontiguousarray(model, dtype=np.float32).reshape(9)
    return lib().orc_gt_inliers_homography(_p(points, _f32p), points.shape[0], _p(model, _f32p),
                                           ctypes.c_float(thr))


def std_termination(inliers, n, m, p, max_iters=10000):
    return lib().orc_std_termination(inliers, n, m, ctypes.c_float(p), max_iters)


def ransac_run(kind, points, thr, p, seed, max_iters=10000, dlt_mode=DLT_THIN, rec_cap=4096,
               sampler=SAMPLER_UNIFORM, sprt=False, lo=LO_NONE, lo_params=(14, 4, 20, 10), cell_size=50,
               neighbors=NEIGHBORS_GRID, knn=7, spatial_coherence_gc=0.1):
    points = np.ascontiguousarray(points, dtype=np.float32)
    n = points.shape[0]
    res = OrcResult()
    inl = np.zeros(max(n, 1), dtype=np.int32)
    ri = np.zeros(rec_cap, dtype=np.uint32)
    rc = np.zeros(rec_cap, dtype=np.int32)
    rs = np.zeros(rec_cap, dtype=np.float32)
    cfg = OrcConfig(thr, p, max_iters, seed, dlt_mode, sampler, 1 if sprt else 0, lo, *lo_params, cell_size,
                    neighbors, knn, spatial_coherence_gc)
    ret = lib().orc_ransac_run_cfg(kind, _p(points, _f32p), n, ctypes.byref(cfg), ctypes.byref(res), _p(inl, _i32p),
                                   _p(ri, _u32p), _p(rc, _i32p), _p(rs, _f32p), rec_cap)
    k = min(res.n_records, rec_cap)
    return {
        "ret": ret,
        "model": np.array(res.model[:], dtype=np.float32),
        "inliers": res.inliers,
        "iters": res.iters,
        "polish_passes": res.polish_passes,
        "minimal_model": np.array(res.minimal_model[:], dtype=np.float32),
        "minimal_inliers": res.minimal_inliers,
        "inlier_idx": inl[: res.inliers].copy() if ret == 0 else np.zeros(0, np.int32),
        "records": list(zip(ri[:k].tolist(), rc[:k].tolist(), rs[:k].tolist())),
        "sprt_rejected": res.sprt_rejected,
        "sprt_histories": res.sprt_histories,
        "prosac_term_len": res.prosac_term_len,
        "lo_inner_iters": res.lo_inner_iters,
        "lo_iterative_iters": res.lo_iterative_iters,
    }


def knn(points, k):
    """KNN neighbours (nearest_neighbors.cpp:69-128): (idx n x k int32, d2 n x k float32),
    self excluded, equal distances by ascending index."""
    L = lib()
    pts = np.ascontiguousarray(points, dtype=np.float32)
    n, cols = pts.shape
    idx = np.zeros((n, k), dtype=np.int32)
    d2 = np.zeros((n, k), dtype=np.float32)
    L.orc_knn.argtypes = [_f32p, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint, _i32p, _f32p]
    L.orc_knn.restype = None
    L.orc_knn(_p(pts, _f32p), n, cols, k, _p(idx, _i32p), _p(d2, _f32p))
    return idx, d2


def _bk_args(unary, ei, ej, e00, e01, e10, e11):
    a = [np.ascontiguousarray(unary, np.float32), np.ascontiguousarray(ei, np.int32), np.ascontiguousarray(ej, np.int32)]
    a += [np.ascontiguousarray(x, np.float32) for x in (e00, e01, e10, e11)]
    return a


def _bk_call(fn, unary, ei, ej, e00, e01, e10, e11):
    a = _bk_args(unary, ei, ej, e00, e01, e10, e11)
    n, m = len(a[0]), len(a[1])
    out = np.zeros(n, np.int32)
    fn.restype = ctypes.c_float
    fn.argtypes = [ctypes.c_int, _f32p, ctypes.c_int, _i32p, _i32p, _f32p, _f32p, _f32p, _f32p, _i32p]
    f = fn(n, _p(a[0], _f32p), m, _p(a[1], _i32p), _p(a[2], _i32p), _p(a[3], _f32p), _p(a[4], _f32p),
           _p(a[5], _f32p), _p(a[6], _f32p), _p(out, _i32p))
    return out.astype(bool), f


def bk_label(unary, ei, ej, e00, e01, e10, e11):
    """The oracle's BK restatement: add_term1(i, unary[i], 0), add_term2 per pair, maxflow ->
    (sink mask, flow)."""
    return _bk_call(lib().orc_bk_label, unary, ei, ej, e00, e01, e10, e11)


GCO_REF_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_ref", "libgco_ref.so")
_gco = None


def gco_ref_available():
    return os.path.exists(GCO_REF_PATH)


def gco_ref_label(unary, ei, ej, e00, e01, e10, e11):
    """The reference's own gco-v3.0 max-flow (oracle/_ref, built from /root/reference)."""
    global _gco
    if _gco is None:
        _gco = ctypes.CDLL(GCO_REF_PATH)
    return _bk_call(_gco.gco_ref_label, unary, ei, ej, e00, e01, e10, e11)


def grid_neighbors(points, cell_size):
    """Grid neighbour lists (nearest_neighbors.cpp:160-202) as a list of int arrays."""
    L = lib()
    pts = np.ascontiguousarray(points, dtype=np.float32)
    L.orc_grid_new.restype = ctypes.c_void_p
    L.orc_grid_new.argtypes = [_f32p, ctypes.c_uint, ctypes.c_int]
    L.orc_grid_count.argtypes = [ctypes.c_void_p, ctypes.c_uint]
    L.orc_grid_list.argtypes = [ctypes.c_void_p, ctypes.c_uint]
    L.orc_grid_list.restype = _i32p
    L.orc_grid_free.argtypes = [ctypes.c_void_p]
    g = L.orc_grid_new(_p(pts, _f32p), len(pts), cell_size)
    out = []
    for i in range(len(pts)):
        k = L.orc_grid_count(g, i)
        out.append(np.ctypeslib.as_array(L.orc_grid_list(g, i), shape=(k,)).copy() if k else np.zeros(0, np.int32))
    L.orc_grid_free(g)
    return out


def mt19937_stream(seed, count):
    g = OrcMT()
    lib().orc_mt_seed(ctypes.byref(g), seed)
    return np.array([lib().orc_mt_next(ctypes.byref(g)) for _ in range(count)], dtype=np.uint64)


def mt19937_uniform(seed, max_, count):
    g = OrcMT()
    lib().orc_mt_seed(ctypes.byref(g), seed)
    return np.array([lib().orc_mt_uniform(ctypes.byref(g), max_) for _ in range(count)], dtype=np.int64)


def prosac_samples(seed, n_points, m, count, term_len=None):
    """ProsacSampler stream (termination_length fixed at term_len, default n): count x m."""
    L = lib()
    p = L.orc_prosac_new(m, n_points, seed)
    if term_len is not None:
        L.orc_prosac_set_term_len(p, term_len)
    out = np.zeros((count, m), dtype=np.int32)
    for i in range(count):
        L.orc_prosac_sample(p, _p(out[i], _i32p))
    growth = np.ctypeslib.as_array(L.orc_prosac_growth(p), shape=(n_points,)).copy()
    largest = L.orc_prosac_largest(p)
    L.orc_prosac_free(p)
    return out, growth, largest


def sprt_pool(seed, kind, n_points, m, max_iters=10000):
    """The SPRT random pool after srandom(seed) (consumes n_points glibc draws) and A_0."""
    L = lib()
    L.orc_srandom(ctypes.c_uint(seed))
    s = L.orc_sprt_new(kind, n_points, m, max_iters, 20)
    pool = np.ctypeslib.as_array(L.orc_sprt_pool(s), shape=(n_points,)).copy()
    A = L.orc_sprt_A(s)
    L.orc_sprt_free(s)
    return pool, A


def hypothesis_loop(kind, points, thr, seed, count, dlt_mode=DLT_THIN):
    """Reference-style sample+solve+score loop for `count` hypotheses (CPU baseline)."""
    est = Estimator(kind, points, dlt_mode)
    L = lib()
    L.orc_srandom(ctypes.c_uint(seed))
    s = L.orc_uniform_new(est.n, est.m)
    best_sum = ctypes.c_float(0)
    best = L.orc_hypothesis_loop(est._h, s, count, ctypes.c_float(thr), ctypes.byref(best_sum))
    L.orc_uniform_free(s)
    return best, best_sum.value


def generate_line2d(seed, noise, inliers, outliers, border_x, border_y):
    """Generate2DLinePoints after srand(seed); seed=None continues the rand() stream."""
    pts = np.zeros((inliers + outliers, 2), dtype=np.float32)
    gt = np.zeros(3, dtype=np.float32)
    if seed is None:
        lib().orc_generate_line2d_next(ctypes.c_float(noise), inliers, outliers, border_x, border_y,
                                       _p(pts, _f32p), _p(gt, _f32p))
    else:
        lib().orc_generate_line2d(seed, ctypes.c_float(noise), inliers, outliers, border_x, border_y,
                                  _p(pts, _f32p), _p(gt, _f32p))
    return pts, gt


def generate_line2d_dataset():
    """generate_syntectic_dataset (generator/generator.cpp:6-67): the eight scenes of
    dataset/line2d/ in dataset.txt order on one rand() stream from the default seed 1 ->
    [(name, points, gt_model)]."""
    out = []
    first = True
    for w in (1000, 1200):
        for h in (1000, 1200):
            for pct in (0.02, 0.05):
                outliers = 10000
                inliers = int(outliers * np.float32(pct))
                pts, gt = generate_line2d(1 if first else None, 3.0, inliers, outliers, w, h)
                first = False
                out.append(("w=%d_h=%d_n=3.000000_I=%d_N=%d" % (w, h, inliers, inliers + outliers), pts, gt))
    return out


def set_f8_rank2(on):
    """Rank-2 enforcement in the 8-point polish (eight_points.cpp:58-68, commented out in the
    current reference): the revision that produced results/kusvod2/*.csv ran it.  Test-only."""
    lib().orc_set_f8_rank2(1 if on else 0)


def set_sprt_file_order(on):
    """SPRT point order of the revision that produced results/line2d/*_001.csv: every model
    tested on the points in file order from point 0 (no shuffled pool, no rolling index; the
    current sprt.hpp:93-107,211-223 shuffles and rolls).  Test-only."""
    lib().orc_set_sprt_file_order(1 if on else 0)


def hypothesis_loop_mt(kind, points, thr, seed, count, threads, dlt_mode=DLT_THIN):
    """All-cores CPU baseline: `count` hypotheses of the reference-style loop on `threads`
    pthreads (disjoint ranges, one estimator each) -> (wall seconds, best inlier count)."""
    pts = np.ascontiguousarray(points, dtype=np.float32)
    L = lib()
    L.orc_hypothesis_loop_mt.restype = ctypes.c_double
    L.orc_hypothesis_loop_mt.argtypes = [ctypes.c_int, _f32p, ctypes.c_uint, ctypes.c_int, ctypes.c_float,
                                         ctypes.c_uint, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    best = ctypes.c_int(0)
    dt = L.orc_hypothesis_loop_mt(kind, _p(pts, _f32p), pts.shape[0], dlt_mode, thr, seed, count, threads,
                                  ctypes.byref(best))
    return dt, best.value


def sym_eig_min(A):
    """The LSQ fits' 9x9 eigen spec: (smallest-eigenvalue eigenvector, True if inverse iteration
    converged / False if the Jacobi fall-back ran)."""
    A = np.ascontiguousarray(A, dtype=np.float64).reshape(81)
    v = np.zeros(9, dtype=np.float64)
    dp = ctypes.POINTER(ctypes.c_double)
    ok = lib().orc_sym_eig_min(A.ctypes.data_as(dp), v.ctypes.data_as(dp))
    return v, bool(ok)
