"""ransac_amd -- MI355X-native USAC hypothesize-and-verify engine.

Python host mirror of the reference's plugin surface (MathsionYang/Ransac ``usac/``):
``Model`` (usac/model.hpp), ``Ransac`` + ``RansacOutput`` (usac/ransac/ransac.hpp,
ransac_output.hpp), ``Score`` (usac/quality/quality.hpp), and the operator level
``Context`` (Estimator::EstimateModel, Quality::getNumberInliers, ... batched).  All
compute goes through the C-ABI of ``libransac_amd.so`` (include/usac_gpu.h) into the HIP
kernels; there is no Python or CPU compute fallback -- if the library or a GPU is
missing, the calls raise.
"""
import ctypes
import enum
import os
import subprocess

import numpy as np

__all__ = ["ESTIMATOR", "SAMPLER", "LocOpt", "NeighborsSearch", "DLT", "Model", "Ransac", "RansacOutput", "Score", "Context", "Record",
           "RandomGenerator", "Sampler", "TerminationCriteria", "SPRT", "LocalOptimization", "SprtState",
           "build", "lib", "std_termination", "uniform_samples", "prosac_samples", "sprt_pool", "UsacError"]

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RANSAC_AMD_LIB") or os.path.join(_HERE, "libransac_amd.so")  # override: A/B builds


class ESTIMATOR(enum.IntEnum):  # usac/model.hpp:10
    NullE = 0
    Line2d = 1
    Homography = 2
    Fundamental = 3
    Essential = 4


class SAMPLER(enum.IntEnum):  # usac/model.hpp:11
    NullS = 0
    Uniform = 1
    ProgressiveNAPSAC = 2
    Napsac = 3
    Prosac = 4
    Evsac = 5
    ProsacNapsac = 6


class LocOpt(enum.IntEnum):  # usac/model.hpp:13 (IRLS is out of scope: debug prints only)
    NullLO = 0
    InItLORsc = 1
    InItFLORsc = 2
    GC = 3


class NeighborsSearch(enum.IntEnum):  # usac/model.hpp:12 (NullN / Nanoflann = KNN on the device)
    NullN = 0
    Nanoflann = 1
    Grid = 2


class DLT(enum.IntEnum):
    THIN = 0        # reference semantics: vt.row(7) of the thin 8x9 SVD (dlt.cpp:43-48)
    NULLSPACE = 1   # true null vector


class UsacError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("usac error %d: %s" % (code, msg))
        self.code = code


class Record(ctypes.Structure):
    _fields_ = [("hyp_index", ctypes.c_uint64), ("inliers", ctypes.c_int32), ("score", ctypes.c_float),
                ("model", ctypes.c_float * 9), ("valid", ctypes.c_int32)]

    def as_dict(self):
        return {"hyp_index": int(self.hyp_index), "inliers": int(self.inliers), "score": float(self.score),
                "model": np.array(self.model[:], dtype=np.float32), "valid": bool(self.valid)}


class _Params(ctypes.Structure):
    _fields_ = [("threshold", ctypes.c_float), ("desired_prob", ctypes.c_float), ("max_iterations", ctypes.c_uint32),
                ("seed", ctypes.c_uint32), ("dlt_mode", ctypes.c_int32), ("batch", ctypes.c_uint32),
                ("sampler", ctypes.c_int32), ("sprt", ctypes.c_int32), ("lo", ctypes.c_int32),
                ("lo_sample_size", ctypes.c_uint32), ("lo_iterative_iterations", ctypes.c_uint32),
                ("lo_inner_iterations", ctypes.c_uint32), ("lo_threshold_multiplier", ctypes.c_uint32),
                ("cell_size", ctypes.c_int32), ("neighbors", ctypes.c_int32), ("knn", ctypes.c_uint32),
                ("spatial_coherence_gc", ctypes.c_float), ("max_hypothesis_test_before_sprt", ctypes.c_uint32)]


class SprtState(ctypes.Structure):
    """usac_sprt_state (include/usac_gpu.h): the loop state in / out of usac_sprt_replay."""
    _fields_ = [("iters", ctypes.c_uint32), ("max_iters", ctypes.c_uint32), ("best_inliers", ctypes.c_int32),
                ("best_score", ctypes.c_float), ("sample", ctypes.c_uint32), ("slot", ctypes.c_uint32),
                ("found", ctypes.c_int32), ("inliers", ctypes.c_int32), ("score", ctypes.c_float),
                ("found_sample", ctypes.c_uint32), ("found_slot", ctypes.c_uint32), ("rejected", ctypes.c_uint32)]


class _RunOutput(ctypes.Structure):
    _fields_ = [("model", ctypes.c_float * 9), ("inliers", ctypes.c_int32), ("iters", ctypes.c_uint32),
                ("time_us", ctypes.c_int64), ("n_records", ctypes.c_int32), ("polish_passes", ctypes.c_int32),
                ("minimal_model", ctypes.c_float * 9), ("minimal_inliers", ctypes.c_int32),
                ("batches", ctypes.c_uint32), ("sprt_rejected", ctypes.c_int32), ("sprt_histories", ctypes.c_int32),
                ("prosac_term_len", ctypes.c_uint32), ("rollbacks", ctypes.c_uint32),
                ("lo_inner_iters", ctypes.c_uint32), ("lo_iterative_iters", ctypes.c_uint32),
                ("lo_rounds", ctypes.c_uint32), ("lo_stages", ctypes.c_uint32), ("sum_models", ctypes.c_uint32),
                ("lo_fits", ctypes.c_uint32), ("spec_batches", ctypes.c_uint32), ("spec_rollbacks", ctypes.c_uint32),
                ("spec_wasted", ctypes.c_uint32)]


# every symbol include/usac_gpu.h declares (checked by tests/test_abi.py)
ABI_SYMBOLS = [
    "usac_create", "usac_destroy", "usac_last_error", "usac_abi_version", "usac_set_dlt_mode", "usac_sample_size",
    "usac_num_points", "usac_estimate_models", "usac_score_models", "usac_get_inliers", "usac_knn", "usac_bk_label",
    "usac_nonminimal", "usac_lsq_fit",
    "usac_hypothesize_score", "usac_hypothesize_async", "usac_fetch_best", "usac_sync", "usac_last_timings",
    "usac_set_score_chunks", "usac_set_score_variant", "usac_last_counts", "usac_std_termination", "usac_ransac_run", "usac_ransac_run_sharded", "usac_uniform_samples",
    "usac_prosac_samples", "usac_sprt_pool", "usac_set_sprt", "usac_sprt_tested", "usac_set_device_sampler",
    "usac_draw_samples", "usac_set_cell_size", "usac_grid_neighbors",
    "usac_comm_unique_id", "usac_comm_init", "usac_comm_count", "usac_allgather_records", "usac_merge_records",
    "usac_exchange_best_async", "usac_exchange_best_wait",
    "usac_random_create", "usac_random_next", "usac_random_destroy", "usac_sampler_create", "usac_sampler_generate",
    "usac_sampler_generate_batch", "usac_sampler_state", "usac_sampler_destroy", "usac_termination_create",
    "usac_termination_bound", "usac_prosac_termination", "usac_termination_destroy", "usac_sprt_create",
    "usac_sprt_verify", "usac_sprt_upper_bound", "usac_sprt_stats", "usac_sprt_replay", "usac_sprt_destroy",
    "usac_lo_create", "usac_lo_get_model_score", "usac_lo_iters", "usac_lo_destroy", "usac_batch_sprt_info",
    "usac_selftest_rpoly", "usac_selftest_logexp", "usac_set_timing",
]


def build(jobs=8):
    """Compile libransac_amd.so for gfx950 in-tree (hipcc via ransac_amd/Makefile)."""
    subprocess.run(["make", "-s", "-C", _HERE, "-j%d" % jobs], check=True)


_lib = None
_P = ctypes.POINTER
_vp = ctypes.c_void_p


def lib():
    """Load libransac_amd.so (raises if it is missing: no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError("ransac_amd: %s is missing -- run ransac_amd.build() (hipcc, gfx950)" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    f32p, i32p, u32p, u8p = _P(ctypes.c_float), _P(ctypes.c_int32), _P(ctypes.c_uint32), _P(ctypes.c_uint8)
    sig = {
        "usac_create": (ctypes.c_int, [_P(_vp), ctypes.c_int, ctypes.c_int, f32p, ctypes.c_uint32, ctypes.c_uint32]),
        "usac_destroy": (None, [_vp]),
        "usac_last_error": (ctypes.c_char_p, [_vp]),
        "usac_abi_version": (ctypes.c_int, []),
        "usac_set_dlt_mode": (ctypes.c_int, [_vp, ctypes.c_int]),
        "usac_set_score_chunks": (ctypes.c_int, [_vp, ctypes.c_int]),
        "usac_set_score_variant": (ctypes.c_int, [_vp, ctypes.c_int]),
        "usac_last_counts": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_float),
                                            ctypes.c_uint32]),
        "usac_sample_size": (ctypes.c_uint32, [_vp]),
        "usac_num_points": (ctypes.c_uint32, [_vp]),
        "usac_estimate_models": (ctypes.c_int, [_vp, i32p, ctypes.c_uint32, f32p, i32p]),
        "usac_score_models": (ctypes.c_int, [_vp, f32p, ctypes.c_uint32, ctypes.c_float, i32p, f32p]),
        "usac_get_inliers": (ctypes.c_int, [_vp, f32p, ctypes.c_float, i32p, u32p, f32p]),
        "usac_knn": (ctypes.c_int, [_vp, ctypes.c_uint32, i32p, f32p]),
        "usac_bk_label": (ctypes.c_float, [ctypes.c_int, f32p, ctypes.c_int, i32p, i32p, f32p, f32p, f32p, f32p, i32p]),
        "usac_nonminimal": (ctypes.c_int, [_vp, i32p, ctypes.c_uint32, f32p]),
        "usac_lsq_fit": (ctypes.c_int, [_vp, i32p, ctypes.c_uint32, f32p, f32p]),
        "usac_hypothesize_score": (ctypes.c_int, [_vp, i32p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64,
                                                  ctypes.c_float, i32p, f32p, _P(Record)]),
        "usac_hypothesize_async": (ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64,
                                                  ctypes.c_float]),
        "usac_fetch_best": (ctypes.c_int, [_vp, _P(Record)]),
        "usac_sync": (ctypes.c_int, [_vp]),
        "usac_last_timings": (ctypes.c_int, [_vp, f32p]),
        "usac_set_timing": (ctypes.c_int, [_vp, ctypes.c_int]),
        "usac_std_termination": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                   ctypes.c_float, ctypes.c_uint32]),
        "usac_ransac_run": (ctypes.c_int, [_vp, _P(_Params), _P(_RunOutput), i32p, _P(Record), ctypes.c_uint32]),
        "usac_ransac_run_sharded": (ctypes.c_int, [_vp, _P(_Params), ctypes.c_int, ctypes.c_int, _vp, _vp,
                                                   _P(_RunOutput), i32p, _P(Record), ctypes.c_uint32]),
        "usac_uniform_samples": (ctypes.c_int, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                i32p]),
        "usac_prosac_samples": (ctypes.c_int, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                               ctypes.c_uint32, i32p]),
        "usac_sprt_pool": (ctypes.c_int, [ctypes.c_uint32, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, u32p,
                                          _P(ctypes.c_double)]),
        "usac_set_sprt": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_uint32, ctypes.c_double, ctypes.c_double]),
        "usac_set_device_sampler": (ctypes.c_int, [_vp, ctypes.c_int]),
        "usac_draw_samples": (ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64, _vp]),
        "usac_set_cell_size": (ctypes.c_int, [_vp, ctypes.c_int]),
        "usac_grid_neighbors": (ctypes.c_int, [_vp, ctypes.c_int, u32p, u32p, u32p, u32p, i32p, i32p, u32p]),
        "usac_sprt_tested": (ctypes.c_int, [_vp, _P(ctypes.c_uint64)]),
        "usac_batch_sprt_info": (ctypes.c_int, [_vp, _P(ctypes.c_double), u32p, ctypes.c_uint32]),
        "usac_comm_unique_id": (ctypes.c_int, [u8p]),
        "usac_comm_init": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, u8p]),
        "usac_comm_count": (ctypes.c_int, [_vp, i32p, i32p, i32p]),
        "usac_allgather_records": (ctypes.c_int, [_vp, _P(Record), _P(Record)]),
        "usac_exchange_best_async": (ctypes.c_int, [_vp, _vp, ctypes.c_uint32]),
        "usac_exchange_best_wait": (ctypes.c_int, [_vp, ctypes.c_uint32, _P(Record)]),
        "usac_merge_records": (ctypes.c_int, [_P(Record), ctypes.c_uint32, _P(Record)]),
        "usac_random_create": (ctypes.c_int, [ctypes.c_uint32, _P(_vp)]),
        "usac_random_next": (ctypes.c_uint32, [_vp]),
        "usac_random_destroy": (None, [_vp]),
        "usac_sampler_create": (ctypes.c_int, [_vp, _P(_Params), _vp, _P(_vp)]),
        "usac_sampler_generate": (ctypes.c_int, [_vp, i32p]),
        "usac_sampler_generate_batch": (ctypes.c_int, [_vp, ctypes.c_uint32, i32p]),
        "usac_sampler_state": (ctypes.c_int, [_vp, _P(ctypes.c_uint64), u32p, u32p]),
        "usac_sampler_destroy": (None, [_vp]),
        "usac_termination_create": (ctypes.c_int, [_vp, _P(_Params), _vp, _P(_vp)]),
        "usac_termination_bound": (ctypes.c_uint32, [_vp, ctypes.c_uint32, ctypes.c_uint32]),
        "usac_prosac_termination": (ctypes.c_int, [_vp, ctypes.c_uint32, f32p, u32p, u32p]),
        "usac_termination_destroy": (None, [_vp]),
        "usac_sprt_create": (ctypes.c_int, [_vp, _P(_Params), _vp, _P(_vp)]),
        "usac_sprt_verify": (ctypes.c_int, [_vp, f32p, ctypes.c_int32, ctypes.c_uint32, i32p, i32p, f32p]),
        "usac_sprt_upper_bound": (ctypes.c_uint32, [_vp, ctypes.c_uint32]),
        "usac_sprt_stats": (ctypes.c_int, [_vp, u32p, u32p]),
        "usac_sprt_replay": (ctypes.c_int, [_vp, f32p, i32p, ctypes.c_uint32, _P(SprtState)]),
        "usac_sprt_destroy": (None, [_vp]),
        "usac_lo_create": (ctypes.c_int, [_vp, _P(_Params), _P(_vp)]),
        "usac_lo_get_model_score": (ctypes.c_int, [_vp, f32p, i32p, f32p]),
        "usac_lo_iters": (ctypes.c_int, [_vp, u32p, u32p]),
        "usac_lo_destroy": (None, [_vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def _ptr(a, t):
    return a.ctypes.data_as(_P(t)) if a is not None else None


def bk_label(unary, ei, ej, e00, e01, e10, e11):
    """The graph-cut LO's host min cut (usac_bk_label): add_term1(i, unary[i], 0), add_term2 per
    pair, BK max-flow -> (sink mask, flow).  No device work."""
    a = [np.ascontiguousarray(unary, np.float32), np.ascontiguousarray(ei, np.int32), np.ascontiguousarray(ej, np.int32)]
    a += [np.ascontiguousarray(x, np.float32) for x in (e00, e01, e10, e11)]
    out = np.zeros(len(a[0]), np.int32)
    f = lib().usac_bk_label(len(a[0]), _ptr(a[0], ctypes.c_float), len(a[1]), _ptr(a[1], ctypes.c_int32),
                            _ptr(a[2], ctypes.c_int32), _ptr(a[3], ctypes.c_float), _ptr(a[4], ctypes.c_float),
                            _ptr(a[5], ctypes.c_float), _ptr(a[6], ctypes.c_float), _ptr(out, ctypes.c_int32))
    return out.astype(bool), f


def std_termination(inliers, points_size, sample_size, desired_prob, max_iterations=10000):
    """StandardTerminationCriteria::getUpBoundIterations (standard_termination_criteria.hpp:52-62)."""
    return int(lib().usac_std_termination(inliers, points_size, sample_size, ctypes.c_float(desired_prob),
                                          max_iterations))


def prosac_samples(seed, n_points, m, count, termination_length=None):
    """Host ProsacSampler stream (mt19937 seeded with `seed`), count x m int32."""
    out = np.zeros((count, m), dtype=np.int32)
    tl = n_points if termination_length is None else termination_length
    rc = lib().usac_prosac_samples(seed, n_points, m, count, tl, _ptr(out, ctypes.c_int32))
    if rc:
        raise UsacError(rc, "usac_prosac_samples")
    return out


def sprt_pool(seed, estimator, n_points, m):
    """SPRT random pool after srandom(seed) and the first threshold A."""
    pool = np.zeros(n_points, dtype=np.uint32)
    A = ctypes.c_double(0)
    rc = lib().usac_sprt_pool(seed, int(estimator), n_points, m, _ptr(pool, ctypes.c_uint32), ctypes.byref(A))
    if rc:
        raise UsacError(rc, "usac_sprt_pool")
    return pool, A.value


def uniform_samples(seed, n_points, m, count):
    """UniformSampler stream after srandom(seed) (uniform_sampler.hpp:42-54): count x m int32."""
    out = np.zeros((count, m), dtype=np.int32)
    rc = lib().usac_uniform_samples(seed, n_points, m, count, _ptr(out, ctypes.c_int32))
    if rc:
        raise UsacError(rc, "usac_uniform_samples")
    return out


class Context:
    """One device + estimator + resident correspondence set (operator-level API)."""

    def __init__(self, estimator, points, device=0):
        L = lib()
        self.points = np.ascontiguousarray(points, dtype=np.float32)
        if self.points.ndim != 2:
            raise ValueError("points must be N x cols")
        self.estimator = ESTIMATOR(estimator)
        self.n, self.cols = self.points.shape
        h = _vp()
        rc = L.usac_create(ctypes.byref(h), device, int(self.estimator), _ptr(self.points, ctypes.c_float), self.n,
                           self.cols)
        if rc != 0:
            raise UsacError(rc, "usac_create(device=%d, estimator=%s, n=%d, cols=%d) failed (no usable GPU?)"
                            % (device, self.estimator.name, self.n, self.cols))
        self._h = h
        self.m = int(L.usac_sample_size(h))
        # model slots per minimal sample: the 7-point solver returns up to 3 models
        self.spk = 3 if self.estimator == ESTIMATOR.Fundamental else 1

    def close(self):
        if getattr(self, "_h", None):
            lib().usac_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc, what):
        if rc != 0:
            msg = lib().usac_last_error(self._h)
            raise UsacError(rc, "%s: %s" % (what, msg.decode() if msg else ""))

    def set_dlt_mode(self, mode):
        self._check(lib().usac_set_dlt_mode(self._h, int(mode)), "set_dlt_mode")

    def set_score_chunks(self, chunks):
        self._check(lib().usac_set_score_chunks(self._h, int(chunks)), "set_score_chunks")

    def selftest_rpoly(self, coeffs):
        """The device's 5-point root step alone (usac_selftest_rpoly) on polynomials of 11 ascending
        coefficients -> (roots B x 10, numbers of real zeros), rpoly's order."""
        a = np.ascontiguousarray(coeffs, dtype=np.float64).reshape(-1, 11)
        r = np.zeros((a.shape[0], 10), np.float64)
        n = np.zeros(a.shape[0], np.int32)
        self._check(lib().usac_selftest_rpoly(self._h, _ptr(a, ctypes.c_double), a.shape[0], _ptr(r, ctypes.c_double),
                                              _ptr(n, ctypes.c_int32)), "selftest_rpoly")
        return r, n

    def selftest_logexp(self, x):
        """The root step's correctly rounded log / exp on the device (usac_selftest_logexp)."""
        v = np.ascontiguousarray(x, dtype=np.float64)
        lg = np.zeros_like(v)
        ex = np.zeros_like(v)
        self._check(lib().usac_selftest_logexp(self._h, _ptr(v, ctypes.c_double), len(v), _ptr(lg, ctypes.c_double),
                                               _ptr(ex, ctypes.c_double)), "selftest_logexp")
        return lg, ex

    def last_counts(self, n):
        """Per-slot (counts, sums) of the last batch as the score kernel left them."""
        c = np.zeros(n, dtype=np.int32)
        sm = np.zeros(n, dtype=np.float32)
        self._check(lib().usac_last_counts(self._h, _ptr(c, ctypes.c_int32), _ptr(sm, ctypes.c_float), n),
                    "last_counts")
        return c, sm

    def set_score_variant(self, variant):
        """0 = guard-band fast path (default), 1 = exact reference expression for every pair."""
        self._check(lib().usac_set_score_variant(self._h, int(variant)), "set_score_variant")

    def estimate_models(self, samples):
        """Estimator::EstimateModel over a batch of minimal samples -> (models, n_models):
        models is B x 9, or B x 3 x 9 for the fundamental 7-point solver (valid models first,
        zero-filled)."""
        s = np.ascontiguousarray(samples, dtype=np.int32).reshape(-1, self.m)
        B = s.shape[0]
        models = np.zeros((B, self.spk, 9), dtype=np.float32)
        nm = np.zeros(B, dtype=np.int32)
        self._check(lib().usac_estimate_models(self._h, _ptr(s, ctypes.c_int32), B, _ptr(models, ctypes.c_float),
                                               _ptr(nm, ctypes.c_int32)), "estimate_models")
        return (models[:, 0] if self.spk == 1 else models), nm

    def score_models(self, models, thr):
        """Quality::getNumberInliers for each model -> (counts, sums)."""
        m = np.ascontiguousarray(models, dtype=np.float32)
        if m.ndim == 1:
            m = m.reshape(1, -1)
        full = np.zeros((m.shape[0], 9), dtype=np.float32)
        full[:, : m.shape[1]] = m
        c = np.zeros(full.shape[0], dtype=np.int32)
        s = np.zeros(full.shape[0], dtype=np.float32)
        self._check(lib().usac_score_models(self._h, _ptr(full, ctypes.c_float), full.shape[0], ctypes.c_float(thr),
                                            _ptr(c, ctypes.c_int32), _ptr(s, ctypes.c_float)), "score_models")
        return c, s

    def knn(self, k, distances=True):
        """NearestNeighbors::getNearestNeighbors_nanoflann (nearest_neighbors.cpp:69-128) on the
        device -> (idx n x k int32, d2 n x k float32 or None): self excluded, ascending squared
        distance, equal distances by ascending index, -1 / inf where n - 1 < k."""
        idx = np.zeros((self.n, int(k)), dtype=np.int32)
        d2 = np.zeros((self.n, int(k)), dtype=np.float32) if distances else None
        self._check(lib().usac_knn(self._h, int(k), _ptr(idx, ctypes.c_int32),
                                   _ptr(d2, ctypes.c_float) if distances else None), "knn")
        return idx, d2

    def get_inliers(self, model, thr):
        """Quality::getNumberInliers(get_inliers=true) -> (count, sum, ascending indices)."""
        full = np.zeros(9, dtype=np.float32)
        mm = np.asarray(model, dtype=np.float32).reshape(-1)
        full[: mm.size] = mm
        idx = np.zeros(self.n, dtype=np.int32)
        n = ctypes.c_uint32(0)
        s = ctypes.c_float(0)
        self._check(lib().usac_get_inliers(self._h, _ptr(full, ctypes.c_float), ctypes.c_float(thr),
                                           _ptr(idx, ctypes.c_int32), ctypes.byref(n), ctypes.byref(s)),
                    "get_inliers")
        return n.value, s.value, idx[: n.value].copy()

    def nonminimal(self, idx):
        """Estimator::EstimateModelNonMinimalSample on the listed points."""
        i = np.ascontiguousarray(idx, dtype=np.int32)
        out = np.zeros(9, dtype=np.float32)
        self._check(lib().usac_nonminimal(self._h, _ptr(i, ctypes.c_int32), i.size, _ptr(out, ctypes.c_float)),
                    "nonminimal")
        return out

    def lsq_fit(self, idx, weights=None):
        """usac_lsq_fit: EstimateModelNonMinimalSample(sample, n[, weights], model) -- weights (one
        float per point of the context, by point index) select the weighted overload
        (estimator.hpp:26; homography and fundamental)."""
        i = np.ascontiguousarray(idx, dtype=np.int32)
        out = np.zeros(9, dtype=np.float32)
        wp = None
        if weights is not None:
            w = np.ascontiguousarray(weights, dtype=np.float32)
            if w.size != self.n:
                raise ValueError("weights: one per point (%d), got %d" % (self.n, w.size))
            wp = _ptr(w, ctypes.c_float)
        self._check(lib().usac_lsq_fit(self._h, _ptr(i, ctypes.c_int32), i.size, wp, _ptr(out, ctypes.c_float)),
                    "lsq_fit")
        return out

    def hypothesize_score(self, B=None, samples=None, seed=0, first_hyp=0, thr=2.0, per_hypothesis=True):
        """Fused sample + solve + score (+ batch best).  samples=None -> device sampler.
        Per-model outputs have B * spk entries (slot 3b + j = j-th valid model of sample b
        for the fundamental solver; count -1 marks an empty slot)."""
        L = lib()
        if samples is not None:
            s = np.ascontiguousarray(samples, dtype=np.int32).reshape(-1, self.m)
            B = s.shape[0]
        else:
            s = None
        c = np.zeros(B * self.spk, dtype=np.int32) if per_hypothesis else None
        sm = np.zeros(B * self.spk, dtype=np.float32) if per_hypothesis else None
        best = Record()
        self._check(L.usac_hypothesize_score(self._h, _ptr(s, ctypes.c_int32), B, seed, first_hyp,
                                             ctypes.c_float(thr), _ptr(c, ctypes.c_int32), _ptr(sm, ctypes.c_float),
                                             ctypes.byref(best)), "hypothesize_score")
        return c, sm, best.as_dict()

    def set_sprt(self, enable, seed=1, epsilon=0.0, delta=0.0):
        """Batch SPRT verification for the throughput entry points (reference defaults when
        epsilon / delta are 0)."""
        self._check(lib().usac_set_sprt(self._h, 1 if enable else 0, seed, epsilon, delta), "set_sprt")

    def set_device_sampler(self, sampler):
        """Sampler of the throughput batches' device stream: SAMPLER.Uniform, SAMPLER.Prosac
        (the reference's PROSAC subset schedule; points sorted by quality) or SAMPLER.Napsac
        (grid neighbours built on the device, cell size of set_cell_size)."""
        self._check(lib().usac_set_device_sampler(self._h, int(sampler)), "set_device_sampler")

    def set_cell_size(self, cell_size):
        """Grid cell of the device NAPSAC sampler (model.hpp:43, default 50)."""
        self._check(lib().usac_set_cell_size(self._h, int(cell_size)), "set_cell_size")

    def grid_neighbors(self, cell_size):
        """NearestNeighbors::getGridNearestNeighbors on the device -> dict of the CSR: cell, rank,
        start (n_cells + 1), members, and eligible (points with >= m neighbours)."""
        n = self.n
        nc, ne = ctypes.c_uint32(0), ctypes.c_uint32(0)
        cell = np.zeros(n, dtype=np.uint32)
        rank = np.zeros(n, dtype=np.uint32)
        start = np.zeros(n + 1, dtype=np.uint32)
        members = np.zeros(n, dtype=np.int32)
        elig = np.zeros(n, dtype=np.int32)
        u32 = ctypes.c_uint32
        self._check(lib().usac_grid_neighbors(self._h, int(cell_size), ctypes.byref(nc), _ptr(cell, u32),
                                              _ptr(rank, u32), _ptr(start, u32), _ptr(members, ctypes.c_int32),
                                              _ptr(elig, ctypes.c_int32), ctypes.byref(ne)), "grid_neighbors")
        return {"cell": cell, "rank": rank, "start": start[: nc.value + 1].copy(), "members": members,
                "eligible": elig[: ne.value].copy()}

    def draw_samples(self, B, seed, first_hyp=0):
        """The device stream's samples for hypotheses first_hyp .. first_hyp + B - 1 (B x m)."""
        out = np.zeros((B, self.m), dtype=np.int32)
        self._check(lib().usac_draw_samples(self._h, B, seed, first_hyp, out.ctypes.data_as(ctypes.c_void_p)),
                    "draw_samples")
        return out

    def batch_sprt_info(self, n_slots=0):
        """The batch SPRT's (epsilon, delta, A) and each slot's first pool position in the last batch."""
        eda = np.zeros(3, dtype=np.float64)
        st = np.zeros(max(n_slots, 1), dtype=np.uint32)
        self._check(lib().usac_batch_sprt_info(self._h, _ptr(eda, ctypes.c_double),
                                               _ptr(st, ctypes.c_uint32) if n_slots else None, n_slots),
                    "batch_sprt_info")
        return tuple(float(x) for x in eda), st[:n_slots]

    def sprt_tested(self):
        t = ctypes.c_uint64(0)
        self._check(lib().usac_sprt_tested(self._h, ctypes.byref(t)), "sprt_tested")
        return int(t.value)

    def hypothesize_async(self, B, seed, first_hyp, thr):
        self._check(lib().usac_hypothesize_async(self._h, B, seed, first_hyp, ctypes.c_float(thr)),
                    "hypothesize_async")

    def fetch_best(self):
        r = Record()
        self._check(lib().usac_fetch_best(self._h, ctypes.byref(r)), "fetch_best")
        return r

    def sync(self):
        self._check(lib().usac_sync(self._h), "sync")

    def set_timing(self, on):
        """usac_set_timing (ABI 14): record the batches' HIP events (default) or not."""
        self._check(lib().usac_set_timing(self._h, 1 if on else 0), "set_timing")

    def last_timings(self):
        ms = np.zeros(3, dtype=np.float32)
        self._check(lib().usac_last_timings(self._h, _ptr(ms, ctypes.c_float)), "last_timings")
        return {"batch_ms": float(ms[0]), "score_ms": float(ms[1]), "solve_ms": float(ms[2])}

    # ---- multi-GPU
    @staticmethod
    def comm_unique_id():
        buf = (ctypes.c_uint8 * 128)()
        rc = lib().usac_comm_unique_id(buf)
        if rc:
            raise UsacError(rc, "usac_comm_unique_id")
        return bytes(buf)

    def comm_init(self, nranks, rank, uid):
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        self._check(lib().usac_comm_init(self._h, nranks, rank, buf), "comm_init")
        self.nranks = nranks

    def comm_count(self):
        """(nranks, rank, device) as RCCL reports them for this context's communicator."""
        v = np.zeros(3, dtype=np.int32)
        p = [v[i:].ctypes.data_as(ctypes.POINTER(ctypes.c_int32)) for i in range(3)]
        self._check(lib().usac_comm_count(self._h, *p), "comm_count")
        return int(v[0]), int(v[1]), int(v[2])

    def allgather_record(self, rec):
        allr = (Record * self.nranks)()
        self._check(lib().usac_allgather_records(self._h, ctypes.byref(rec), allr), "allgather_records")
        return list(allr)

    XRING = 8  # USAC_XRING

    def exchange_best_async(self, batch_ctx, slot):
        """All-gather the batch best that hypothesize_async left on batch_ctx (same device) over
        this context's communicator, on its exchange stream, after batch_ctx's stream (no host
        staging, no wait on any compute stream); slot < XRING names it for exchange_best_wait."""
        self._check(lib().usac_exchange_best_async(self._h, batch_ctx._h, slot), "exchange_best_async")

    def exchange_best_wait(self, slot):
        allr = (Record * self.nranks)()
        self._check(lib().usac_exchange_best_wait(self._h, slot, allr), "exchange_best_wait")
        return list(allr)


def record_better(a, b):
    """usac_merge_records' order in Python (usac_api.cpp rec_better): a valid record beats an invalid
    one, then more inliers, then the larger Σ score (Score::bigger), then the earlier hypothesis."""
    if not a.valid:
        return False
    if not b.valid:
        return True
    if a.inliers != b.inliers:
        return a.inliers > b.inliers
    if a.score != b.score:
        return a.score > b.score
    return a.hyp_index < b.hyp_index


def merge_records(records):
    """Score::bigger over records, earliest hyp_index on exact ties."""
    arr = (Record * len(records))(*records)
    out = Record()
    rc = lib().usac_merge_records(arr, len(records), ctypes.byref(out))
    if rc:
        raise UsacError(rc, "usac_merge_records")
    return out


# --------------------------------------------------------------------------- plugin API
class Score:
    """usac/quality/quality.hpp:16-37"""

    def __init__(self, inlier_number=0, score=0.0):
        self.inlier_number = int(inlier_number)
        self.score = float(np.float32(score))

    def bigger(self, other):
        if self.inlier_number > other.inlier_number:
            return True
        if self.inlier_number == other.inlier_number:
            return self.score > other.score
        return False


class Model:
    """usac/model.hpp:15-139 (fields and setters the ported loop reads)."""

    def __init__(self, threshold, sample_number, desired_prob, knn, estimator, sampler):
        self.threshold = float(threshold)
        self.sample_size = int(sample_number)
        self.desired_prob = float(desired_prob)
        self.k_nearest_neighbors = int(knn)
        self.estimator = ESTIMATOR(estimator)
        self.sampler = SAMPLER(sampler)
        self.max_iterations = 10000
        self.min_iterations = 20
        self.reset_random_generator = True
        self.sprt = False
        self.lo = 0
        self.seed = 0
        self.dlt_mode = DLT.THIN
        self.batch = 0
        self.device = 0
        self.lo = LocOpt.NullLO
        self.lo_sample_size = 14
        self.lo_iterative_iterations = 4
        self.lo_inner_iterations = 20
        self.lo_threshold_multiplier = 10
        self.cell_size = 50
        self.neighborsType = NeighborsSearch.NullN
        self.spatial_coherence_gc = 0.1
        self.max_hypothesis_test_before_sprt = 20  # model.hpp:40

    def ResetRandomGenerator(self, reset):
        self.reset_random_generator = bool(reset)

    def setSeed(self, seed):
        """Seed of the glibc sampler stream (srandom(seed)); replaces srand(time(NULL))."""
        self.seed = int(seed)

    def setThreshold(self, thr):
        self.threshold = float(thr)

    def setDesiredProbability(self, p):
        self.desired_prob = float(p)

    def setSprt(self, sprt):
        self.sprt = bool(sprt)

    def setLOParametres(self, lo_iterative_iters, lo_inner_iters, lo_thresh_mult):
        self.lo_iterative_iterations = int(lo_iterative_iters)
        self.lo_inner_iterations = int(lo_inner_iters)
        self.lo_threshold_multiplier = int(lo_thresh_mult)

    def setCellSize(self, cell_size):
        self.cell_size = int(cell_size)

    def setNeighborsType(self, t):
        self.neighborsType = NeighborsSearch(t)

    def setDLTMode(self, mode):
        self.dlt_mode = DLT(mode)


class RansacOutput:
    """usac/ransac/ransac_output.hpp:11-99 getters."""

    def __init__(self, model, inliers, time_us, n_inliers, iters, raw, lo_iters=0):
        self._model = model
        self._inliers = inliers
        self._time = time_us
        self._n = n_inliers
        self._iters = iters
        self.raw = raw
        self._lo = lo_iters

    def getModel(self):
        return self._model

    def getInliers(self):
        return self._inliers

    def getTimeMicroSeconds(self):
        return self._time

    def getNumberOfInliers(self):
        return self._n

    def getNumberOfMainIterations(self):
        return self._iters

    def getLOIters(self):
        return self._lo


def _params(m):
    """usac_params of a Model (the fields the device loop and the plugins read)."""
    seed = m.seed
    if m.reset_random_generator and seed == 0:
        seed = int.from_bytes(os.urandom(4), "little") or 1
    return _Params(m.threshold, m.desired_prob, m.max_iterations, seed, int(m.dlt_mode), m.batch, int(m.sampler),
                   1 if m.sprt else 0, int(m.lo), m.lo_sample_size, m.lo_iterative_iterations,
                   m.lo_inner_iterations, m.lo_threshold_multiplier, m.cell_size, int(m.neighborsType),
                   m.k_nearest_neighbors, m.spatial_coherence_gc, m.max_hypothesis_test_before_sprt)


# usac_allgather_fn (include/usac_gpu.h)
_ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p)


class Ransac:
    """usac/ransac/ransac.hpp:41-115 -- Ransac(model, points); run(); getRansacOutput()."""

    def __init__(self, model, points, ctx=None):
        """ctx: an existing Context over the same points to run on (e.g. the one holding the RCCL
        communicator of a sharded run); by default a new one."""
        if model.sampler not in (SAMPLER.Uniform, SAMPLER.Prosac, SAMPLER.Napsac):
            raise NotImplementedError("sampler %s is not supported (Uniform, Napsac, Prosac)" % model.sampler.name)
        if int(model.lo) not in (0, 1, 2, 3):
            raise NotImplementedError("LO %r is not supported (InItLORsc, InItFLORsc, GC)" % model.lo)
        self.model = model
        self.ctx = ctx if ctx is not None else Context(model.estimator, points, device=model.device)
        self._out = None
        self.records = []

    def run(self, rec_cap=4096, shard=None):
        """shard = (nranks, rank, gather): hypothesis-sharded batches (usac_ransac_run_sharded);
        gather(bytes) -> list of nranks bytes objects in rank order (e.g. a gloo all_gather), or
        gather = "rccl" for the communicator set up with Context.comm_init."""
        L = lib()
        p = _params(self.model)
        out = _RunOutput()
        inl = np.empty(self.ctx.n, dtype=np.int32)
        # the record array is the run's largest host allocation (rec_cap x 56 B, zero-filled): one
        # per Context and capacity, reused (the records are copied out below)
        cache = self.ctx.__dict__.setdefault("_rec_bufs", {})
        recs = cache.get(rec_cap)
        if recs is None:
            recs = cache[rec_cap] = (Record * rec_cap)()
        if shard is None:
            rc = L.usac_ransac_run(self.ctx._h, ctypes.byref(p), ctypes.byref(out), _ptr(inl, ctypes.c_int32), recs,
                                   rec_cap)
        else:
            nranks, rank, gather = shard
            cb = None
            if gather != "rccl":
                def _cb(user, send, nbytes, recv):
                    try:
                        parts = gather(ctypes.string_at(send, nbytes))
                        buf = b"".join(parts)
                        if len(parts) != nranks or len(buf) != nranks * nbytes:
                            return -1
                        ctypes.memmove(recv, buf, len(buf))
                        return 0
                    except Exception:  # reported as a failed all-gather (usac_last_error)
                        return -1
                cb = _ALLGATHER_FN(_cb)
            rc = L.usac_ransac_run_sharded(self.ctx._h, ctypes.byref(p), int(nranks), int(rank),
                                           ctypes.cast(cb, _vp) if cb is not None else None, None,
                                           ctypes.byref(out), _ptr(inl, ctypes.c_int32), recs, rec_cap)
        if rc == -111:
            raise UsacError(rc, "best score is 0 (ransac.cpp:143-147)")
        self.ctx._check(rc, "ransac_run")
        k = min(out.n_records, rec_cap)
        self.records = [(int(recs[i].hyp_index), int(recs[i].inliers), float(recs[i].score)) for i in range(k)]
        raw = {"minimal_model": np.array(out.minimal_model[:], dtype=np.float32),
               "minimal_inliers": out.minimal_inliers, "polish_passes": out.polish_passes,
               "n_records": out.n_records, "batches": out.batches, "sprt_rejected": out.sprt_rejected,
               "sprt_histories": out.sprt_histories, "prosac_term_len": out.prosac_term_len,
               "rollbacks": out.rollbacks, "lo_iterative_iters": out.lo_iterative_iters,
               "lo_rounds": out.lo_rounds, "lo_stages": out.lo_stages, "sum_models": out.sum_models,
               "lo_fits": out.lo_fits, "spec_batches": out.spec_batches, "spec_rollbacks": out.spec_rollbacks,
               "spec_wasted": out.spec_wasted}
        self._out = RansacOutput(np.array(out.model[:], dtype=np.float32), inl[: out.inliers].copy(), out.time_us,
                                 out.inliers, out.iters, raw, out.lo_inner_iters)

    def getRansacOutput(self):
        return self._out


# --------------------------------------------------------------------------- stateful plugins
# The reference's per-call plugin surface (include/usac_gpu.h, ABI 11): a caller that keeps its own
# Ransac::run loop (ransac.cpp:58-139) swaps plugin by plugin.  Every handle created on a Context
# must be closed before it (close(), or garbage collection in creation-reverse order).
class _Handle:
    _destroy = None

    def close(self):
        h = getattr(self, "_h", None)
        if h:
            getattr(lib(), self._destroy)(h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class RandomGenerator(_Handle):
    """The reference's global glibc random() stream after srandom(seed) (usac_random)."""
    _destroy = "usac_random_destroy"

    def __init__(self, seed):
        h = _vp()
        rc = lib().usac_random_create(int(seed), ctypes.byref(h))
        if rc:
            raise UsacError(rc, "usac_random_create")
        self._h = h

    def next(self):
        return int(lib().usac_random_next(self._h))


class Sampler(_Handle):
    """Sampler::generateSample (sampler.hpp:11-35) as initSampler builds it for model.sampler: Uniform
    (persistent pool on rng), Prosac (own mt19937 seeded with model.seed), Napsac (grid or KNN
    neighbours built on the device, on rng)."""
    _destroy = "usac_sampler_destroy"

    def __init__(self, ctx, model, rng=None):
        h = _vp()
        self.ctx, self.rng = ctx, rng  # kept alive while the handle draws from them
        self._p = _params(model)
        ctx._check(lib().usac_sampler_create(ctx._h, ctypes.byref(self._p), rng._h if rng is not None else None,
                                             ctypes.byref(h)), "sampler_create")
        self._h = h
        self.m = ctx.m
        self._sample = np.zeros(self.m, dtype=np.int32)  # the loop's reused `int sample[m]`

    def generateSample(self):
        self.ctx._check(lib().usac_sampler_generate(self._h, _ptr(self._sample, ctypes.c_int32)), "generateSample")
        return self._sample.copy()

    def generateSamples(self, count):
        out = np.zeros((int(count), self.m), dtype=np.int32)
        self.ctx._check(lib().usac_sampler_generate_batch(self._h, int(count), _ptr(out, ctypes.c_int32)),
                        "generateSamples")
        return out

    def state(self):
        d, sub, lg = ctypes.c_uint64(0), ctypes.c_uint32(0), ctypes.c_uint32(0)
        self.ctx._check(lib().usac_sampler_state(self._h, ctypes.byref(d), ctypes.byref(sub), ctypes.byref(lg)),
                        "sampler_state")
        return {"drawn": int(d.value), "subset_size": int(sub.value), "largest_sample_size": int(lg.value)}


class TerminationCriteria(_Handle):
    """StandardTerminationCriteria, or ProsacTerminationCriteria when built on a Prosac Sampler
    (linked both ways as in the reference)."""
    _destroy = "usac_termination_destroy"

    def __init__(self, ctx, model, prosac_sampler=None):
        h = _vp()
        self.ctx, self.sampler = ctx, prosac_sampler
        self._p = _params(model)
        ctx._check(lib().usac_termination_create(ctx._h, ctypes.byref(self._p),
                                                 prosac_sampler._h if prosac_sampler is not None else None,
                                                 ctypes.byref(h)), "termination_create")
        self._h = h
        self.termination_length = ctx.n

    def getUpBoundIterations(self, a, b=None):
        """(inlier_size[, points_size]) -> standard bound; (hypCount, model array) -> PROSAC's
        getUpBoundIterations(hypCount, model) (prosac_termination_criteria.hpp:148-201)."""
        if b is None or np.ndim(b) == 0:
            return int(lib().usac_termination_bound(self._h, int(a), int(b or 0)))
        m = np.zeros(9, dtype=np.float32)
        mm = np.asarray(b, dtype=np.float32).reshape(-1)
        m[: mm.size] = mm
        mi, tl = ctypes.c_uint32(0), ctypes.c_uint32(0)
        self.ctx._check(lib().usac_prosac_termination(self._h, int(a), _ptr(m, ctypes.c_float), ctypes.byref(mi),
                                                      ctypes.byref(tl)), "prosac_termination")
        self.termination_length = int(tl.value)
        return int(mi.value)


class SPRT(_Handle):
    """SPRT (sprt.hpp:89-491): pool shuffled from rng at construction, verifyModelAndGetModelScore,
    getUpperBoundIterations, and the batch replay of the loop body (usac_sprt_replay)."""
    _destroy = "usac_sprt_destroy"

    def __init__(self, ctx, model, rng):
        h = _vp()
        self.ctx, self.rng = ctx, rng
        self._p = _params(model)
        ctx._check(lib().usac_sprt_create(ctx._h, ctypes.byref(self._p), rng._h, ctypes.byref(h)), "sprt_create")
        self._h = h

    def verifyModelAndGetModelScore(self, model, current_hypothese, maximum_score, score):
        m = np.zeros(9, dtype=np.float32)
        mm = np.asarray(model, dtype=np.float32).reshape(-1)
        m[: mm.size] = mm
        good = ctypes.c_int32(0)
        cnt = ctypes.c_int32(score.inlier_number)
        sc = ctypes.c_float(score.score)
        self.ctx._check(lib().usac_sprt_verify(self._h, _ptr(m, ctypes.c_float), int(current_hypothese),
                                               int(maximum_score), ctypes.byref(good), ctypes.byref(cnt),
                                               ctypes.byref(sc)), "sprt_verify")
        score.inlier_number, score.score = int(cnt.value), float(sc.value)
        return bool(good.value)

    def getUpperBoundIterations(self, inlier_size):
        return int(lib().usac_sprt_upper_bound(self._h, int(inlier_size)))

    def stats(self):
        h, r = ctypes.c_uint32(0), ctypes.c_uint32(0)
        self.ctx._check(lib().usac_sprt_stats(self._h, ctypes.byref(h), ctypes.byref(r)), "sprt_stats")
        return {"histories": int(h.value), "rejected": int(r.value)}

    def replay(self, models, n_models, state):
        """usac_sprt_replay over a batch (models B x slots x 9, n_models[B]); `state` a SprtState,
        updated in place; returns state.found."""
        m = np.ascontiguousarray(models, dtype=np.float32)
        nm = np.ascontiguousarray(n_models, dtype=np.int32)
        self.ctx._check(lib().usac_sprt_replay(self._h, _ptr(m, ctypes.c_float), _ptr(nm, ctypes.c_int32), len(nm),
                                               ctypes.byref(state)), "sprt_replay")
        return bool(state.found)


class LocalOptimization(_Handle):
    """LocalOptimization::GetModelScore (local_optimization.hpp:19) as initLocalOptimization builds it
    for model.lo: InItLORsc / InItFLORsc (inner + iterative LO-RANSAC) or GC (graph cut)."""
    _destroy = "usac_lo_destroy"

    def __init__(self, ctx, model):
        h = _vp()
        self.ctx = ctx
        self._p = _params(model)
        ctx._check(lib().usac_lo_create(ctx._h, ctypes.byref(self._p), ctypes.byref(h)), "lo_create")
        self._h = h

    def GetModelScore(self, best_model, best_score):
        """best_model: float32 array of 9 (line: 3) improved in place; best_score: a Score."""
        m = np.zeros(9, dtype=np.float32)
        m[: best_model.size] = best_model.reshape(-1)
        cnt = ctypes.c_int32(best_score.inlier_number)
        sc = ctypes.c_float(best_score.score)
        self.ctx._check(lib().usac_lo_get_model_score(self._h, _ptr(m, ctypes.c_float), ctypes.byref(cnt),
                                                      ctypes.byref(sc)), "lo_get_model_score")
        best_model.reshape(-1)[:] = m[: best_model.size]
        best_score.inlier_number, best_score.score = int(cnt.value), float(sc.value)

    def iters(self):
        a, b = ctypes.c_uint32(0), ctypes.c_uint32(0)
        self.ctx._check(lib().usac_lo_iters(self._h, ctypes.byref(a), ctypes.byref(b)), "lo_iters")
        return int(a.value), int(b.value)
