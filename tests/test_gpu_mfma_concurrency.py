"""Exact recounts beside matrix-core batches.

Round 5's loop saw its exact recount (k_inl_flags: quality.hpp:60-101) miscount while a k_score_h16
batch ran on another stream.  tools/h16_race.cpp and tools/mfma_interference.cpp pinned the cause:
on gfx950 packed fp32 VALU instructions (v_pk_fma/mul/add_f32, which the compiler's SLP vectoriser
had put into the recount) return wrong values in lanes 48-63 while another kernel's waves execute
MFMAs on the same CU (profiles/r6/mfma_interference.log); no other VALU class is affected.  The
library now issues no packed fp32 instruction (usac_pk.hpp; tests/test_no_packed_fp32.py checks the
built code objects).  Here: exact recounts through the C-ABI on one context while another context's
matrix-core batches (h16, e16) are in flight on their own stream -- every count, Σ and inlier list
equal to the same recount run alone."""
import numpy as np
import pytest

from ransac_amd import synthetic

pytestmark = pytest.mark.gpu


def _perturbed(M, rng, k, scale):
    base = M.reshape(9).astype(np.float64)
    return [(base * (1 + scale * rng.standard_normal(9))).astype(np.float32) for _ in range(k)]


@pytest.mark.parametrize("kind", ["H", "E"])
def test_exact_recount_beside_matrix_core_batches(usac, kind, monkeypatch):
    monkeypatch.setenv("USAC_E16", "1")  # the essential matrix-core scorer (the default), pinned on
    rng = np.random.default_rng(3)
    if kind == "H":
        pts, M, _ = synthetic.homography_points(n=20000, inlier_ratio=0.3, seed=12)
        est, thr, B, scale = usac.ESTIMATOR.Homography, 2.0, 262144, 1e-3
    else:
        pts, M, _ = synthetic.fundamental_points(n=50000, inlier_ratio=0.3, seed=12, normalized=True)
        est, thr, B, scale = usac.ESTIMATOR.Essential, 0.002, 65536, 1e-3
    models = _perturbed(M / np.linalg.norm(M), rng, 24, scale)
    with usac.Context(est, pts) as busy, usac.Context(est, pts) as rc:
        busy.set_score_chunks(8 if kind == "H" else 96)
        quiet = [rc.get_inliers(m, thr) for m in models]
        assert sum(q[0] for q in quiet) > 0
        differ = checked = 0
        for rep in range(8):
            busy.hypothesize_async(B, 7, rep * B, thr)  # in flight on busy's stream
            for m, q in zip(models, quiet):
                c, s, idx = rc.get_inliers(m, thr)
                checked += 1
                differ += int(c != q[0] or np.float32(s) != np.float32(q[1]) or not np.array_equal(idx, q[2]))
            busy.fetch_best()
    assert differ == 0, "%d of %d recounts beside matrix-core batches differ" % (differ, checked)
