"""bench.py's parity plumbing for N > 1 lines, CPU only: the oracle's best
update over a batch (Score::bigger, earliest hypothesis on ties -- ransac.cpp:103-132), the
multi-threaded oracle equal to the single-threaded one, the first timed batch's merged record
checked against the union of all ranks' samples redrawn from (seed, global index), the ranks'
records merged (usac_merge_records, host-only) and compared with the exchange's list, and the RCCL
rank report's refusal."""
import sys

import numpy as np
import pytest

from tests.conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402
from ransac_amd import synthetic  # noqa: E402


def test_oracle_best_is_score_bigger_earliest():
    c = np.array([3, 7, 7, 7, -1, 2])
    s = np.array([1.0, 5.0, 6.0, 6.0, 0.0, 9.0], np.float32)
    occ = c >= 0
    assert bench.oracle_best(c, s, occ) == 2  # most inliers, then the larger score, then the earliest
    assert bench.oracle_best(c, s, np.zeros(6, bool)) is None


@pytest.mark.parametrize("kind", ["homography", "fundamental"])
def test_oracle_batch_threads_equal_one_thread(oracle, kind):
    if kind == "fundamental":
        pts, _, _ = synthetic.fundamental_points(n=1500, inlier_ratio=0.3, seed=4)
        m = 7
    else:
        pts, _, _ = synthetic.homography_points(n=1500, inlier_ratio=0.3, seed=4)
        m = 4
    smp = oracle.uniform_samples(9, len(pts), m, 96)
    one = bench.oracle_batch(kind, pts, 2.0, 0, smp)
    many = bench.oracle_batch_mt(kind, pts, 2.0, 0, smp, 5)
    for a, b in zip(one, many):
        assert a.shape == b.shape and (a.view(np.int32) == b.view(np.int32)).all()


class _FakeCtx:
    """draw_samples keyed by (seed, global index), as the device samplers are."""

    def __init__(self, oracle, n, m):
        self.O, self.n, self.m = oracle, n, m

    def draw_samples(self, B, seed, first):
        return self.O.uniform_samples(seed * 100003 + first, self.n, self.m, B)


def test_first_batch_parity_union_of_ranks(oracle, usac):
    pts, _, _ = synthetic.homography_points(n=1200, inlier_ratio=0.3, seed=6)
    ctx = _FakeCtx(oracle, len(pts), 4)
    B, world, step, seed = 64, 3, 2, 5
    firsts = [(step * world + r) * B for r in range(world)]
    smp = np.concatenate([ctx.draw_samples(B, seed, f) for f in firsts])
    oc, osum, occ = bench.oracle_batch("homography", pts, 2.0, 0, smp)
    k = bench.oracle_best(oc, osum, occ)
    right = usac.Record(hyp_index=firsts[k // B] + k % B, inliers=int(oc[k]), score=float(osum[k]), valid=1)
    out = bench.first_batch_parity(usac, ctx, "homography", pts, 2.0, 0, seed, B, step, world, right, 4)
    assert out["ok"] and out["hypotheses"] == world * B and out["oracle_best"]["hyp_index"] == right.hyp_index
    wrong = usac.Record(hyp_index=right.hyp_index + 1, inliers=right.inliers, score=right.score, valid=1)
    assert not bench.first_batch_parity(usac, ctx, "homography", pts, 2.0, 0, seed, B, step, world, wrong, 4)["ok"]


def _tk(rec, exp, ok=True, sprt=True, exchanged=None):
    d = {"ok": ok, "record": rec, "expected_record": exp}
    if sprt:
        d["sprt_accepted"] = 10
    if exchanged is not None:
        d["exchanged"] = exchanged
    return d


def test_ranks_parity_merge_and_exchange(usac):
    recs = [{"inliers": 40, "hyp_index": 7}, {"inliers": 55, "hyp_index": 300}, {"inliers": 55, "hyp_index": 600}]
    tk = [_tk(r, dict(r), exchanged=list(recs)) for r in recs]
    out = bench.ranks_parity(usac, tk, "rccl_allgather")
    assert out["ok"] and out["merge_equal"] and out["exchange_equal"]
    assert out["expected_merge"] == {"inliers": 55, "hyp_index": 300}
    # a rank whose slice failed, or an exchange that returned something else, fails the line
    tk[2]["ok"] = False
    assert not bench.ranks_parity(usac, tk, "rccl_allgather")["ok"]
    tk[2]["ok"] = True
    tk[1]["exchanged"] = [recs[0], recs[0], recs[2]]
    assert not bench.ranks_parity(usac, tk, "rccl_allgather")["ok"]
    # the one-GPU gloo rehearsal has no exchange list to compare; non-SPRT lines leave the merge to
    # first_batch_parity (the records' Σ are the fast kernel's)
    plain = [_tk(r, dict(r), sprt=False) for r in recs]
    out = bench.ranks_parity(usac, plain, "gloo_allgather")
    assert out["ok"] and "merge_equal" not in out and "exchange_equal" not in out


def test_rccl_report_without_rccl():
    assert bench.rccl_report(None, "gloo_allgather", None, 2, 0) is None
    assert bench.rccl_report(None, "none", None, 1, 0) is None


class _FakeCommCtx:
    def __init__(self, n, r, dev):
        self.v = (n, r, dev)

    def comm_count(self):
        return self.v


class _FakeDist:
    def __init__(self, allv):
        self.allv = allv

    def all_gather_object(self, out, obj):
        out[:] = self.allv


def test_rccl_report_refuses_a_short_communicator():
    ok = bench.rccl_report(_FakeCommCtx(2, 0, 0), "rccl_allgather", _FakeDist([(2, 0, 0), (2, 1, 1)]), 2, 0)
    assert ok["ranks"] == 2 and ok["devices"] == [0, 1]
    with pytest.raises(SystemExit) as e:  # RCCL saw one rank of two
        bench.rccl_report(_FakeCommCtx(1, 0, 0), "rccl_allgather", _FakeDist([(1, 0, 0), (1, 0, 1)]), 2, 0)
    assert e.value.code == 4
    with pytest.raises(SystemExit):  # two ranks on one device
        bench.rccl_report(_FakeCommCtx(2, 0, 0), "rccl_allgather", _FakeDist([(2, 0, 0), (2, 1, 0)]), 2, 0)


def test_cfg5_roofline_prices_a_kernel_its_runs_execute():
    """the cfg5 line's roofline comes from the committed trace + PMC summary of
    `bench.py --cfg5` itself (tools/profile_round.sh cfg5: workload batch 0, every dispatch of the
    profiled runs), so the kernel it names is one those runs executed -- not the throughput batches'
    matrix-core scorer, which usac_ransac_run does not use."""
    import glob
    import json
    import os

    r = bench.run_roofline(100000, 3.5)
    assert r is not None, "no committed cfg5 summary (profiles/r*_summary.json, workload batch 0)"
    src = json.load(open(os.path.join(ROOT, r["source"])))
    assert src["workload"]["batch"] == 0 and src["workload"]["runs"] > 0
    traced = {bench._kname_key(k) for k in src["kernels"]}
    assert any(bench._kname_key(form % r["kernel"]) in traced for form in ("void usac::%s(", "usac::%s(")), r["kernel"]
    assert "k_score_h16" not in r["kernel"]
    assert 0.0 < r["frac"] <= 1.0 and r["kernels_by_device_time"][0]["kernel"] == r["kernel"]
    # the summary's calls per run follow from its dispatch counts
    for row in r["kernels_by_device_time"]:
        assert row["calls_per_run"] > 0 and row["device_us_per_run"] > 0
    assert glob.glob(os.path.join(ROOT, "profiles", "r*_cfg5_summary.json"))


def test_record_better_equals_merge_records(usac):
    """bench.py keeps the timed batches' best with usac.record_better (no ctypes round trip per
    step); it must order records exactly as the library's usac_merge_records (host-only code)."""
    rng = np.random.default_rng(4)
    recs = []
    for _ in range(400):
        r = usac.Record()
        r.hyp_index = int(rng.integers(0, 50))
        r.inliers = int(rng.integers(-1, 4))
        r.score = float(np.float32(rng.choice([0.5, 1.0, 1.5])))
        r.valid = int(rng.random() < 0.85)
        recs.append(r)
    for a, b in zip(recs[::2], recs[1::2]):
        m = usac.merge_records([b, a])  # b unless a is better
        w = a if usac.record_better(a, b) else b
        assert (m.hyp_index, m.inliers, m.score, m.valid) == (w.hyp_index, w.inliers, w.score, w.valid)
