"""RCCL path of the multi-GPU bench on the real device: a single-rank communicator
(usac_comm_unique_id -> usac_comm_init -> usac_allgather_records) returns the record it was
given, byte for byte.  (N > 1 needs one GPU per rank; the merge logic across ranks is covered
by tests/test_distributed.py with gloo.)"""
import ctypes

import numpy as np
import pytest

from ransac_amd import synthetic

pytestmark = pytest.mark.gpu


def test_single_rank_rccl_allgather(usac):
    pts, _, _ = synthetic.homography_points(n=1000, inlier_ratio=0.3, seed=2)
    with usac.Context(usac.ESTIMATOR.Homography, pts, device=0) as ctx:
        uid = usac.Context.comm_unique_id()
        ctx.comm_init(1, 0, uid)
        ctx.hypothesize_async(4096, 3, 0, 2.0)
        best = ctx.fetch_best()
        got = ctx.allgather_record(best)
        assert len(got) == 1 and bytes(got[0]) == bytes(best)
        assert usac.merge_records(got).hyp_index == best.hyp_index


def test_exchange_ring_matches_batch_records(usac):
    """usac_exchange_best_async / _wait (the bench's N > 1 exchange, off the compute streams):
    with three contexts in flight and a one-rank communicator, every batch's exchanged record is
    the record that batch produced (same device RNG stream run one batch at a time), and the
    ring slots are reused across more exchanges than it holds."""
    pts, _, _ = synthetic.homography_points(n=2000, inlier_ratio=0.3, seed=4)
    B, nb, P = 8192, 3 * usac.Context.XRING + 2, 3
    ref = []
    with usac.Context(usac.ESTIMATOR.Homography, pts, device=0) as c:
        for i in range(nb):
            c.hypothesize_async(B, 5, i * B, 2.0)
            ref.append(bytes(c.fetch_best()))
    ctxs = [usac.Context(usac.ESTIMATOR.Homography, pts, device=0) for _ in range(P)]
    try:
        ctx = ctxs[0]
        ctx.comm_init(1, 0, usac.Context.comm_unique_id())
        got = []
        for i in range(nb):
            ctxs[i % P].hypothesize_async(B, 5, i * B, 2.0)
            ctx.exchange_best_async(ctxs[i % P], i % usac.Context.XRING)
            if i >= P - 1:
                j = i - P + 1
                got.append(ctx.exchange_best_wait(j % usac.Context.XRING))
        for j in range(nb - P + 1, nb):
            got.append(ctx.exchange_best_wait(j % usac.Context.XRING))
        assert [len(g) for g in got] == [1] * nb
        assert [bytes(g[0]) for g in got] == ref
    finally:
        for c in ctxs:
            c.close()
