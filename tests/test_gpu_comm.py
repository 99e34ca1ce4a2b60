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
