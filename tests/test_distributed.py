"""N > 1 path on CPU: hypothesis sharding + the per-batch best-record exchange.

Two gloo ranks each score their own hypothesis index range (bench.py's sharding:
rank r owns [(step*W + r)*B, +B)), build their shard best, all-gather the records and merge
them with the library's usac_merge_records; the merged best must equal the best of a single
process that scored all hypotheses in global order (Score::bigger, earliest index on ties).
Per-hypothesis scores come from the CPU oracle (no GPU here); the exchanged bytes are the
library's usac_record layout.
"""
import ctypes
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scores(B, world, steps):
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    from ransac_amd import synthetic

    pts, _, _ = synthetic.homography_points(n=600, inlier_ratio=0.4, seed=3)
    total = B * world * steps
    samples = O.uniform_samples(5, len(pts), 4, total)
    est = O.Estimator(O.HOMOGRAPHY, pts)
    models, _ = est.estimate_batch(samples)
    c, s = est.score_models(models, 2.0)
    return models, c, s


def _worker(rank, world, port, B, steps, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    import ransac_amd as usac

    dist.init_process_group("gloo", rank=rank, world_size=world)
    models, c, s = _scores(B, world, steps)
    best = None
    for step in range(steps):
        first = (step * world + rank) * B
        idx = np.arange(first, first + B)
        order = sorted(idx.tolist(), key=lambda i: (-c[i], -s[i], i))
        i = order[0]
        rec = usac.Record(i, int(c[i]), float(s[i]), (ctypes.c_float * 9)(*models[i].tolist()), 1)
        buf = torch.frombuffer(bytearray(bytes(rec)), dtype=torch.uint8)
        gathered = [torch.zeros_like(buf) for _ in range(world)]
        dist.all_gather(gathered, buf)
        recs = [usac.Record.from_buffer_copy(bytes(g.numpy().tobytes())) for g in gathered]
        merged = usac.merge_records(recs)
        best = merged if best is None else usac.merge_records([best, merged])
    if rank == 0:
        q.put((int(best.hyp_index), int(best.inliers), float(best.score)))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_best_equals_global_best():
    import multiprocessing as mp

    B, world, steps = 64, 2, 3
    models, c, s = _scores(B, world, steps)
    order = sorted(range(len(c)), key=lambda i: (-c[i], -s[i], i))
    expect = (order[0], int(c[order[0]]), float(s[order[0]]))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, B, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got == expect


def test_shards_are_disjoint_and_cover():
    B, world, steps = 128, 4, 5
    seen = []
    for step in range(steps):
        for rank in range(world):
            first = (step * world + rank) * B
            seen.extend(range(first, first + B))
    assert sorted(seen) == list(range(B * world * steps))
