"""Child process of tests/test_gpu_sharded_run.py: one rank of a hypothesis-sharded
usac_ransac_run whose per-batch all-gather travels over a torch.distributed gloo group (two
ranks share the one GPU of the test box, which RCCL refuses).  Writes its RansacOutput to
argv[4] (.npz).  Started as a fresh process, never forked from a GPU-initialised one."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    rank, world, port, out_path, case = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5]
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    import ransac_amd as usac
    from test_gpu_sharded_run import make_case

    pts, mdl = make_case(usac, case)

    def gather(b):
        t = torch.frombuffer(bytearray(b), dtype=torch.uint8)
        parts = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        return [p.numpy().tobytes() for p in parts]

    r = usac.Ransac(mdl, pts)
    r.run(shard=(world, rank, gather))
    o = r.getRansacOutput()
    np.savez(out_path, model=o.getModel(), inliers=o.getInliers(), iters=o.getNumberOfMainIterations(),
             lo=o.getLOIters(), records=np.array(r.records, dtype=np.float64).reshape(-1, 3),
             batches=o.raw["batches"], sprt_rejected=o.raw["sprt_rejected"], sprt_histories=o.raw["sprt_histories"], lo_fits=o.raw["lo_fits"], lo_rounds=o.raw["lo_rounds"])
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
