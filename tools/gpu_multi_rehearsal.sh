#!/bin/bash
# N = 2 rehearsal of bench.py's multi-rank paths on ONE GPU (two ranks share the device; the
# record exchange falls back to gloo there, RCCL refuses two ranks on one device): the
# throughput line and the hypothesis-sharded cfg5 line.  Distinct GPUs use RCCL (driver runs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export USAC_BENCH_SAME_DEVICE=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 30 --warmup 5 > gpurun_out/multi_h.json 2> gpurun_out/multi_h.err || { tail -20 gpurun_out/multi_h.err; exit 1; }
cat gpurun_out/multi_h.json | cut -c1-400
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29518 bench.py --cfg5 --gpus 2 --steps 20 --warmup 2 --cpu-seconds 0 > gpurun_out/multi_cfg5.json 2> gpurun_out/multi_cfg5.err || { tail -20 gpurun_out/multi_cfg5.err; exit 1; }
cat gpurun_out/multi_cfg5.json | cut -c1-600
