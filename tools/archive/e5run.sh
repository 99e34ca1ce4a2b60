#!/bin/bash
# quick GPU round: GPU tests, essential/fundamental bench lines, one unpipelined kernel trace
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --estimator essential --steps 5 --warmup 2 --cpu-seconds 0 $BE_ARGS > gpurun_out/be.log 2>&1 || exit 2
timeout -k 10 200 python bench.py --estimator fundamental --steps 5 --warmup 2 --cpu-seconds 0 $BF_ARGS > gpurun_out/bf.log 2>&1 || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/profe4 -o p --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --estimator essential --steps 3 --warmup 1 --pipeline 1 --cpu-seconds 0 $BE_ARGS > $GRAFT_REPO_ROOT/gpurun_out/bep.log 2>&1 || exit 4
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/proff4 -o p --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --estimator fundamental --steps 3 --warmup 1 --pipeline 1 --cpu-seconds 0 $BF_ARGS > $GRAFT_REPO_ROOT/gpurun_out/bfp.log 2>&1 || exit 5
