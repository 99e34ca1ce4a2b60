mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --estimator essential --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/be.log 2>&1 || exit 2
timeout -k 10 200 python bench.py --estimator essential --steps 5 --warmup 2 --cpu-seconds 0 --batch 262144 > gpurun_out/be2.log 2>&1 || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/profe4 -o p --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --estimator essential --steps 3 --warmup 1 --pipeline 1 --cpu-seconds 0 > $GRAFT_REPO_ROOT/gpurun_out/bep.log 2>&1 || exit 4
