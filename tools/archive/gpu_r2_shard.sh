set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sharded_run.py tests/test_gpu_quality_api.py > gpurun_out/t6.log 2>&1; rc=$?; tail -15 gpurun_out/t6.log; [ $rc -eq 0 ] || exit $rc
USAC_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --cfg5 --gpus 2 --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/cfg5_n2.json 2> gpurun_out/cfg5_n2.err; rc=$?; cat gpurun_out/cfg5_n2.json; tail -5 gpurun_out/cfg5_n2.err; exit $rc
