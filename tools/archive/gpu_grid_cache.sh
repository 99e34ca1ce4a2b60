set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_napsac_lo.py tests/test_gpu_graphcut.py tests/test_gpu_plugins.py tests/test_gpu_cpp_consumer.py tests/test_gpu_knn.py tests/test_gpu_loop.py tests/test_gpu_sharded_run.py tests/test_gpu_reference_statistics.py > gpurun_out/gc.log 2>&1 || { tail -30 gpurun_out/gc.log; exit 1; }
tail -1 gpurun_out/gc.log
bash tools/gpu_cfg5_ctx.sh
