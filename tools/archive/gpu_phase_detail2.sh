set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_loop.py tests/test_gpu_baseline_sizes.py tests/test_gpu_essential.py tests/test_gpu_plugins.py tests/test_gpu_fundamental.py tests/test_gpu_knn.py tests/test_gpu_graphcut.py tests/test_gpu_napsac_lo.py tests/test_gpu_sharded_run.py tests/test_gpu_reference_statistics.py > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
bash tools/gpu_phase_detail.sh
