set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_loop.py tests/test_gpu_baseline_sizes.py tests/test_gpu_polish_fused.py tests/test_gpu_essential.py tests/test_gpu_quality_api.py > gpurun_out/su.log 2>&1 || { tail -30 gpurun_out/su.log; exit 1; }
tail -1 gpurun_out/su.log
for rep in 1 2 3; do
  for lib in ransac_amd/var_libs/lib_base.so ransac_amd/libransac_amd.so; do
    RANSAC_AMD_LIB=$PWD/$lib timeout -k 10 300 python bench.py --sprt-exact --steps 40 --cpu-seconds 0 > gpurun_out/sux.json 2>/dev/null || exit 1
    python3 -c "
import json;d=json.loads(open('gpurun_out/sux.json').read().strip().splitlines()[-1]);print('$lib', 'exact', round(d['ms_per_step'],4), d['run_stats']['library_ms_per_run'], all(d['parity'].values()))"
  done
done
