set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fundamental.py tests/test_gpu_baseline_sizes.py tests/test_gpu_loop.py tests/test_gpu_device_sampler.py tests/test_gpu_plugins.py > gpurun_out/bs.log 2>&1 || { tail -30 gpurun_out/bs.log; exit 1; }
tail -1 gpurun_out/bs.log
for rep in 1 2; do
  for lib in ransac_amd/var_libs/lib_base.so ransac_amd/libransac_amd.so; do
    RANSAC_AMD_LIB=$PWD/$lib timeout -k 10 300 python bench.py --sprt-exact --steps 40 --cpu-seconds 0 > gpurun_out/bsx.json 2>/dev/null || exit 1
    RANSAC_AMD_LIB=$PWD/$lib timeout -k 10 300 python bench.py --estimator fundamental --cpu-seconds 0 > gpurun_out/bsb.json 2>/dev/null || exit 1
    python3 -c "
import json;d=json.loads(open('gpurun_out/bsx.json').read().strip().splitlines()[-1]);e=json.loads(open('gpurun_out/bsb.json').read().strip().splitlines()[-1]);print('$lib', 'exact', round(d['ms_per_step'],4), d['run_stats']['library_ms_per_run'], all(d['parity'].values()), 'batch', round(e['value']/1e9,3), e['roofline'].get('solve_kernel_ms'), e['parity'].get('inlier_counts_equal'))"
  done
done
