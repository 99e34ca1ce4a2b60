set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_napsac_lo.py tests/test_gpu_loop.py tests/test_gpu_baseline_sizes.py tests/test_gpu_polish_fused.py tests/test_gpu_graphcut.py tests/test_gpu_seqsum.py > gpurun_out/seg.log 2>&1 || { tail -30 gpurun_out/seg.log; exit 1; }
tail -1 gpurun_out/seg.log
for rep in 1 2; do
  for lib in ransac_amd/var_libs/lib_seg32.so ransac_amd/libransac_amd.so; do
    RANSAC_AMD_LIB=$PWD/$lib timeout -k 10 300 python bench.py --cfg5 --cpu-seconds 0 > gpurun_out/segab.json 2>/dev/null || exit 1
    python3 -c "
import json;d=json.loads(open('gpurun_out/segab.json').read().strip().splitlines()[-1]);print('$lib', round(d['ms_per_step'],4), all(d['parity'].values()) if isinstance(d['parity'],dict) else d['parity'])"
    RANSAC_AMD_LIB=$PWD/$lib timeout -k 10 300 python bench.py --sprt-exact --steps 40 --cpu-seconds 0 > gpurun_out/segab3.json 2>/dev/null || exit 1
    python3 -c "
import json;d=json.loads(open('gpurun_out/segab3.json').read().strip().splitlines()[-1]);print('   cfg3x', round(d['ms_per_step'],4), d['run_stats']['library_ms_per_run'])"
  done
done
