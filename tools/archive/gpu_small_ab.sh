set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_loop.py tests/test_gpu_baseline_sizes.py tests/test_gpu_essential.py tests/test_gpu_fundamental.py tests/test_gpu_plugins.py tests/test_gpu_polish_fused.py tests/test_gpu_sharded_run.py tests/test_gpu_knn.py tests/test_gpu_graphcut.py tests/test_gpu_napsac_lo.py tests/test_gpu_quality_api.py tests/test_gpu_reference_statistics.py > gpurun_out/ta.log 2>&1 || { tail -40 gpurun_out/ta.log; exit 1; }
tail -1 gpurun_out/ta.log
for v in 0 1 0 1; do
if [ $v = 1 ]; then export USAC_INLIERS_SMALL=0; else unset USAC_INLIERS_SMALL; fi
timeout -k 10 300 python bench.py --sprt-exact --steps 40 --warmup 5 --cpu-seconds 0 > gpurun_out/tab.json 2>/dev/null || exit 1
python3 -c "
import json;d=json.loads(open('gpurun_out/tab.json').read().strip().splitlines()[-1]);print('small_off', '$v', round(d['ms_per_step'],4), round(d['run_stats']['library_ms_per_run'],4), all(v for k,v in d['parity'].items()))"
done
unset USAC_INLIERS_SMALL
FUSED=0 bash tools/gpu_pf_prof.sh > /dev/null
bash tools/gpu_phase_detail.sh | head -1
