set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_polish_fused.py > gpurun_out/pf.log 2>&1 || { tail -40 gpurun_out/pf.log; exit 1; }
grep -E "passed|failed" gpurun_out/pf.log | tail -2
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_loop.py tests/test_gpu_baseline_sizes.py tests/test_gpu_essential.py tests/test_gpu_napsac_lo.py tests/test_gpu_graphcut.py > gpurun_out/pf2.log 2>&1 || { tail -40 gpurun_out/pf2.log; exit 1; }
tail -1 gpurun_out/pf2.log
bash tools/gpu_phase_detail.sh | head -1
python3 -c "
import json;d=json.loads(open('gpurun_out/px.json').read().strip().splitlines()[-1]);print(d['ms_per_step'],d['run_stats'],all(v for k,v in d['parity'].items()))"
