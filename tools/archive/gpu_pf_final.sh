set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/gpu_polish_fused.sh
FUSED=1 bash tools/gpu_pf_prof.sh | tail -2
for f in 0 1 0 1; do
USAC_POLISH_FUSED=$f timeout -k 10 300 python bench.py --sprt-exact --steps 40 --warmup 5 --cpu-seconds 0 > gpurun_out/pfab.json 2>/dev/null || exit 1
python3 -c "
import json;d=json.loads(open('gpurun_out/pfab.json').read().strip().splitlines()[-1]);print('fused', '$f', round(d['ms_per_step'],4), round(d['run_stats']['library_ms_per_run'],4), all(v for k,v in d['parity'].items()))"
done
