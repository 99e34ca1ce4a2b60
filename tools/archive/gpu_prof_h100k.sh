set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=r5g WORKLOADS="h100k" bash tools/profile_round.sh > gpurun_out/prof_h100k.log 2>&1 || { tail -20 gpurun_out/prof_h100k.log; exit 1; }
tail -3 gpurun_out/prof_h100k.log
cp gpurun_out/prof_r5g/summaries/r5g_h100k_summary.json profiles/ && timeout -k 10 300 python bench.py --cfg5 --cpu-seconds 0 > gpurun_out/cfg5_roof.json 2>/dev/null
python3 -c "
import json;d=json.loads(open('gpurun_out/cfg5_roof.json').read().strip().splitlines()[-1]);r=d['roofline'];print(d['ms_per_step'], r.get('frac'), r.get('source'), r.get('kernel_ms'), r.get('mfma',{}).get('frac'), r.get('hbm',{}).get('frac'))"
