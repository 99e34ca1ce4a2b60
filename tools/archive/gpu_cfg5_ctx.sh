set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
for rep in 1 2; do
  USAC_PROFILE=1 timeout -k 10 300 python bench.py --cfg5 --cpu-seconds 0 > gpurun_out/c5.json 2> gpurun_out/c5.err || { tail -5 gpurun_out/c5.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/c5.json').read().strip().splitlines()[-1]);print('cfg5', round(d['ms_per_step'],4), all(d['parity'].values()), d['roofline'].get('frac'))"
  grep "usac_ransac_run ms" gpurun_out/c5.err | tail -2 | cut -c1-200
done
