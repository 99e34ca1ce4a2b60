set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
for rep in 1 2 3; do
  for g in 4 2 1; do
    USAC_POLISH_GROUP=$g timeout -k 10 300 python bench.py --sprt-exact --steps 60 --cpu-seconds 0 > gpurun_out/pg.json 2>/dev/null || exit 1
    G=$g python3 -c "
import json, os;d=json.loads(open('gpurun_out/pg.json').read().strip().splitlines()[-1]);print('group', os.environ['G'], round(d['ms_per_step'],4), d['run_stats']['library_ms_per_run'], all(d['parity'].values()))"
  done
done
