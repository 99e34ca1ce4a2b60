set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
true
true
for rep in 1 2 3 4; do
  for v in 0 1; do
    USAC_COMPACT_PSUM=$v timeout -k 10 300 python bench.py --cfg5 --steps 30 --cpu-seconds 0 > gpurun_out/cpab.json 2>/dev/null || exit 1
    python3 -c "
import json;d=json.loads(open('gpurun_out/cpab.json').read().strip().splitlines()[-1]);print('compact_psum $v cfg5', round(d['ms_per_step'],4), all(d['parity'].values()))"
  done
done
