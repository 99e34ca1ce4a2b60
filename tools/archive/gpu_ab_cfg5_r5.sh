set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
for v in "USAC_X=0" "USAC_H16=0" "USAC_X=0" "USAC_H16=0"; do
  env $v timeout -k 10 300 python bench.py --cfg5 --cpu-seconds 0 > gpurun_out/c5.json 2> gpurun_out/c5.err || { tail -5 gpurun_out/c5.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c5.json').read().strip().splitlines()[-1]); print('$v', 'ms/run %.3f' % d['ms_per_step'], d['parity'].get('model_bit_equal'))"
done
