set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
for rep in 1 2 3; do
  for lib in ransac_amd/var_libs/lib_base.so ransac_amd/libransac_amd.so; do
    RANSAC_AMD_LIB=$PWD/$lib timeout -k 10 300 python bench.py --sprt-exact --steps 40 --cpu-seconds 0 > gpurun_out/rw.json 2>/dev/null || exit 1
    LIB=$lib python3 -c "
import json, os;d=json.loads(open('gpurun_out/rw.json').read().strip().splitlines()[-1]);print(os.environ['LIB'], round(d['ms_per_step'],4), d['run_stats'], all(d['parity'].values()))"
  done
done
