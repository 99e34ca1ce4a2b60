#!/bin/bash
# per-file vectoriser flags ("mix": kernels_fund.hip vectorised, packed-fp32-ops off everywhere) vs all off ("cur")
set -o pipefail
O=gpurun_out/r6dd; mkdir -p $O
run() {  # name, env..., -- bench args
  local n=$1; shift
  env "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -5 $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n', round(d['value']/1e6,3), round(d['ms_per_step'],4), d.get('parity',{}).get('ok'))"
}
for r in 1 2; do for v in cur mix; do
L=RANSAC_AMD_LIB=ransac_amd/var_libs/lib_$v.so
run f_${v}_$r $L timeout -k 10 200 python -u bench.py --estimator fundamental --steps 20 --warmup 5 --cpu-seconds 0
run h_${v}_$r $L timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 0
run e_${v}_$r $L timeout -k 10 200 python -u bench.py --estimator essential --steps 20 --warmup 5 --cpu-seconds 0
done; done
