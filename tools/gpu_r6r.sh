#!/bin/bash
# same-box A/B: the r6o build (e16 stacks, before the CU-mask option) vs the current build, cfg4
set -o pipefail
O=gpurun_out/r6r; mkdir -p $O
for r in 1 2; do for v in e16stack cur; do
RANSAC_AMD_LIB=ransac_amd/var_libs/lib_$v.so timeout -k 10 200 python -u bench.py --estimator essential --steps 20 --warmup 5 --cpu-seconds 0 > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { echo "bench failed"; tail -5 $O/b_${v}_$r.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b_${v}_$r.json'));print('$v', round(d['value']/1e6,2), round(d['ms_per_step'],4), d.get('parity',{}).get('ok'))"
done; done
