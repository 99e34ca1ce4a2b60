#!/bin/bash
# cfg3 batch SPRT: cost of the no-packed-fp32 rule (diagnostic packed build, same box)
set -o pipefail
O=gpurun_out/r6bb; mkdir -p $O
for r in 1 2; do for v in cur packed; do
RANSAC_AMD_LIB=ransac_amd/var_libs/lib_$v.so timeout -k 10 200 python -u bench.py --estimator fundamental --steps 20 --warmup 5 --cpu-seconds 0 > $O/f_${v}_$r.json 2> $O/f_${v}_$r.err || { echo "bench failed"; tail -5 $O/f_${v}_$r.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/f_${v}_$r.json'));r=d['roofline'];print('$v', round(d['value']/1e6,1), round(d['ms_per_step'],4), r.get('score_kernel_ms'), r.get('solve_kernel_ms'), d.get('parity',{}).get('ok'))"
done; done
