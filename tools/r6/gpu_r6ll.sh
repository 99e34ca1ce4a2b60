#!/bin/bash
# k_solve_h4 capped at 256 registers (2 waves/SIMD, 104 B spill) vs 282 (1 wave): cfg2 lines, same box
set -o pipefail
O=gpurun_out/r6ll; mkdir -p $O
for r in 1 2 3; do for v in cur h4w2; do
RANSAC_AMD_LIB=ransac_amd/var_libs/lib_$v.so timeout -k 10 200 python -u bench.py --steps 40 --warmup 5 --cpu-seconds 0 > $O/h_${v}_$r.json 2> $O/h_${v}_$r.err || { echo "bench failed"; tail -5 $O/h_${v}_$r.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/h_${v}_$r.json'));r=d['roofline'];print('$v', round(d['value']/1e6,1), round(d['ms_per_step'],4), r.get('solve_kernel_ms'), r.get('solve_kernel_ms_in_pipeline'), d['parity']['ok'])"
done; done
