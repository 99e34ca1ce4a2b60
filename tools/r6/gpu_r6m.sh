#!/bin/bash
# A/B of the h16 append path: HEAD's vs the working tree's, interleaved cfg2 bench lines
set -o pipefail
O=gpurun_out/r6m; mkdir -p $O
for r in 1 2; do for v in h16head cur; do
RANSAC_AMD_LIB=ransac_amd/var_libs/lib_$v.so timeout -k 10 200 python -u bench.py --steps 40 --warmup 5 --cpu-seconds 0 > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { echo "bench $v failed"; tail $O/b_${v}_$r.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b_${v}_$r.json'));print('$v', d['value']/1e6, d['ms_per_step'], d['roofline']['kernel_ms'])"
done; done
