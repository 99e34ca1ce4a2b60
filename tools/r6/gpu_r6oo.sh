#!/bin/bash
# e16 drain-round threshold: 48 lanes (cur) vs 32 / 56
set -o pipefail
O=gpurun_out/r6oo; mkdir -p $O
for v in cur r32 r56; do
RANSAC_AMD_LIB=ransac_amd/var_libs/lib_$v.so timeout -k 10 100 python -u tools/e_phase.py > $O/phase_$v.log 2>&1 || { echo "phase failed"; exit 1; }
echo $v; head -1 $O/phase_$v.log
done
for r in 1 2; do for v in cur r32 r56; do
RANSAC_AMD_LIB=ransac_amd/var_libs/lib_$v.so timeout -k 10 200 python -u bench.py --estimator essential --steps 30 --warmup 5 --cpu-seconds 0 > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { echo "bench failed"; tail -5 $O/b_${v}_$r.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b_${v}_$r.json'));print('$v', round(d['value']/1e6,2), round(d['ms_per_step'],4), d.get('parity',{}).get('ok'))"
done; done
