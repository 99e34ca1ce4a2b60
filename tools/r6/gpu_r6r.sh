#!/bin/bash
# same-box A/B: the r6o build (e16 stacks, before the CU-mask option) vs the current build, cfg4
set -o pipefail
O=gpurun_out/r6r; mkdir -p $O
for r in 1 2; do for v in e16stack cur; do
RANSAC_AMD_LIB=ransac_amd/var_libs/lib_$v.so timeout -k 10 200 python -u bench.py --estimator essential --steps 20 --warmup 5 --cpu-seconds 0 > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { echo "bench failed"; tail -5 $O/b_${v}_$r.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b_${v}_$r.json'));print('$v', round(d['value']/1e6,2), round(d['ms_per_step'],4), d.get('parity',{}).get('ok'))"
done; done
timeout -k 10 200 python -u bench.py --sprt-exact --steps 20 --warmup 3 --cpu-seconds 0 > $O/cfg3x.json 2> $O/cfg3x.err || { echo "cfg3x failed"; tail -5 $O/cfg3x.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/cfg3x.json'));print('cfg3x', d['ms_per_step'], d['parity'])"
USAC_PROFILE=1 timeout -k 10 200 python -u bench.py --sprt-exact --steps 10 --warmup 2 --cpu-seconds 0 > $O/cfg3x_prof.json 2> $O/cfg3x_prof.err || { echo "cfg3x prof failed"; exit 1; }
grep "usac_ransac_run ms" $O/cfg3x_prof.err | tail -4
timeout -k 10 300 python -u bench.py --cfg5 --steps 20 --warmup 2 --cpu-seconds 0 > $O/cfg5.json 2> $O/cfg5.err || { echo "cfg5 failed"; tail -5 $O/cfg5.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/cfg5.json'));print('cfg5', d['ms_per_step'], d['parity'], d['roofline'].get('kernel'), d['roofline'].get('frac'))"
