#!/bin/bash
# round-6 head after the seqsum load fixes: each config default bench line and rocprof stats of
# cfg2 / cfg4 / cfg5 (the GPU suite and smoke at the same build: tools/r6/gpu_r6s5.sh)
set -o pipefail
O=gpurun_out/r6final3; mkdir -p $O
export TMPDIR=/tmp
line() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -5 $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));r=d['roofline'];print('$n', d['value'], d['ms_per_step'], r.get('kernel'), r.get('frac'), d.get('cpu_baseline',{}).get('value'), d.get('parity',{}).get('ok', d.get('parity')))"
}
line cfg2 --steps 20 --warmup 5
line cfg3 --estimator fundamental --steps 20 --warmup 5
line cfg3x --sprt-exact --steps 20 --warmup 3
line cfg4 --estimator essential --steps 20 --warmup 5
line cfg5 --cfg5 --steps 20 --warmup 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof_cfg2 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $O/prof_cfg2.json 2> $O/prof_cfg2.err || { echo "prof cfg2 failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof_cfg4 -o run --output-format csv -- python3 bench.py --estimator essential --steps 20 --warmup 5 --cpu-seconds 0 > $O/prof_cfg4.json 2> $O/prof_cfg4.err || { echo "prof cfg4 failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof_cfg5 -o run --output-format csv -- python3 bench.py --cfg5 --steps 20 --warmup 2 --cpu-seconds 0 > $O/prof_cfg5.json 2> $O/prof_cfg5.err || { echo "prof cfg5 failed"; exit 1; }
echo done
