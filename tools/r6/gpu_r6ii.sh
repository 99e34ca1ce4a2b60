#!/bin/bash
# bench: timing events on the first context only + Python record order (this tree) vs timings every fourth batch (bench_prev.py)
set -o pipefail
O=gpurun_out/r6ii; mkdir -p $O
for r in 1 2 3; do for v in prev cur; do
B=bench.py; [ $v = prev ] && B=tools/bench_prev.py
timeout -k 10 200 python -u $B --steps 40 --warmup 5 --cpu-seconds 0 > $O/h_${v}_$r.json 2> $O/h_${v}_$r.err || { echo "bench failed"; tail -5 $O/h_${v}_$r.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/h_${v}_$r.json'));r=d['roofline'];print('$v', round(d['value']/1e6,1), round(d['ms_per_step'],4), r.get('kernel_ms_in_pipeline'))"
done; done
cat /proc/loadavg
