#!/bin/bash
set -o pipefail
O=gpurun_out/r6j; mkdir -p $O
for b in 128 320; do USAC_E5_BUDGET=$b timeout -k 10 200 python -u bench.py --estimator essential --steps 10 --warmup 3 --cpu-seconds 0 > $O/bench_b$b.json 2> $O/bench_b$b.err; echo "budget $b rc=$?"; python3 -c "import json;d=json.load(open('$O/bench_b$b.json'));print(d['value']/1e6, d['ms_per_step'])"; done
USAC_E16=1 timeout -k 10 200 python -u bench.py --estimator essential --steps 10 --warmup 3 --cpu-seconds 0 > $O/bench_e16.json 2> $O/bench_e16.err; echo "e16 rc=$?"; python3 -c "import json;d=json.load(open('$O/bench_e16.json'));print(d['value']/1e6, d['ms_per_step'])"
