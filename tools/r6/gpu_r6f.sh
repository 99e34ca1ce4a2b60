#!/bin/bash
set -o pipefail
O=gpurun_out/r6f; mkdir -p $O
for P in 3 6 10; do
timeout -k 10 200 python -u bench.py --estimator essential --steps 10 --warmup 3 --cpu-seconds 0 --pipeline $P > $O/bench_e_p$P.json 2> $O/bench_e_p$P.err; echo "pipeline $P rc=$?"; python3 -c "import json;d=json.load(open('$O/bench_e_p$P.json'));print(d['value']/1e6, d['ms_per_step'])"
done
for flag in 0 1; do
USAC_E16=$flag timeout -k 10 200 python -u bench.py --estimator essential --steps 10 --warmup 3 --cpu-seconds 0 --pipeline 6 > $O/bench_e16_$flag.json 2> $O/bench_e16_$flag.err; echo "e16=$flag rc=$?"; python3 -c "import json;d=json.load(open('$O/bench_e16_$flag.json'));print(d['value']/1e6, d['ms_per_step'])"
done
