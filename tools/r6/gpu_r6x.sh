#!/bin/bash
# cfg5 per-run phase split (USAC_PROFILE) and cfg3-exact split
set -o pipefail
O=gpurun_out/r6x; mkdir -p $O
USAC_PROFILE=1 timeout -k 10 300 python -u bench.py --cfg5 --steps 10 --warmup 2 --cpu-seconds 0 > $O/cfg5.json 2> $O/cfg5.err || { echo "cfg5 failed"; tail -5 $O/cfg5.err; exit 1; }
grep "usac_ransac_run ms" $O/cfg5.err | tail -6
python3 -c "import json;d=json.load(open('$O/cfg5.json'));print('cfg5', d['ms_per_step'], d['run_stats'])"
