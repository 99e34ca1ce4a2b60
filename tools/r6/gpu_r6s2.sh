#!/bin/bash
# cfg5 kernel trace of the current build (per-kernel averages after the link staging fix)
set -o pipefail
O=gpurun_out/r6s2; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof -o run --output-format csv -- python3 bench.py --cfg5 > $O/prof.json 2> $O/prof.err || { echo "prof failed"; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats_cfg5.csv
python3 - <<PY
import csv,json
d=json.load(open('$O/prof.json')); runs=d['config'].get('runs') or 1
print('ms', d['ms_per_step'], 'runs', runs)
rows=list(csv.DictReader(open('$O/kernel_stats_cfg5.csv')))
for r in sorted(rows, key=lambda r:-float(r['TotalDurationNs']))[:24]: print(r['Name'][:48], r['Calls'], round(float(r['AverageNs'])/1e3,2), round(float(r['TotalDurationNs'])/1e3,1))
PY
