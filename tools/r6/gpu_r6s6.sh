#!/bin/bash
# cfg5 line forms on one box: the default command (100 timed runs after 10 warm-up runs) and the
# 20 / 2 form of the round's earlier tables, interleaved twice
set -o pipefail
O=gpurun_out/r6s6; mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --cfg5 --cpu-seconds 0 > $O/cfg5_default_$r.json 2> $O/cfg5_default_$r.err || { echo "cfg5 default failed"; exit 1; }
  timeout -k 10 200 python -u bench.py --cfg5 --steps 20 --warmup 2 --cpu-seconds 0 > $O/cfg5_s20_$r.json 2> $O/cfg5_s20_$r.err || { echo "cfg5 s20 failed"; exit 1; }
  timeout -k 10 200 python -u bench.py --cfg5 --steps 20 --warmup 10 --cpu-seconds 0 > $O/cfg5_s20w10_$r.json 2> $O/cfg5_s20w10_$r.err || { echo "cfg5 s20w10 failed"; exit 1; }
  for v in default s20 s20w10; do python3 -c "import json;d=json.load(open('$O/cfg5_${v}_$r.json'));print('$v', d['steps'], d['warmup'], d['ms_per_step'], all(d['parity'].values()))"; done
done
