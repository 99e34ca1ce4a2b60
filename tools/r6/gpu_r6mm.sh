#!/bin/bash
# cfg2 batches in flight (3 default) and hardware queues, after the host-path trims
set -o pipefail
O=gpurun_out/r6mm; mkdir -p $O
run() {  # name, env..., -- bench args
  local n=$1; shift
  env "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -5 $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n', round(d['value']/1e6,1), round(d['ms_per_step'],4), d['parity']['ok'])"
}
B="timeout -k 10 200 python -u bench.py --steps 40 --warmup 5 --cpu-seconds 0"
for r in 1 2; do
run p3_$r $B
run p4_$r $B --pipeline 4
run p4q8_$r GPU_MAX_HW_QUEUES=8 $B --pipeline 4
run p2_$r $B --pipeline 2
done
cat /proc/loadavg
